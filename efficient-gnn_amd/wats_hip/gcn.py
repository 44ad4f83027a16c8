"""Sparse propagation for the base model WATS wraps.

The reference base model ``CompatibleGCN`` (``src/gnn/model.py:7-53``) builds
``adj_norm = adj / deg`` with ``deg = adj.sum(dim=1)``, ``deg[deg == 0] = 1``
(``model.py:43-45``) and propagates twice with a dense ``torch.mm(adj_norm,
x)`` (``model.py:47,51``).  That is an O(N^2) dense product per call, paid
every epoch of ``WATS.calib_train`` (``calibration/WATS.py:149`` ->
``WATS.forward`` -> ``base_model(x, adj)``, ``WATS.py:128``).

Here ``adj_norm`` becomes a CSR operator on the HIP library's step kernel
(``wg_rownorm_create`` / ``wg_spmm``, ``csrc/gcn.hip``): y = adj_norm @ x with
float64 row sums.  :class:`RowNormalizedAdjacency` holds the operator and its
transpose; :func:`propagate` is differentiable w.r.t. ``x`` (backward:
``adj_norm^T @ grad``).  :class:`SparseCompatibleGCN` is ``CompatibleGCN`` with
that propagation.  It has the same constructor, parameter names
(``gc1``/``gc2``) and state dict, so weights move between the two.  It does not
support a gradient w.r.t. ``adj``, which the calibration attacks take
(``calib_attack/calib_fga.py:864-868``); it raises there, and the dense
reference model is the one to use for attacks.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from ._lib import check, ptr
from .laplacian import dense_to_csr, require_gpu, stream_handle


class _Op:
    """One wg handle (adj_norm or its transpose), destroyed with the object."""

    def __init__(self, n, indptr, indices, values, transpose: bool, reorder: bool, device):
        lib = _lib.load()
        h = ctypes.c_void_p()
        flags = (_lib.WG_FLAG_TRANSPOSE if transpose else 0) | (0 if reorder else _lib.WG_FLAG_NO_REORDER)
        nnz = int(indices.numel())
        with torch.cuda.device(device):
            check(lib.wg_rownorm_create(n, nnz, ptr(indptr), ptr(indices) if nnz else None,
                                        ptr(values) if (nnz and values is not None) else None, flags,
                                        stream_handle(device), ctypes.byref(h)), "rownorm_create")
        self.h = h
        self.n = n
        self.device = device

    def apply(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.device, torch.float32).contiguous()
        if x.dim() != 2 or x.shape[0] != self.n:
            raise ValueError(f"expected ({self.n}, F) features, got {tuple(x.shape)}")
        y = torch.empty_like(x)
        if x.shape[1] == 0 or self.n == 0:
            return y
        with torch.cuda.device(self.device):
            check(_lib.load().wg_spmm(self.h, x.shape[1], ptr(x), ptr(y), stream_handle(self.device)), "spmm")
        return y

    def __del__(self):
        h = getattr(self, "h", None)
        try:
            if h is not None and _lib._lib is not None:
                _lib._lib.wg_laplacian_destroy(h)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass
        self.h = None


class RowNormalizedAdjacency:
    """``adj_norm = adj / deg`` of ``CompatibleGCN.forward`` (model.py:43-45)
    as a device CSR operator plus its transpose."""

    def __init__(self, n: int, indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor | None = None,
                 reorder: bool = True, device=None):
        device = require_gpu(device if device is not None else (indptr.device if indptr.is_cuda else None))
        self.device = device
        indptr = indptr.to(device=device, dtype=torch.int64).contiguous()
        indices = indices.to(device=device, dtype=torch.int32).contiguous()
        if values is not None:
            values = values.to(device=device, dtype=torch.float32).contiguous()
        if indptr.numel() != n + 1:
            raise ValueError("indptr must have n + 1 entries")
        self.n = int(n)
        self.nnz = int(indices.numel())
        self.fwd = _Op(self.n, indptr, indices, values, False, reorder, device)
        self.bwd = _Op(self.n, indptr, indices, values, True, reorder, device)

    @classmethod
    def from_dense(cls, adj: torch.Tensor, **kw):
        """From the dense (N, N) adjacency the reference model receives
        (on-device compaction, entries != 0 kept)."""
        if adj.dim() != 2 or adj.shape[0] != adj.shape[1]:
            raise ValueError("adjacency must be square")
        indptr, indices, values = dense_to_csr(adj)
        return cls(adj.shape[0], indptr, indices, values, device=indptr.device, **kw)

    @classmethod
    def from_scipy(cls, A, **kw):
        import numpy as np
        import scipy.sparse as sp
        A = sp.csr_matrix(A)
        return cls(A.shape[0], torch.from_numpy(A.indptr.astype(np.int64)),
                   torch.from_numpy(A.indices.astype(np.int32)), torch.from_numpy(A.data.astype(np.float32)), **kw)

    def __matmul__(self, x: torch.Tensor) -> torch.Tensor:
        return propagate(self, x)


class _Propagate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, op):
        ctx.op = op
        return op.fwd.apply(x)

    @staticmethod
    def backward(ctx, g):
        return ctx.op.bwd.apply(g), None


def propagate(op: RowNormalizedAdjacency, x: torch.Tensor) -> torch.Tensor:
    """``adj_norm @ x`` (model.py:47, 51), differentiable w.r.t. ``x``."""
    return _Propagate.apply(x, op)


class SparseCompatibleGCN(nn.Module):
    """``CompatibleGCN`` (reference ``src/gnn/model.py:7-53``) with the two
    propagations on the HIP SpMM.  Same constructor, parameters and state dict.

    ``forward(x, adj)`` accepts the dense adjacency the reference takes (the
    CSR operator is built once and cached while ``adj`` is unchanged) or a
    :class:`RowNormalizedAdjacency`."""

    DATASET_CLASSES = {
        'cora': 7, 'citeseer': 6, 'pubmed': 3, 'reddit': 41, 'amazon-computers': 10, 'amazon-photo': 8,
        'coauthor-cs': 15, 'coauthor-physics': 5, 'dblp': 4, 'ogbn-arxiv': 40,
    }

    def __init__(self, nfeat: int, dataset_name: str = None, nclass: int = None, nhid: int = 64,
                 dropout: float = 0.5):
        super().__init__()
        if dataset_name and dataset_name.lower() in self.DATASET_CLASSES:
            nclass = self.DATASET_CLASSES[dataset_name.lower()]
        elif nclass is None:
            raise ValueError("Either dataset_name or nclass must be provided")
        self.gc1 = nn.Linear(nfeat, nhid)
        self.gc2 = nn.Linear(nhid, nclass)
        self.dropout = nn.Dropout(dropout)
        self._op_key = None
        self._op = None

    def operator(self, adj) -> RowNormalizedAdjacency:
        if isinstance(adj, RowNormalizedAdjacency):
            return adj
        if adj.requires_grad:
            raise NotImplementedError("SparseCompatibleGCN has no gradient w.r.t. adj; use the dense "
                                      "CompatibleGCN for attacks that differentiate through the adjacency")
        key = (adj.data_ptr(), tuple(adj.shape), adj._version, str(adj.device))
        if self._op is None or self._op_key != key:
            device = next(self.parameters()).device
            self._op = RowNormalizedAdjacency.from_dense(adj.to(device))
            self._op_key = key
        return self._op

    def forward(self, x: torch.Tensor, adj) -> torch.Tensor:
        device = next(self.parameters()).device
        x = x.to(device)
        op = self.operator(adj)
        x = propagate(op, x)                # model.py:47
        x = F.relu(self.gc1(x))             # model.py:48
        x = self.dropout(x)                 # model.py:49
        x = propagate(op, x)                # model.py:51
        return self.gc2(x)                  # model.py:52
