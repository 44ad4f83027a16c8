"""Device-resident rescaled normalised Laplacian ``L_hat`` (a1 + a2).

Mirrors ``compute_normalized_laplacian`` (reference ``calibration/WATS.py:24-27``,
i.e. ``scipy.sparse.csgraph.laplacian(adj, normed=True)``, scipy
``_laplacian.py:467-475``) followed by the rescale ``(2/2.0)*L - identity(N)``
(``calibration/WATS.py:55``).  The operator lives on the GPU as a handle of the
HIP library; nothing is copied back to the host.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import LaplacianInfo, check, ptr


def require_gpu(device=None) -> torch.device:
    """The product path runs on a ROCm GPU only -- fail loudly otherwise."""
    if not torch.cuda.is_available():
        raise RuntimeError("wats_hip: no ROCm GPU visible (torch.cuda.is_available() is False); "
                           "the graph-wavelet path has no CPU fallback")
    _lib.load()
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError(f"wats_hip: device {device} is not a GPU")
    return device


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def dense_to_csr(adj: torch.Tensor):
    """On-device replacement of ``csr_matrix(adj.cpu().numpy())``
    (``calibration/WATS.py:99``): returns (indptr int64, indices int32,
    values float32) device tensors; keeps entries != 0 in column order."""
    if adj.dim() != 2:
        raise ValueError("adj must be 2-D")
    device = require_gpu(adj.device if adj.is_cuda else None)
    a = adj.detach().to(device=device, dtype=torch.float32)
    if a.stride(1) != 1:
        a = a.contiguous()
    n_rows, n_cols = a.shape
    lib = _lib.load()
    indptr = torch.empty(n_rows + 1, dtype=torch.int64, device=device)
    nnz = ctypes.c_int64(0)
    with torch.cuda.device(device):
        st = stream_handle(device)
        check(lib.wg_dense_to_csr_count(ptr(a), n_rows, n_cols, a.stride(0), ptr(indptr), ctypes.byref(nnz), st),
              "dense_to_csr_count")
        indices = torch.empty(max(nnz.value, 1), dtype=torch.int32, device=device)[: nnz.value]
        values = torch.empty(max(nnz.value, 1), dtype=torch.float32, device=device)[: nnz.value]
        check(lib.wg_dense_to_csr_fill(ptr(a), n_rows, n_cols, a.stride(0), ptr(indptr), ptr(indices),
                                       ptr(values), st), "dense_to_csr_fill")
    return indptr, indices, values


class NormalizedLaplacian:
    """``L_hat = L_sym - I`` of a graph, materialised on one GPU.

    Build with :meth:`from_csr`, :meth:`from_dense`, :meth:`from_scipy` or
    :func:`compute_normalized_laplacian`.  For a row shard (multi-GPU) the
    columns are ``[owned rows | halo rows]`` and ``w_cols`` carries the global
    column degrees (see ``wats_hip.dist``).  ``sort_columns=False`` keeps
    each row's entries in the caller's order (``WG_FLAG_KEEP_COLUMN_ORDER``)
    instead of sorting them by internal column, which the gather kernels prefer.
    """

    def __init__(self, n_rows: int, indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor | None = None,
                 n_cols: int | None = None, w_cols: torch.Tensor | None = None, reorder: bool = True,
                 sort_columns: bool = True, device=None):
        device = require_gpu(device if device is not None else (indptr.device if indptr.is_cuda else None))
        self.device = device
        n_cols = n_rows if n_cols is None else int(n_cols)
        indptr = indptr.to(device=device, dtype=torch.int64).contiguous()
        indices = indices.to(device=device, dtype=torch.int32).contiguous()
        if values is not None:
            values = values.to(device=device, dtype=torch.float32).contiguous()
        if w_cols is not None:
            w_cols = w_cols.to(device=device, dtype=torch.float32).contiguous()
            if w_cols.numel() != n_cols:
                raise ValueError("w_cols must have n_cols entries")
        if indptr.numel() != n_rows + 1:
            raise ValueError("indptr must have n_rows + 1 entries")
        nnz = int(indices.numel())
        lib = _lib.load()
        handle = ctypes.c_void_p()
        flags = _lib.WG_FLAG_NONE if reorder else _lib.WG_FLAG_NO_REORDER
        if not sort_columns:
            flags |= _lib.WG_FLAG_KEEP_COLUMN_ORDER
        with torch.cuda.device(device):
            check(lib.wg_laplacian_create(n_rows, n_cols, nnz, ptr(indptr), ptr(indices) if nnz else None,
                                          ptr(values) if nnz else None, ptr(w_cols), flags,
                                          stream_handle(device), ctypes.byref(handle)), "laplacian_create")
        self._h = handle
        info = LaplacianInfo()
        check(lib.wg_laplacian_get_info(self._h, ctypes.byref(info)), "laplacian_get_info")
        self.info = info.as_dict()
        self.n = int(n_rows)
        self.n_cols = n_cols
        self.is_literal = False

    # ------------------------------------------------------------------ builders
    @classmethod
    def literal(cls, indptr, indices, values, n: int, reorder: bool = True, sort_columns: bool = True, device=None):
        """A LITERAL operator: every stored entry applied with its value
        (float32), diagonal included, nothing normalised (``wg_operator_create``).
        What :func:`chebyshev_polynomials` applies to an explicit matrix, e.g.
        the reference's ``L_rescaled`` (calibration/WATS.py:55,62)."""
        to_t = lambda a, dt: a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a, dtype=dt))
        device = require_gpu(device)
        indptr = to_t(indptr, np.int64).to(device=device, dtype=torch.int64).contiguous()
        indices = to_t(indices, np.int32).to(device=device, dtype=torch.int32).contiguous()
        values = to_t(values, np.float32).to(device=device, dtype=torch.float32).contiguous()
        if indptr.numel() != n + 1:
            raise ValueError("indptr must have n + 1 entries")
        nnz = int(indices.numel())
        flags = _lib.WG_FLAG_NONE if reorder else _lib.WG_FLAG_NO_REORDER
        if not sort_columns:
            flags |= _lib.WG_FLAG_KEEP_COLUMN_ORDER
        handle = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(_lib.load().wg_operator_create(n, nnz, ptr(indptr), ptr(indices) if nnz else None,
                                                 ptr(values) if nnz else None, flags, stream_handle(device),
                                                 ctypes.byref(handle)), "operator_create")
        self = cls.__new__(cls)
        self.device = device
        self._h = handle
        info = LaplacianInfo()
        check(_lib.load().wg_laplacian_get_info(self._h, ctypes.byref(info)), "laplacian_get_info")
        self.info = info.as_dict()
        self.n = int(n)
        self.n_cols = int(n)
        self.is_literal = True
        return self

    @classmethod
    def from_csr(cls, indptr, indices, values=None, n: int | None = None, **kw):
        if n is None:
            n = int(len(indptr) - 1)
        to_t = lambda a, dt: a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a, dtype=dt))
        return cls(n, to_t(indptr, np.int64), to_t(indices, np.int32),
                   None if values is None else to_t(values, np.float32), **kw)

    @classmethod
    def from_scipy(cls, A, **kw):
        import scipy.sparse as sp
        A = sp.csr_matrix(A)
        if A.shape[0] != A.shape[1]:
            raise ValueError("adjacency must be square")
        if not A.has_canonical_format:
            A = A.copy()
            A.sum_duplicates()
        return cls.from_csr(A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.astype(np.float32),
                            n=A.shape[0], **kw)

    @classmethod
    def from_dense(cls, adj: torch.Tensor, **kw):
        if adj.shape[0] != adj.shape[1]:
            raise ValueError("adjacency must be square")
        indptr, indices, values = dense_to_csr(adj)
        return cls(adj.shape[0], indptr, indices, values, device=indptr.device, **kw)

    @classmethod
    def from_graph(cls, g, **kw):
        """From a ``wats_hip.graphgen.CSRGraph``."""
        return cls.from_csr(g.indptr, g.indices, g.values, n=g.n, **kw)

    # ------------------------------------------------------------------ API
    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("NormalizedLaplacian has been closed")
        return self._h

    @property
    def nnz(self) -> int:
        return int(self.info["nnz"])

    def log1p_degree(self) -> torch.Tensor:
        """``X0 = log1p(rowsum(A))`` as (N, 1) float32 (calibration/WATS.py:58-59)."""
        x0 = torch.empty(self.n, 1, dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            check(_lib.load().wg_log1p_degree(self.handle, ptr(x0), stream_handle(self.device)), "log1p_degree")
        return x0

    def export(self):
        """L_hat in caller numbering -> (indptr, indices, values, iso) CPU numpy
        (off-diagonal entries; iso marks L_hat_ii = -1)."""
        n = self.n
        indptr = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        nnz = self.nnz
        indices = torch.empty(max(nnz, 1), dtype=torch.int32, device=self.device)
        values = torch.empty(max(nnz, 1), dtype=torch.float32, device=self.device)
        iso = torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            check(_lib.load().wg_laplacian_export(self.handle, ptr(indptr), ptr(indices), ptr(values), ptr(iso),
                                                  stream_handle(self.device)), "laplacian_export")
        torch.cuda.synchronize(self.device)
        return (indptr.cpu().numpy(), indices[:nnz].cpu().numpy(), values[:nnz].cpu().numpy(),
                iso[:n].cpu().numpy().astype(bool))

    def to_scipy(self):
        """Dense-equivalent scipy CSR of L_hat (float64, diagonal -1 on isolated
        rows) in caller numbering -- for parity checks only."""
        import scipy.sparse as sp
        indptr, indices, values, iso = self.export()
        off = sp.csr_matrix((values.astype(np.float64), indices, indptr), shape=(self.n, self.n_cols))
        return (off - sp.diags(iso.astype(np.float64), shape=(self.n, self.n_cols))).tocsr()

    def permute(self, x: torch.Tensor, to_internal: bool) -> torch.Tensor:
        """Rows caller order <-> internal (degree-relabelled) order."""
        x = x.contiguous()
        F = x.shape[1]
        out = torch.empty_like(x)
        with torch.cuda.device(self.device):
            check(_lib.load().wg_permute_rows(self.handle, 0 if to_internal else 1, F, ptr(x), ptr(out),
                                              stream_handle(self.device)), "permute_rows")
        return out

    def step(self, k: int, t_km1: torch.Tensor, t_km2: torch.Tensor | None, out: torch.Tensor | None,
             S: torch.Tensor | None = None, H: torch.Tensor | None = None, alpha0: float = 1.0,
             alpha_k: float = 0.0) -> None:
        """One fused Chebyshev step in INTERNAL order (see wg_cheb_step)."""
        F = t_km1.shape[1]
        with torch.cuda.device(self.device):
            check(_lib.load().wg_cheb_step(self.handle, int(k), F, ptr(t_km1), ptr(t_km2), ptr(out), ptr(S), ptr(H),
                                           float(alpha0), float(alpha_k), stream_handle(self.device)), "cheb_step")

    def tune(self, **knobs) -> None:
        """Step-kernel tuning knobs: iter, chunk_iter, tiles, ... (wg_laplacian_tune in wats_hip.h)."""
        for k, v in knobs.items():
            check(_lib.load().wg_laplacian_tune(self.handle, k.encode(), int(v)), f"tune {k}")

    def lds_plan_info(self, active_only: bool = True) -> dict | None:
        """Shape of the F == 1 LDS kernel's plan (None when it does not apply)."""
        out = (ctypes.c_int64 * 8)()
        with torch.cuda.device(self.device):
            check(_lib.load().wg_lds_plan_info(self.handle, 1 if active_only else 0, out), "lds_plan_info")
        if out[0] == 0:
            return None
        keys = ("mode", "blocks", "rows", "cols", "nnz", "segments", "chunks", "workgroups")
        return dict(zip(keys, [int(v) for v in out]))

    def describe(self, F: int = 1) -> str:
        """The step kernel's launch plan for an F-column signal."""
        return _lib.load().wg_laplacian_describe(self.handle, int(F)).decode()

    def chain_status(self) -> bool:
        """True if the handle's last one-launch chain (csrc/chain.hip) gave up a
        wait (its results are NaN) and no call has reported it yet.  Waits for
        that launch only (an event, not a device sync).  A timeout switches the
        handle to the multi-launch path until the next tune()."""
        out = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            check(_lib.load().wg_chain_status(self.handle, ctypes.byref(out)), "chain_status")
        return bool(out.value)

    def profile_enable(self, enable: bool = True) -> None:
        """Record HIP events around each step launch of graph_wavelet_features."""
        check(_lib.load().wg_profile_enable(self.handle, 1 if enable else 0), "profile_enable")

    def profile_collect(self) -> dict:
        """Synchronise on the recorded events -> {sum_ms, launches, max_ms}; resets."""
        s, n, m = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0)
        check(_lib.load().wg_profile_collect(self.handle, ctypes.byref(s), ctypes.byref(n), ctypes.byref(m)),
              "profile_collect")
        return dict(sum_ms=s.value, launches=n.value, max_ms=m.value)

    def profile_durations(self, cap: int = 1 << 16) -> list:
        """Synchronise on the recorded events -> each launch's ms, in launch order; resets."""
        buf = (ctypes.c_double * cap)()
        n = ctypes.c_int64(0)
        check(_lib.load().wg_profile_durations(self.handle, buf, cap, ctypes.byref(n)), "profile_durations")
        return [buf[i] for i in range(min(n.value, cap))]

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.load().wg_laplacian_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def shape(self):
        return (self.n, self.n_cols)

    def __repr__(self):
        if self.is_literal:
            return f"NormalizedLaplacian.literal(n={self.n}, nnz={self.nnz}, device={self.device})"
        return f"NormalizedLaplacian(n={self.n}, nnz={self.nnz}, isolated={self.info['n_isolated']}, device={self.device})"
