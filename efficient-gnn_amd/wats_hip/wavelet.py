"""Reference-shaped functions of the graph-wavelet hot path (MI355X / HIP).

Same names, argument meaning and defaults as ``calibration/WATS.py``:

* :func:`compute_normalized_laplacian` -- WATS.py:24-27 (+ the rescale of :55);
* :func:`chebyshev_polynomials`        -- WATS.py:29-37;
* :func:`graph_wavelet_features`       -- WATS.py:39-74 (``k=3, s=0.8``).

Differences, by design: inputs may be a dense torch adjacency (ingested on the
device), a scipy sparse matrix, a :class:`CSRGraph` or an already-built
:class:`NormalizedLaplacian`; outputs are float32 torch tensors on the GPU
(the reference returns float64 numpy and the caller casts to float32 at
WATS.py:100); ``X0`` may carry F signal columns.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._lib import check, ptr
from .laplacian import NormalizedLaplacian, require_gpu, stream_handle


def as_laplacian(adj, **kw) -> NormalizedLaplacian:
    if isinstance(adj, NormalizedLaplacian):
        return adj
    if isinstance(adj, torch.Tensor):
        if adj.is_sparse or adj.layout == torch.sparse_csr:
            a = adj.to_sparse_csr()
            return NormalizedLaplacian(a.shape[0], a.crow_indices(), a.col_indices(), a.values(), **kw)
        return NormalizedLaplacian.from_dense(adj, **kw)
    try:
        import scipy.sparse as sp
        if sp.issparse(adj):
            return NormalizedLaplacian.from_scipy(adj, **kw)
    except ImportError:  # pragma: no cover
        pass
    if hasattr(adj, "indptr") and hasattr(adj, "indices"):
        return NormalizedLaplacian.from_graph(adj, **kw)
    import numpy as np
    return NormalizedLaplacian.from_dense(torch.as_tensor(np.asarray(adj, dtype=np.float32)), **kw)


def compute_normalized_laplacian(adj, **kw) -> NormalizedLaplacian:
    """Device ``L_hat = (2/2.0)*laplacian(adj, normed=True) - I`` (WATS.py:24-27, :55)."""
    return as_laplacian(adj, **kw)


def _signal(L: NormalizedLaplacian, X0) -> torch.Tensor:
    if X0 is None:
        return L.log1p_degree()
    X0 = torch.as_tensor(X0)
    if X0.dim() == 1:
        X0 = X0.reshape(-1, 1)
    if X0.shape[0] != L.n:
        raise ValueError(f"X0 has {X0.shape[0]} rows, graph has {L.n}")
    return X0.to(device=L.device, dtype=torch.float32).contiguous()


def heat_coefficients(k: int, s: float) -> list:
    """``alpha_i = exp(-s*i)`` (WATS.py:65)."""
    return [math.exp(-s * i) for i in range(k + 1)]


def chebyshev_polynomials(L, k: int, X0) -> list:
    """``[T_0, ..., T_k]`` with ``T_0 = X0``, ``T_1 = L_hat X0``,
    ``T_i = 2 L_hat T_{i-1} - T_{i-2}`` (WATS.py:29-37); float32 device tensors
    in the caller's row order.  ``L`` is the rescaled operator (what the
    reference passes at WATS.py:62), or anything :func:`as_laplacian` accepts."""
    L = as_laplacian(L)
    X0 = _signal(L, X0)
    T = [X0]
    if k <= 0:
        return T
    cur_m2 = None
    cur_m1 = L.permute(X0, to_internal=True)
    for i in range(1, k + 1):
        out = torch.empty_like(cur_m1)
        L.step(i, cur_m1, cur_m2, out)
        T.append(L.permute(out, to_internal=False))
        cur_m2, cur_m1 = cur_m1, out
    return T


def graph_wavelet_features(adj_matrix, k: int = 3, s: float = 0.8, X0=None, return_S: bool = False):
    """WATS.py:39-74 on the GPU: ``H = rownorm_L1(sum_i exp(-s i) T_i(L_hat) X0)``.

    ``X0`` defaults to the reference signal ``log1p(rowsum(A))`` (N, 1).
    Returns ``H`` (N, F) float32 on the GPU, or ``(H, S)`` with ``return_S``.
    """
    L = as_laplacian(adj_matrix)
    X = _signal(L, X0)
    n, F = X.shape
    S = torch.empty(n, F, dtype=torch.float32, device=L.device)
    H = torch.empty(n, F, dtype=torch.float32, device=L.device)
    with torch.cuda.device(L.device):
        check(_lib.load().wg_wavelet_features(L.handle, ptr(X), F, int(k), float(s), ptr(S), ptr(H),
                                              stream_handle(L.device)), "wavelet_features")
    return (H, S) if return_S else H


def row_l1_normalize(S: torch.Tensor) -> torch.Tensor:
    """``H = S / (||S||_1,row + 1e-8)`` (WATS.py:71-72) on the GPU."""
    device = require_gpu(S.device if S.is_cuda else None)
    S = S.to(device=device, dtype=torch.float32).contiguous()
    if S.dim() == 1:
        S = S.reshape(-1, 1)
    H = torch.empty_like(S)
    with torch.cuda.device(device):
        check(_lib.load().wg_row_l1_normalize(ptr(S), ptr(H), S.shape[0], S.shape[1], stream_handle(device)),
              "row_l1_normalize")
    return H
