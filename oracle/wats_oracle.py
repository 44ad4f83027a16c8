"""CPU oracle for the WATS graph-wavelet hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the HIP implementation in
``efficient-gnn_amd/wats_hip``.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker /
the timed CPU baseline -- never as the thing measured or shipped.  The product
path (``wats_hip``) never imports this file and fails loudly when its HIP
library is missing.

It is a numpy/scipy restatement of the reference algorithm in
``calibration/WATS.py`` (CaptainCuong/Efficient-GNN), generalised to F signal
columns and arbitrary (K, s), with the exact dtype flow of the reference:

* ``L`` = ``scipy.sparse.csgraph.laplacian(A, normed=True)``  (float32 COO)
  -- WATS.py:24-27, scipy ``_laplacian.py:467-475``;
* ``L_hat = (2/2.0)*L - identity(N)``  (float64 CSR)          -- WATS.py:55;
* ``X0 = log1p(A.sum(axis=1))``  (float32, (N,1))             -- WATS.py:58-59;
* ``T_0 = X0, T_1 = L_hat X0, T_i = (2 L_hat) T_{i-1} - T_{i-2}`` (float64)
  -- WATS.py:29-37;
* ``S = sum_i exp(-s i) T_i``  (python ``sum`` from int 0, float64) -- WATS.py:65-68;
* ``H = S / (||S||_1,row + 1e-8)``                             -- WATS.py:71-72.

Parity pinning: the restatement is checked against golden vectors produced by
importing the reference module itself in the build container
(``tools/gen_golden.py`` -> ``tests/golden/*.npz``; see DESIGN.md "Oracle").
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from scipy.sparse import csgraph

__all__ = [
    "compute_normalized_laplacian",
    "rescaled_laplacian",
    "laplacian_explicit",
    "log1p_degree",
    "chebyshev_polynomials",
    "heat_coefficients",
    "heat_kernel_combine",
    "row_l1_normalize",
    "graph_wavelet_features",
    "eigen_kat_expected_S",
]


def compute_normalized_laplacian(adj: sp.spmatrix):
    """``L_sym = I - D^-1/2 A D^-1/2`` exactly as WATS.py:24-27 obtains it
    (``csgraph.laplacian(adj, normed=True)``; degree = column sums minus the
    diagonal, scipy ``_laplacian.py:467``)."""
    return csgraph.laplacian(adj, normed=True)


def rescaled_laplacian(adj: sp.spmatrix) -> sp.csr_matrix:
    """``L_hat = (2/2.0) * L - identity(N)`` (WATS.py:53-55) -> float64 CSR.

    Off-diagonals are the float32 values ``-((a_ij / sqrt(w_i)) / sqrt(w_j))``
    upcast to float64; the diagonal is 0 (pruned) for nodes with in-degree
    (excluding self loops) > 0 and -1 for isolated nodes.
    """
    n = adj.shape[0]
    L = compute_normalized_laplacian(adj)
    return ((2 / 2.0) * L - sp.identity(n)).tocsr()


def laplacian_explicit(adj: sp.csr_matrix):
    """Explicit restatement of scipy ``_laplacian.py:467-475`` + WATS.py:55.

    Returns ``(indptr, indices, values_f32, iso_mask, w_sqrt_f32)`` for the
    off-diagonal part of ``L_hat`` (CSR, diagonal removed, same column order as
    ``adj``) -- this is the device layout the HIP prologue produces, so tests can
    compare it bit-for-bit.
    """
    A = sp.csr_matrix(adj, dtype=np.float32)
    n = A.shape[0]
    # _laplacian.py:467  w = m.sum(axis=0) - m.diagonal()   (float32, axis 0 = column sums)
    w = np.asarray(A.sum(axis=0)).ravel().astype(np.float32) - A.diagonal().astype(np.float32)
    iso = w == 0                                            # :470
    sw = np.where(iso, np.float32(1), np.sqrt(w)).astype(np.float32)  # :471
    rows = np.repeat(np.arange(n), np.diff(A.indptr))
    cols = A.indices
    keep = rows != cols                                      # diagonal overwritten by setdiag (:475)
    data = A.data.astype(np.float32)
    vals = -((data / sw[rows]) / sw[cols])                  # :472-474, float32 op order
    vals = vals.astype(np.float32)
    counts = np.bincount(rows[keep], minlength=n)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    return indptr, cols[keep].astype(np.int32), vals[keep], iso, sw


def log1p_degree(adj: sp.spmatrix) -> np.ndarray:
    """WATS.py:58-59: ``X0 = log1p(A.sum(axis=1))`` as float32 (N, 1).

    Note the degree here is the ROW sum INCLUDING self loops -- a different
    degree than the Laplacian's column sum excluding the diagonal.
    """
    degrees = np.array(adj.sum(axis=1)).flatten()
    return np.log1p(degrees).reshape(-1, 1)


def chebyshev_polynomials(L: sp.spmatrix, k: int, X0: np.ndarray) -> list:
    """WATS.py:29-37: ``[T_0 .. T_k]`` with ``T_0 = X0`` (kept in its own dtype),
    ``T_1 = L X0``, ``T_i = (2 L) T_{i-1} - T_{i-2}`` (float64 for float64 L)."""
    T = [X0]
    if k > 0:
        T.append(L @ X0)
    for _ in range(2, k + 1):
        T.append(2 * L @ T[-1] - T[-2])
    return T


def heat_coefficients(k: int, s: float) -> list:
    """WATS.py:65: ``alpha_i = exp(-s * i)`` for i = 0..k (numpy float64 scalars)."""
    return [np.exp(-s * i) for i in range(k + 1)]


def heat_kernel_combine(T: list, s: float) -> np.ndarray:
    """WATS.py:68: ``S = sum(alpha[i] * T[i])`` -- python ``sum`` starting from
    int 0, left to right, float64 (numpy-2 promotion of np.float64 * float32)."""
    alpha = heat_coefficients(len(T) - 1, s)
    return sum(alpha[i] * T[i] for i in range(len(T)))


def row_l1_normalize(S: np.ndarray) -> np.ndarray:
    """WATS.py:71-72: ``H = S / (||S||_1,row + 1e-8)``."""
    row_sums = np.linalg.norm(S, ord=1, axis=1, keepdims=True) + 1e-8
    return S / row_sums


def graph_wavelet_features(adj, k: int = 3, s: float = 0.8, X0=None, return_all: bool = False):
    """WATS.py:39-74 generalised: optional F-column signal ``X0`` (default the
    reference signal ``log1p(rowsum)``).  Returns ``H`` or, with
    ``return_all``, ``dict(H, S, T, L_hat, X0)``."""
    A = sp.csr_matrix(adj) if not sp.issparse(adj) else adj
    L_hat = rescaled_laplacian(A)
    if X0 is None:
        X0 = log1p_degree(A)
    T = chebyshev_polynomials(L_hat, k, X0)
    S = heat_kernel_combine(T, s)
    S = np.asarray(S, dtype=np.float64)
    H = row_l1_normalize(S)
    if return_all:
        return dict(H=H, S=S, T=T, L_hat=L_hat, X0=X0)
    return H


def eigen_kat_expected_S(adj_sym: sp.spmatrix, k: int, s: float):
    """Analytic known-answer test: for a SYMMETRIC ``A``,
    ``v = sqrt(w)`` (w = row sums excluding the diagonal) satisfies
    ``L_hat v = -v``, so with ``X0 = v`` every ``T_k = (-1)^k X0`` and
    ``S = X0 * sum_k (-1)^k exp(-s k)``.  Returns ``(X0 f32 (N,1), coef)``.
    Isolated nodes have ``L_hat_ii = -1`` and ``v_i = 0``, consistent."""
    A = sp.csr_matrix(adj_sym, dtype=np.float32)
    w = np.asarray(A.sum(axis=1)).ravel().astype(np.float64) - A.diagonal().astype(np.float64)
    X0 = np.sqrt(w).astype(np.float32).reshape(-1, 1)
    coef = sum(((-1.0) ** i) * np.exp(-s * i) for i in range(k + 1))
    return X0, coef
