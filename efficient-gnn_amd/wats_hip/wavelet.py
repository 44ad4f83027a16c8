"""Reference-shaped functions of the graph-wavelet hot path (MI355X / HIP).

Same names, argument meaning and defaults as ``calibration/WATS.py``:

* :func:`compute_normalized_laplacian` -- WATS.py:24-27 (``L_sym``; the
  rescale of :55 is the reference's own arithmetic on the returned object);
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

import numpy as np
import torch

from . import _lib
from ._lib import WaveletError, check, ptr
from .laplacian import NormalizedLaplacian, require_gpu, stream_handle


def as_laplacian(adj, **kw) -> NormalizedLaplacian:
    if isinstance(adj, NormalizedLaplacian):
        return adj
    if isinstance(adj, SymNormalizedLaplacian):
        return adj.laplacian_hat()
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


def _scalar(c):
    import numbers
    if isinstance(c, numbers.Real) and not isinstance(c, bool):
        return float(c)
    if isinstance(c, (np.floating, np.integer)) or (isinstance(c, np.ndarray) and c.ndim == 0):
        return float(c)
    return None


def _identity_multiple(other, n: int):
    """``d`` if ``other`` is ``d * identity(n)`` (scipy sparse, numpy or torch), else None."""
    import scipy.sparse as sp
    if sp.issparse(other):
        if other.shape != (n, n):
            return None
        o = sp.csr_matrix(other)
        o.sum_duplicates()
        o.eliminate_zeros()
        diag = o.diagonal()
        if o.nnz != np.count_nonzero(diag) or (n and not np.all(diag == diag[0])):
            return None
        return float(diag[0]) if n else 0.0
    return None


class SymNormalizedLaplacian:
    """``scale * L_sym - shift * I`` of an adjacency, with
    ``L_sym = I - D^{-1/2} A D^{-1/2}`` exactly as scipy's
    ``csgraph.laplacian(adj, normed=True)`` builds it (the value
    :func:`compute_normalized_laplacian` returns, reference
    calibration/WATS.py:24-27).

    Supports the reference's own arithmetic on it -- ``(2 / 2.0) * L -
    identity(N)`` (WATS.py:55) -- and ``@`` with a signal.  Nothing touches the
    GPU until the operator is used: the rescale the reference performs maps to
    the device L_hat handle (:class:`NormalizedLaplacian`, the fused step
    kernels); any other scale / shift is applied literally (a valued CSR,
    ``wg_operator_create``)."""

    def __init__(self, adj, scale: float = 1.0, shift: float = 0.0, _base=None):
        self.adj = adj
        self.scale = float(scale)
        self.shift = float(shift)
        self._base = _base if _base is not None else {}   # shared: the built L_hat handle
        n = adj.n if (isinstance(adj, NormalizedLaplacian) or not hasattr(adj, "shape")) else adj.shape[0]
        self.shape = (int(n), int(n))

    # ---- the reference's arithmetic (WATS.py:55): scalar * L, L -/+ d * identity(N)
    def _with(self, scale, shift):
        return SymNormalizedLaplacian(self.adj, scale, shift, self._base)

    def __mul__(self, c):
        c = _scalar(c)
        if c is None:
            return NotImplemented
        return self._with(self.scale * c, self.shift * c)

    __rmul__ = __mul__

    def __truediv__(self, c):
        c = _scalar(c)
        if c is None:
            return NotImplemented
        return self._with(self.scale / c, self.shift / c)

    def __neg__(self):
        return self._with(-self.scale, -self.shift)

    def __sub__(self, other):
        d = _identity_multiple(other, self.shape[0])
        if d is None:
            raise NotImplementedError("wats_hip: only scalar multiples of identity(N) can be subtracted from L")
        return self._with(self.scale, self.shift + d)

    def __add__(self, other):
        d = _identity_multiple(other, self.shape[0])
        if d is None:
            raise NotImplementedError("wats_hip: only scalar multiples of identity(N) can be added to L")
        return self._with(self.scale, self.shift - d)

    __radd__ = __add__

    @property
    def is_rescaled(self) -> bool:
        """True for ``L_sym - I`` = L_hat, the operator of the fused chain."""
        return self.scale == 1.0 and self.shift == 1.0

    # ---- device operators
    def laplacian_hat(self) -> NormalizedLaplacian:
        """The device handle of ``L_hat = L_sym - I`` (built once, shared by
        every scaled copy of this object)."""
        L = self._base.get("L_hat")
        if L is None:
            L = self.adj if isinstance(self.adj, NormalizedLaplacian) else as_laplacian(self.adj)
            self._base["L_hat"] = L
        return L

    def operator(self) -> NormalizedLaplacian:
        """The handle :func:`chebyshev_polynomials` applies: the L_hat handle
        for the reference's rescale, else a literal ``scale * L_sym - shift * I``."""
        if self.is_rescaled:
            return self.laplacian_hat()
        key = ("literal", self.scale, self.shift)
        op = self._base.get(key)
        if op is None:
            L = self.laplacian_hat()
            indptr, indices, values, iso = L.export()
            n = L.n
            # off-diagonal: scale * L_sym_ij (= scale * L_hat_ij); diagonal: scale * (1 - iso) - shift
            rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(indptr))
            diag = self.scale * (1.0 - iso.astype(np.float64)) - self.shift
            r = np.concatenate([rows, np.arange(n, dtype=np.int64)])
            c = np.concatenate([indices.astype(np.int64), np.arange(n, dtype=np.int64)])
            v = np.concatenate([self.scale * values.astype(np.float64), diag])
            order = np.lexsort((c, r))
            r, c, v = r[order], c[order], v[order].astype(np.float32)
            ip = np.zeros(n + 1, dtype=np.int64)
            np.cumsum(np.bincount(r, minlength=n), out=ip[1:])
            op = NormalizedLaplacian.literal(ip, c.astype(np.int32), v, n=n, device=L.device)
            self._base[key] = op
        return op

    def __matmul__(self, X):
        """``(scale L_sym - shift I) X`` on the GPU (float32 (N, F) tensor)."""
        op = self.operator()
        return chebyshev_polynomials(op, 1, X)[1]

    def to_scipy(self):
        """float64 scipy CSR of this operator (caller numbering), for checks."""
        import scipy.sparse as sp
        L_hat = self.laplacian_hat().to_scipy()          # L_sym - I
        n = self.shape[0]
        return (self.scale * L_hat + (self.scale - self.shift) * sp.identity(n)).tocsr()

    def __repr__(self):
        return f"SymNormalizedLaplacian(n={self.shape[0]}, scale={self.scale}, shift={self.shift})"


def compute_normalized_laplacian(adj, **kw) -> SymNormalizedLaplacian:
    """``L_sym = I - D^{-1/2} A D^{-1/2}`` (reference calibration/WATS.py:24-27,
    scipy ``csgraph.laplacian(adj, normed=True)``, ``_laplacian.py:467-475``).

    Returns a :class:`SymNormalizedLaplacian`; the reference's next line,
    ``L_rescaled = (2 / 2.0) * L - identity(N)`` (WATS.py:55), works on it
    unchanged and yields the device ``L_hat`` operator that
    :func:`chebyshev_polynomials` runs on the fused step kernel."""
    if kw:
        return SymNormalizedLaplacian(as_laplacian(adj, **kw))
    return SymNormalizedLaplacian(adj)


def as_operator(L) -> NormalizedLaplacian:
    """What :func:`chebyshev_polynomials` applies, taken LITERALLY (the
    reference applies whatever matrix it is given, WATS.py:32-36): a
    :class:`SymNormalizedLaplacian` expression, a device handle, or an
    explicit scipy / numpy / torch matrix (uploaded as a valued CSR, no
    normalisation)."""
    if isinstance(L, SymNormalizedLaplacian):
        return L.operator()
    if isinstance(L, NormalizedLaplacian):
        return L
    import scipy.sparse as sp
    if isinstance(L, torch.Tensor):
        L = L.detach().to_dense().cpu().numpy() if (L.is_sparse or L.layout != torch.strided) else L.detach().cpu().numpy()
    if not sp.issparse(L):
        L = np.asarray(L)
        if L.ndim != 2:
            raise ValueError("chebyshev_polynomials: L must be a 2-D operator")
    A = sp.csr_matrix(L)
    if A.shape[0] != A.shape[1]:
        raise ValueError("chebyshev_polynomials: L must be square")
    A.sum_duplicates()
    return NormalizedLaplacian.literal(A.indptr.astype(np.int64), A.indices.astype(np.int32),
                                       A.data.astype(np.float32), n=A.shape[0])


def _signal(L: NormalizedLaplacian, X0) -> torch.Tensor:
    if X0 is None:
        if L.is_literal:
            raise ValueError("X0 is required with an explicit operator (the reference passes it, WATS.py:62)")
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
    """``[T_0, ..., T_k]`` with ``T_0 = X0``, ``T_1 = L X0``,
    ``T_i = 2 L T_{i-1} - T_{i-2}`` (WATS.py:29-37); float32 device tensors
    in the caller's row order.  ``L`` is applied as given (see
    :func:`as_operator`): the reference's ``L_rescaled = (2/2.0) *
    compute_normalized_laplacian(adj) - identity(N)`` (WATS.py:55,62) runs on
    the device L_hat handle; an explicit matrix runs as a literal CSR."""
    L = as_operator(L)
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
    lib = _lib.load()
    with torch.cuda.device(L.device):
        def run():
            check(lib.wg_wavelet_features(L.handle, ptr(X), F, int(k), float(s), ptr(S), ptr(H),
                                          stream_handle(L.device)), "wavelet_features")
        try:
            run()
        except WaveletError as e:
            # an earlier asynchronous call's one-launch chain timed out (reported now, WG_ERR_TIMEOUT);
            # the handle has switched to the multi-launch path: this call runs there
            if "status -5:" not in str(e):   # WG_ERR_TIMEOUT
                raise
            run()
        # the one-launch chain (csrc/chain.hip, F = 1 small graphs) waits on other workgroups, so
        # it needs every worker resident; on a GPU shared with another process a wait can give up
        # (its rows are then NaN).  Check that chain alone (an event wait, not a device sync; the
        # reference returns host arrays anyway) and rerun the call on the multi-launch path, which
        # the handle now keeps.  Skipped while the caller captures a graph (no waits allowed then).
        if F == 1 and not torch.cuda.is_current_stream_capturing() and L.chain_status():
            run()
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
