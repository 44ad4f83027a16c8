"""ctypes binding of the C restatement of the oracle (oracle/wats_chain.c) --
TEST INFRASTRUCTURE ONLY.

Same contract as :mod:`oracle.wats_oracle` (only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s checks may use it, as the
checker), for graphs where the numpy/scipy restatement is too slow: the
Reddit-size (114.6 M nonzeros) and 8M R-MAT (268 M) parity checks.  Pinned to
:mod:`oracle.wats_oracle` -- itself pinned bit for bit to the reference's
golden vectors -- by ``tests/test_oracle.py::test_c_oracle_matches_python_oracle``.
Build: ``make -C oracle`` (``__graft_entry__.build()`` does it).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# WATS_ORACLE_LIB selects another build of the same source (make -C oracle asan: the sanitizer build)
LIB_PATH = os.environ.get("WATS_ORACLE_LIB") or os.path.join(_HERE, "build", "libwats_oracle.so")
_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"C oracle not built ({LIB_PATH}); run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        lib.wo_wavelet_features.restype = ctypes.c_int
        lib.wo_wavelet_features.argtypes = [i64, vp, vp, vp, vp, i64, i32, vp, vp, vp, i32]
        _lib = lib
    return _lib


def heat_coefficients(k: int, s: float) -> np.ndarray:
    """alpha_i = np.exp(-s * i) exactly as WATS.py:65 computes them."""
    return np.array([np.exp(-s * i) for i in range(k + 1)], dtype=np.float64)


def graph_wavelet_features(indptr, indices, values, X0, k: int, s: float = 0.8, threads: int = 0,
                           return_H: bool = True):
    """S (and H) of WATS.py:39-74 for the adjacency CSR (indptr int64,
    indices int32, values float32 or None = all ones; canonical rows) and an
    (N, F) float32 signal.  Returns (S, H) float64 arrays (H None unless
    ``return_H``)."""
    lib = load()
    indptr = np.ascontiguousarray(indptr, dtype=np.int64)
    indices = np.ascontiguousarray(indices, dtype=np.int32)
    n = len(indptr) - 1
    X0 = np.ascontiguousarray(np.asarray(X0, dtype=np.float32).reshape(n, -1))
    F = X0.shape[1]
    vals = None if values is None else np.ascontiguousarray(values, dtype=np.float32)
    alpha = heat_coefficients(k, s)
    S = np.empty((n, F), dtype=np.float64)
    H = np.empty((n, F), dtype=np.float64) if return_H else None
    rc = lib.wo_wavelet_features(n, indptr.ctypes.data, indices.ctypes.data if indices.size else None,
                                 None if vals is None else vals.ctypes.data, X0.ctypes.data, F, int(k),
                                 alpha.ctypes.data, S.ctypes.data, None if H is None else H.ctypes.data,
                                 int(threads))
    if rc != 0:
        raise MemoryError("C oracle: allocation failed")
    return S, H
