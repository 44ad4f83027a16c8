"""wats_hip -- MI355X-native graph-wavelet feature extractor (WATS hot path).

Drop-in for the hot path of ``calibration/WATS.py`` (CaptainCuong/Efficient-GNN):
the Chebyshev-polynomial heat-kernel wavelet features computed by hand-written
gfx950 HIP kernels behind a C ABI (``include/wats_hip.h``).

Public surface (reference names):
    compute_normalized_laplacian (-> SymNormalizedLaplacian, L_sym with the
    reference's `(2/2.0)*L - identity(N)` arithmetic), chebyshev_polynomials
    (applies its operator literally), graph_wavelet_features,
    WATS  (calibrator), NormalizedLaplacian (device L_hat handle).
Section 8(f): SparseCompatibleGCN / RowNormalizedAdjacency (the base model's
propagation as a HIP SpMM), metrics (device ECE).
"""
from ._lib import LIB_PATH, WaveletError  # noqa: F401
from .graphgen import CSRGraph, named_graph, rmat_graph  # noqa: F401
from .laplacian import NormalizedLaplacian, dense_to_csr  # noqa: F401
from .wavelet import (  # noqa: F401
    SymNormalizedLaplacian,
    as_laplacian,
    as_operator,
    chebyshev_polynomials,
    compute_normalized_laplacian,
    graph_wavelet_features,
    heat_coefficients,
    row_l1_normalize,
)
from .WATS import WATS, accuracy  # noqa: F401
from .gcn import RowNormalizedAdjacency, SparseCompatibleGCN, propagate  # noqa: F401
from .head import wats_head  # noqa: F401

__version__ = "0.1.0"
