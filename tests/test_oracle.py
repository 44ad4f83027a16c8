"""CPU tests: pin the oracle to the reference's golden vectors, and check the
analytic known-answer tests.  No GPU needed."""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import assert_parity, golden_csr, golden_names, load_golden
from oracle import wats_oracle as O


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_golden(name):
    """The oracle restatement reproduces the reference's own outputs (generated
    by importing calibration/WATS.py, tools/gen_golden.py) bit for bit."""
    d = load_golden(name)
    A = golden_csr(d)
    k, s = int(d["k"]), float(d["s"])
    X0 = d["X0"] if "H_ref_fn" not in d else None
    out = O.graph_wavelet_features(A, k=k, s=s, X0=X0, return_all=True)
    np.testing.assert_array_equal(np.asarray(out["X0"], np.float32), d["X0"])
    np.testing.assert_array_equal(out["S"], d["S"])
    np.testing.assert_array_equal(out["H"], d["H"])
    if "H_ref_fn" in d:
        np.testing.assert_array_equal(out["H"], d["H_ref_fn"])
    if "T" in d:
        for i, t in enumerate(out["T"]):
            np.testing.assert_array_equal(np.asarray(t, np.float64), d["T"][i])
    if "L_values" in d:
        L = out["L_hat"]
        L.sort_indices()
        np.testing.assert_array_equal(L.indptr, d["L_indptr"])
        np.testing.assert_array_equal(L.indices, d["L_indices"])
        np.testing.assert_array_equal(L.data, d["L_values"])


@pytest.mark.parametrize("name", [n for n in golden_names() if "L_values" in load_golden(n)])
def test_explicit_laplacian_matches_scipy(name):
    """laplacian_explicit (the device layout: off-diagonal CSR + iso flags)
    equals scipy's L_hat exactly."""
    d = load_golden(name)
    A = golden_csr(d)
    indptr, indices, vals, iso, _ = O.laplacian_explicit(A)
    n = A.shape[0]
    off = sp.csr_matrix((vals.astype(np.float64), indices, indptr), shape=(n, n))
    L = (off - sp.diags(iso.astype(np.float64))).tocsr()
    L.eliminate_zeros()
    L.sort_indices()
    ref = sp.csr_matrix((d["L_values"], d["L_indices"], d["L_indptr"]), shape=(n, n))
    assert (L != ref).nnz == 0


def test_kat4_values():
    """the 4-node edge-case graph."""
    d = load_golden("kat4_k3")
    np.testing.assert_allclose(d["X0"].ravel(), [1.0986123, 1.0986123, 0, 0.6931472], rtol=1e-7)
    np.testing.assert_allclose(d["S"].ravel(), [0.7271161176, 0.7271161176, 0, 0.4587591859], rtol=1e-9)
    np.testing.assert_allclose(d["H"].ravel(), [0.9999999862, 0.9999999862, 0, 0.9999999782], rtol=1e-9)
    Ld = sp.csr_matrix((d["L_values"], d["L_indices"], d["L_indptr"]), shape=(4, 4)).toarray()
    exp = np.array([[0, -1, 0, 0], [-1, 0, -0.70710677, 0], [0, 0, 0, 0], [0, 0, -0.70710677, -1]])
    np.testing.assert_allclose(Ld, exp, rtol=1e-7)


def test_karate_values():
    d = load_golden("karate_k3")
    np.testing.assert_allclose(d["S"].ravel()[:6], [1.7969560919, 1.4945254827, 1.5641316994, 1.2949055938,
                                                    0.9276752638, 1.0831943589], rtol=1e-9)


@pytest.mark.parametrize("k", [0, 1, 3, 16])
def test_eigenvector_kat(k):
    """For symmetric A, X0 = sqrt(w) is the -1 eigenvector of L_hat, so
    S = X0 * sum_k (-1)^k exp(-s k)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "efficient-gnn_amd"))
    from wats_hip.graphgen import rmat_graph
    g = rmat_graph(3000, 30000, seed=2, self_loops=True)
    A = g.to_scipy()
    X0, coef = O.eigen_kat_expected_S(A, k, 0.8)
    out = O.graph_wavelet_features(A, k=k, s=0.8, X0=X0, return_all=True)
    assert_parity(out["S"], X0.astype(np.float64) * coef, tol=1e-6, what="eigen KAT")


def test_heat_coefficients():
    a = O.heat_coefficients(4, 0.8)
    assert a[0] == 1.0
    np.testing.assert_allclose(a, np.exp(-0.8 * np.arange(5)), rtol=0)


@pytest.mark.parametrize("name", golden_names())
def test_c_oracle_matches_reference_golden(name):
    """The C restatement (oracle/wats_chain.c, the checker for the Reddit / 8M
    sizes) reproduces the reference's golden S and H -- the same float64 row
    sums in the same order as scipy's sparsetools, so bit for bit on S."""
    from oracle import wats_oracle_c as C
    d = load_golden(name)
    A = golden_csr(d)
    A.sort_indices()
    k, s = int(d["k"]), float(d["s"])
    X0 = d["X0"].astype(np.float32)
    S, H = C.graph_wavelet_features(A.indptr, A.indices, A.data, X0, k, s, threads=3)
    np.testing.assert_array_equal(S, d["S"])
    np.testing.assert_allclose(H, d["H"], rtol=1e-14, atol=1e-300)


def test_c_oracle_matches_python_oracle_random_graphs():
    """Wider inputs than the fixtures (unweighted R-MAT F=5 K=16; weighted
    directed graph with self loops and isolated nodes): equal to the numpy
    restatement bit for bit on S, for 1 and 4 threads."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "efficient-gnn_amd"))
    from oracle import wats_oracle_c as C
    from wats_hip.graphgen import random_graph, rmat_graph
    for g, F, k in ((rmat_graph(3000, 40000, seed=3), 5, 16),
                    (random_graph(500, 0.02, seed=4, directed=True, weighted=True, self_loop_frac=0.1,
                                  isolated_frac=0.05), 3, 7)):
        A = g.to_scipy()
        X0 = np.random.default_rng(0).standard_normal((g.n, F)).astype(np.float32)
        ref = O.graph_wavelet_features(A, k=k, s=0.8, X0=X0, return_all=True)
        for th in (1, 4):
            S, H = C.graph_wavelet_features(g.indptr, g.indices, g.values, X0, k, 0.8, threads=th)
            np.testing.assert_array_equal(S, ref["S"])
            np.testing.assert_allclose(H, ref["H"], rtol=1e-14, atol=1e-300)


# ----------------------------------------------------------------- ECE (utils/ece.py:8-89), pinned to the reference
def _ece_cases():
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "ece_cases.npz"))
    return d, sorted({k.split("__")[0] for k in d.files})


def test_ece_oracle_bitwise_vs_reference_fixtures():
    """oracle/ece_oracle.py against the reference's own calculate_ece /
    calculate_average_ece outputs (tools/gen_ece_golden.py imports
    utils/ece.py itself): logits and probabilities, probabilities exactly 0
    and on bin edges, bins with < 4 samples, empty classes -- bit for bit."""
    from oracle import ece_oracle as E
    d, names = _ece_cases()
    assert len(names) >= 10
    for nm in names:
        o, y, (c, lg) = d[nm + "__outputs"], d[nm + "__labels"], d[nm + "__meta"]
        per = np.array([E.calculate_ece(o, y, k, logits=bool(lg)) for k in range(c)])
        np.testing.assert_array_equal(per, d[nm + "__per_class"], err_msg=nm)
        assert E.calculate_average_ece(o, y, int(c), logits=bool(lg)) == d[nm + "__average"][0], nm


def test_ece_metrics_cpu_vs_reference_fixtures():
    """wats_hip.metrics (torch, float64 bins) on CPU tensors against the
    reference's outputs: within 1e-7 absolute (the reference averages float32
    probabilities in float32; the bin assignment is identical)."""
    import torch
    from wats_hip import metrics as M
    d, names = _ece_cases()
    for nm in names:
        o, y, (c, lg) = d[nm + "__outputs"], d[nm + "__labels"], d[nm + "__meta"]
        ot, yt = torch.from_numpy(o), torch.from_numpy(y)
        per = np.array([M.calculate_ece(ot, yt, k, logits=bool(lg)) for k in range(c)])
        assert np.abs(per - d[nm + "__per_class"]).max() <= 1e-7, nm
        assert abs(M.calculate_average_ece(ot, yt, int(c), logits=bool(lg)) - d[nm + "__average"][0]) <= 1e-7, nm
