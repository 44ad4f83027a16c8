"""GPU parity tests: the HIP path (through the C ABI) against the reference's
golden vectors and the CPU oracle, on seeded inputs; size-independent
properties (eigenvector KAT, determinism, relabelling invariance) at the
named full sizes."""
import ctypes
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from conftest import assert_parity, golden_csr, golden_names, load_golden
from oracle import wats_oracle as O

pytestmark = pytest.mark.gpu

import wats_hip  # noqa: E402
from wats_hip import NormalizedLaplacian  # noqa: E402
from wats_hip.graphgen import connect_isolated, named_graph, random_graph, rmat_graph  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    wats_hip._lib.load()


def _np(t):
    return t.detach().cpu().numpy()


# ----------------------------------------------------------------- prologue
@pytest.mark.parametrize("name", golden_names())
def test_laplacian_bit_exact_vs_scipy(name):
    """L_hat values equal scipy's float32 values bit for bit (a1 + a2)."""
    d = load_golden(name)
    A = golden_csr(d)
    L = NormalizedLaplacian.from_scipy(A)
    indptr, indices, vals, iso = L.export()
    r_indptr, r_indices, r_vals, r_iso, _ = O.laplacian_explicit(A)
    np.testing.assert_array_equal(indptr, r_indptr)
    np.testing.assert_array_equal(indices, r_indices)
    np.testing.assert_array_equal(vals.view(np.uint32), r_vals.view(np.uint32))
    np.testing.assert_array_equal(iso, r_iso)
    assert L.info["n_isolated"] == int(r_iso.sum())
    if "L_values" in d:
        ref = sp.csr_matrix((d["L_values"], d["L_indices"], d["L_indptr"]), shape=A.shape)
        got = L.to_scipy()
        got.eliminate_zeros()
        assert (got != ref).nnz == 0


@pytest.mark.parametrize("seed,directed,weighted", [(0, True, True), (1, False, True), (2, True, False)])
def test_laplacian_random_graphs(seed, directed, weighted):
    g = random_graph(700, 0.01, seed=seed, directed=directed, weighted=weighted, self_loop_frac=0.05,
                     isolated_frac=0.05)
    A = g.to_scipy()
    L = NormalizedLaplacian.from_graph(g)
    _, indices, vals, iso = L.export()
    _, r_indices, r_vals, r_iso, _ = O.laplacian_explicit(A)
    np.testing.assert_array_equal(indices, r_indices)
    np.testing.assert_array_equal(vals.view(np.uint32), r_vals.view(np.uint32))
    np.testing.assert_array_equal(iso, r_iso)


@pytest.mark.parametrize("name", golden_names())
def test_log1p_degree(name):
    """X0 = log1p(rowsum) within 1 ulp of numpy's float32 log1p (numpy's SIMD
    float32 log1p is itself 1 ulp from correctly rounded; we round correctly)."""
    d = load_golden(name)
    if "H_ref_fn" not in d:
        pytest.skip("fixture uses an explicit signal")
    L = NormalizedLaplacian.from_scipy(golden_csr(d))
    x0 = _np(L.log1p_degree())
    ulp = np.abs(x0.view(np.int32).astype(np.int64) - d["X0"].view(np.int32).astype(np.int64))
    assert ulp.max() <= 1


def test_dense_ingestion_matches_scipy():
    g = random_graph(300, 0.03, seed=9, directed=True, weighted=True, self_loop_frac=0.1)
    dense = torch.tensor(g.to_scipy().toarray(), dtype=torch.float32, device="cuda")
    indptr, indices, values = wats_hip.dense_to_csr(dense)
    ref = sp.csr_matrix(dense.cpu().numpy())
    np.testing.assert_array_equal(_np(indptr), ref.indptr)
    np.testing.assert_array_equal(_np(indices), ref.indices)
    np.testing.assert_array_equal(_np(values), ref.data)


def test_dense_ingestion_strided_and_empty():
    big = torch.zeros(50, 64, device="cuda")
    big[3, 5] = 2.0
    view = big[:, :50]  # ld = 64
    indptr, indices, values = wats_hip.dense_to_csr(view)
    assert _np(indptr)[-1] == 1 and _np(indices).tolist() == [5] and _np(values).tolist() == [2.0]
    indptr, indices, values = wats_hip.dense_to_csr(torch.zeros(7, 7, device="cuda"))
    assert _np(indptr).tolist() == [0] * 8 and indices.numel() == 0


# ----------------------------------------------------------------- the chain
@pytest.mark.parametrize("name", golden_names())
def test_wavelet_features_vs_reference_golden(name):
    """graph_wavelet_features on the GPU matches the reference's S and H."""
    d = load_golden(name)
    A = golden_csr(d)
    k, s = int(d["k"]), float(d["s"])
    X0 = None if "H_ref_fn" in d else torch.from_numpy(d["X0"])
    H, S = wats_hip.graph_wavelet_features(A, k=k, s=s, X0=X0, return_S=True)
    assert_parity(_np(S), d["S"], what=f"{name} S")
    assert_parity(_np(H), d["H"], what=f"{name} H")
    big = np.abs(d["S"]) > 1e-6
    assert np.array_equal(np.sign(_np(H))[big], np.sign(d["H"])[big])


@pytest.mark.parametrize("name", [n for n in golden_names() if "T" in load_golden(n)])
def test_chebyshev_polynomials_vs_reference_golden(name):
    """The reference's own call sequence (calibration/WATS.py:53-62):
    L = compute_normalized_laplacian(adj); L_rescaled = (2/2.0)*L - identity(N);
    T = chebyshev_polynomials(L_rescaled, k, X0) -- against the golden T_k."""
    from scipy.sparse import identity
    d = load_golden(name)
    A = golden_csr(d)
    k = int(d["k"])
    N = A.shape[0]
    X0 = torch.from_numpy(d["X0"].astype(np.float32))
    L = wats_hip.compute_normalized_laplacian(A)
    L_rescaled = (2 / 2.0) * L - identity(N)
    assert L_rescaled.is_rescaled
    T = wats_hip.chebyshev_polynomials(L_rescaled, k, X0)
    assert len(T) == k + 1
    for i, t in enumerate(T):
        assert_parity(_np(t), d["T"][i], what=f"{name} T_{i}")


@pytest.mark.parametrize("name", ["karate_k3", "directed_weighted300_k5", "cora_rmat_k8"])
def test_chebyshev_polynomials_explicit_operator(name):
    """An explicit matrix is applied literally (WATS.py:32-36): the oracle's
    float64 scipy L_rescaled uploaded as a valued CSR gives the golden T_k; a
    different scale (0.5 * L - I, off the fused path) matches the oracle."""
    from scipy.sparse import identity
    d = load_golden(name)
    A = golden_csr(d)
    k = int(d["k"])
    X0 = d["X0"].astype(np.float32)
    T = wats_hip.chebyshev_polynomials(O.rescaled_laplacian(A), k, torch.from_numpy(X0))
    for i, t in enumerate(T):
        assert_parity(_np(t), d["T"][i], what=f"{name} literal T_{i}")
    L = wats_hip.compute_normalized_laplacian(A)
    half = 0.5 * L - identity(A.shape[0])
    ref = O.chebyshev_polynomials((0.5 * O.compute_normalized_laplacian(A) - identity(A.shape[0])).tocsr(), k,
                                  X0.astype(np.float64))
    T = wats_hip.chebyshev_polynomials(half, k, torch.from_numpy(X0))
    for i, t in enumerate(T):
        assert_parity(_np(t), ref[i], what=f"{name} 0.5 L - I T_{i}")
    # L_sym itself applied to a signal (L @ X)
    y = L @ torch.from_numpy(X0)
    assert_parity(_np(y), O.compute_normalized_laplacian(A) @ X0.astype(np.float64), what=f"{name} L_sym @ X0")


def test_dense_adjacency_path_matches_reference():
    """The WATS ingestion path: dense float32 torch adjacency on the device."""
    d = load_golden("cora_rmat_k3")
    dense = torch.tensor(golden_csr(d).toarray(), device="cuda")
    H = wats_hip.graph_wavelet_features(dense)          # defaults k=3, s=0.8
    assert_parity(_np(H), d["H"], what="dense H")


@pytest.mark.parametrize("F", [1, 2, 3, 4, 5, 8, 40, 41, 64, 130, 300])
def test_signal_widths(F):
    """Every F-tiling / vector width against the oracle (weighted, directed,
    self loops, isolated nodes)."""
    g = random_graph(600, 0.02, seed=F, directed=True, weighted=True, self_loop_frac=0.05, isolated_frac=0.05)
    A = g.to_scipy()
    rng = np.random.default_rng(F)
    X = rng.standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=6, s=0.8, X0=X, return_all=True)
    H, S = wats_hip.graph_wavelet_features(A, k=6, s=0.8, X0=torch.from_numpy(X), return_S=True)
    assert_parity(_np(S), ref["S"], what=f"F={F} S")
    assert_parity(_np(H), ref["H"], what=f"F={F} H")


@pytest.mark.parametrize("k", [0, 1, 2, 5, 32])
def test_orders(k):
    g = rmat_graph(4000, 40000, seed=k)
    A = g.to_scipy()
    ref = O.graph_wavelet_features(A, k=k, s=0.8, return_all=True)
    H, S = wats_hip.graph_wavelet_features(A, k=k, return_S=True)
    assert_parity(_np(S), ref["S"], what=f"K={k} S")
    assert_parity(_np(H), ref["H"], what=f"K={k} H")


def test_pubmed_config_vs_oracle():
    """BASELINE config 1: PubMed-size, K=16, F=1."""
    g = named_graph("pubmed")
    A = g.to_scipy()
    ref = O.graph_wavelet_features(A, k=16, s=0.8, return_all=True)
    H, S = wats_hip.graph_wavelet_features(A, k=16, return_S=True)
    assert_parity(_np(S), ref["S"], what="pubmed S")


def test_arxiv_config_vs_oracle():
    """BASELINE config 2 (the metric's workload): ogbn-arxiv-size, K=16, F=40."""
    g = named_graph("ogbn-arxiv")
    A = g.to_scipy()
    rng = np.random.default_rng(1)
    X = rng.standard_normal((g.n, 40)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=16, s=0.8, X0=X, return_all=True)
    H, S = wats_hip.graph_wavelet_features(A, k=16, X0=torch.from_numpy(X), return_S=True)
    assert_parity(_np(S), ref["S"], what="arxiv S")
    assert_parity(_np(H), ref["H"], what="arxiv H")


@pytest.mark.parametrize("F", [4, 8, 40, 64])
def test_padded_csr_gathers(F):
    """The value-free VEC-4 step on the padded CSR (rows padded to 4-entry chunks of
    dropped pad ids) against the oracle, on the arxiv-size graph and the same graph
    with no closed-form rows: the independent-wave kernel (team.hip; team_iter 32 /
    96 / 512: long rows as part waves combined by arrival counters; its late-operand
    and single-chunk-turn variants 9 / 13; waves dispatched in other orders, bitwise
    equal), the workgroup
    kernel with SELL-ordered team ids and with the per-row loop (bitwise equal: same
    chunks, same sums), the old gather loop (gather4 = 0); repeated calls bitwise
    equal."""
    g = named_graph("ogbn-arxiv")
    for gg in (g, connect_isolated(g, seed=7)):
        A = gg.to_scipy()
        X = np.random.default_rng(F).standard_normal((gg.n, F)).astype(np.float32)
        ref = O.graph_wavelet_features(A, k=16, s=0.8, X0=X, return_all=True)
        L = NormalizedLaplacian.from_graph(gg)
        out = {}
        for knobs in ({}, {"team_iter": 32}, {"team_iter": 512}, {"team": 9}, {"team": 13, "team_iter": 32},
                      {"team_order": 0}, {"team_order": 1, "team_iter": 32}, {"team_order": 6},
                      {"team": 0}, {"team": 0, "sell": 0},
                      {"team": 0, "gather4": 41, "sell": 0}, {"gather4": 0}):
            L.tune(**knobs)
            H, S = wats_hip.graph_wavelet_features(L, k=16, X0=torch.from_numpy(X), return_S=True)
            H2, S2 = wats_hip.graph_wavelet_features(L, k=16, X0=torch.from_numpy(X), return_S=True)
            assert torch.equal(S, S2) and torch.equal(H, H2), f"{knobs}: repeated calls differ"
            out[str(knobs)] = (_np(S), _np(H))
            assert_parity(out[str(knobs)][0], ref["S"], what=f"padded CSR F={F} {knobs} S")
            assert_parity(out[str(knobs)][1], ref["H"], what=f"padded CSR F={F} {knobs} H")
            L.tune(gather4=1, sell=1, team=1, team_iter=96, team_order=-1)
        assert np.array_equal(out["{'team': 0}"][0], out["{'team': 0, 'sell': 0}"][0])
        # gather4 = 41 sums 4 chunks per turn (a 16-term float32 tree, not 8): a different kernel
        # really ran (the F = 1 vidx knob used to overwrite the variant, so it never did)
        assert not np.array_equal(out["{'team': 0, 'gather4': 41, 'sell': 0}"][0], out["{'team': 0, 'sell': 0}"][0])
        assert np.array_equal(out["{}"][0], out["{'team_order': 0}"][0]), "the wave order changed the sums"
        assert np.array_equal(out["{}"][0], out["{'team_order': 6}"][0])
        L.close()


def test_hub_rows_long_row_path():
    """A star graph: one row of 20k nonzeros exercises the workgroup-per-row
    path (and fp64 accumulation on a hub)."""
    n = 20001
    src = np.zeros(n - 1, np.int64)
    dst = np.arange(1, n)
    A = sp.coo_matrix((np.ones(2 * (n - 1), np.float32), (np.r_[src, dst], np.r_[dst, src])), shape=(n, n)).tocsr()
    for F in (1, 40):
        X = np.random.default_rng(F).standard_normal((n, F)).astype(np.float32)
        ref = O.graph_wavelet_features(A, k=5, s=0.8, X0=X, return_all=True)
        H, S = wats_hip.graph_wavelet_features(A, k=5, X0=torch.from_numpy(X), return_S=True)
        assert_parity(_np(S), ref["S"], what=f"star F={F}")


# ----------------------------------------------------------------- properties at full size
@pytest.mark.parametrize("name,k", [("ogbn-arxiv", 16), ("pubmed", 32)])
def test_eigenvector_kat_full_size(name, k):
    """X0 = sqrt(w) -> S = X0 * sum_k (-1)^k e^{-sk} exactly (any size)."""
    g = named_graph(name)
    A = g.to_scipy()
    X0, coef = O.eigen_kat_expected_S(A, k, 0.8)
    H, S = wats_hip.graph_wavelet_features(g, k=k, X0=torch.from_numpy(X0), return_S=True)
    assert_parity(_np(S), X0.astype(np.float64) * coef, what=f"{name} eigen KAT")


def test_deterministic_and_reorder_invariant():
    g = named_graph("ogbn-arxiv")
    X = torch.randn(g.n, 8, generator=torch.Generator().manual_seed(0))
    L = NormalizedLaplacian.from_graph(g)
    H1, S1 = wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)
    H2, S2 = wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)
    assert torch.equal(S1, S2) and torch.equal(H1, H2)
    L0 = NormalizedLaplacian.from_graph(g, reorder=False)
    H3, S3 = wats_hip.graph_wavelet_features(L0, k=16, X0=X, return_S=True)
    # relabelling keeps each row's column order; only the lane split of the
    # float64 row sums differs -> agreement far inside the 1e-5 contract
    assert_parity(_np(S3), _np(S1).astype(np.float64), tol=1e-6, what="reorder invariance")


def test_invalid_arguments_raise():
    g = random_graph(50, 0.1, seed=0)
    L = NormalizedLaplacian.from_graph(g)
    with pytest.raises(wats_hip.WaveletError):
        wats_hip.graph_wavelet_features(L, k=-1)
    with pytest.raises(ValueError):
        wats_hip.graph_wavelet_features(L, X0=torch.zeros(49, 1))


# ----------------------------------------------------------------- drop-in
def test_wats_dropin_on_gpu_matches_reference():
    from models import CompatibleGCN
    d = load_golden("wats_forward120")
    n, nfeat = d["x"].shape
    ncls = d["base.gc2.weight"].shape[0]
    base = CompatibleGCN(nfeat, ncls, nhid=d["base.gc1.weight"].shape[0])
    base.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in d.items() if k.startswith("base.")})
    base.eval()
    for p in base.parameters():
        p.requires_grad = False
    x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["y"])
    adj, val = torch.from_numpy(d["adj"]), torch.from_numpy(d["val_mask"])
    w = wats_hip.WATS(base, x, y, adj, val, verbose=False)
    assert w.wavelet_feats.is_cuda
    assert_parity(_np(w.wavelet_feats), d["wavelet_feats"], what="WATS wavelet_feats")
    w.net.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in d.items() if k.startswith("net.")})
    w.eval()
    with torch.no_grad():
        out = _np(w(x, adj))
    np.testing.assert_allclose(out, d["out"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("knobs", [dict(bcast=0), dict(nt=0), dict(iter=2, block_iter=1, chunk_iter=1),
                                   dict(iter=64, block_iter=256, chunk_iter=256), dict(tile_f=8),
                                   dict(bcast=0, iter=4, block_iter=2, chunk_iter=2),
                                   dict(waves=16, block_iter=4, chunk_iter=2), dict(waves=8, iter=4, block_iter=8),
                                   dict(inkernel_combine=0, iter=2, block_iter=1, chunk_iter=1),
                                   dict(inkernel_combine=1, iter=2, block_iter=1, chunk_iter=2, waves=8),
                                   dict(fuse_finalize=0), dict(fuse_finalize=0, tile_f=8), dict(nt=4), dict(nt=8)])
def test_tuning_knobs_preserve_results(knobs):
    _check_knobs(knobs, F=12)


@pytest.mark.parametrize("knobs", [dict(vidx=1), dict(vidx=1, iter=2, block_iter=1, chunk_iter=1), dict(hot=4096), dict(hot=1000, waves=16), dict(hot=32768, waves=4, iter=2, block_iter=1,
                                                                                  chunk_iter=1)])
def test_hot_column_cache_f1(knobs):
    """F == 1 persistent kernel with the LDS hot-column cache."""
    _check_knobs(knobs, F=1)


def _check_knobs(knobs, F):
    """Every plan shape / kernel variant the tuning knobs select computes the
    same features (team, block and split rows, pipelined loads, F tiling)."""
    g = named_graph("pubmed")
    A = g.to_scipy()
    rng = np.random.default_rng(3)
    X = rng.standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=8, s=0.8, X0=X, return_all=True)
    L = NormalizedLaplacian.from_graph(g)
    H0, S0 = wats_hip.graph_wavelet_features(L, k=8, X0=torch.from_numpy(X), return_S=True)
    L.tune(**knobs)
    H1, S1 = wats_hip.graph_wavelet_features(L, k=8, X0=torch.from_numpy(X), return_S=True)
    assert_parity(_np(S1), ref["S"], what=f"{knobs} S")
    assert_parity(_np(H1), ref["H"], what=f"{knobs} H")
    if set(knobs) <= {"bcast", "nt", "inkernel_combine"}:
        assert torch.equal(S0, S1), "same plan must give bitwise-identical results"


@pytest.mark.parametrize("k", [1, 2, 3, 4, 7, 16])
@pytest.mark.parametrize("F,fuse", [(4, 1), (40, 1), (40, 0), (6, 1), (130, 1)])
def test_clenshaw_heat_sum_vs_forward_and_oracle(k, F, fuse):
    """wavelet_features' default heat sum (Clenshaw's recurrence: no S stream,
    b_k written over b_{k+2}) against the oracle's forward recurrence and the
    forward chain (clenshaw = 0), for every K parity / small-K special case,
    fused and unfused finalize, padded (F = 6) and multi-tile (F = 130) widths,
    on a weighted directed graph with self loops and isolated nodes."""
    g = random_graph(700, 0.02, seed=k * 7 + F, directed=True, weighted=True, self_loop_frac=0.05,
                     isolated_frac=0.08)
    A = g.to_scipy()
    X = np.random.default_rng(k + F).standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=k, s=0.8, X0=X, return_all=True)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(fuse_finalize=fuse, clenshaw=1)
    H1, S1 = wats_hip.graph_wavelet_features(L, k=k, X0=torch.from_numpy(X), return_S=True)
    L.tune(clenshaw=0)
    H0, S0 = wats_hip.graph_wavelet_features(L, k=k, X0=torch.from_numpy(X), return_S=True)
    for S, H, tag in ((S1, H1, "clenshaw"), (S0, H0, "forward")):
        assert_parity(_np(S), ref["S"], what=f"K={k} F={F} {tag} S")
        assert_parity(_np(H), ref["H"], what=f"K={k} F={F} {tag} H")


@pytest.mark.parametrize("k", [1, 2, 3, 4, 16])
@pytest.mark.parametrize("F,knobs", [(4, {}), (40, {}), (40, dict(fuse_finalize=0)), (130, {}), (6, {}),
                                     (1, dict(lds=0)), (1, dict(lds=0, vidx=1)), (40, dict(bcast=0)),
                                     (40, dict(iter=2, block_iter=1, chunk_iter=1))])
def test_clenshaw_value_free_unweighted(k, F, knobs):
    """Unweighted graphs: the Clenshaw chain carries u = b * dinv and gathers
    no CSR values (L_hat_ij = -dinv_i dinv_j); isolated rows, split / block /
    team rows, every gather variant, against the oracle and against the
    valued form (uscale = 0)."""
    g = rmat_graph(3000, 30000, seed=k + F)
    A = g.to_scipy()
    X = np.random.default_rng(k * F).standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=k, s=0.8, X0=X, return_all=True)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(uscale=1, **knobs)
    H1, S1 = wats_hip.graph_wavelet_features(L, k=k, X0=torch.from_numpy(X), return_S=True)
    L.tune(uscale=0)
    H0, S0 = wats_hip.graph_wavelet_features(L, k=k, X0=torch.from_numpy(X), return_S=True)
    for S, H, tag in ((S1, H1, "u-scaled"), (S0, H0, "valued")):
        assert_parity(_np(S), ref["S"], what=f"K={k} F={F} {knobs} {tag} S")
        if F > 1:
            assert_parity(_np(H), ref["H"], what=f"K={k} F={F} {knobs} {tag} H")


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_clenshaw_value_free_directed_selfloops(seed):
    """The value-free chain on unweighted DIRECTED graphs with self loops and
    isolated nodes (w = column sum minus the diagonal, WATS.py:26 -> scipy
    _laplacian.py:467): L_hat_ij = -dinv_i dinv_j still holds off the diagonal."""
    g = random_graph(900, 0.01, seed=seed, directed=True, weighted=False, self_loop_frac=0.1, isolated_frac=0.1)
    A = g.to_scipy()
    X = np.random.default_rng(seed).standard_normal((g.n, 8)).astype(np.float32)
    for k in (3, 8):
        ref = O.graph_wavelet_features(A, k=k, s=0.8, X0=X, return_all=True)
        H, S = wats_hip.graph_wavelet_features(A, k=k, s=0.8, X0=torch.from_numpy(X), return_S=True)
        assert_parity(_np(S), ref["S"], what=f"directed unweighted seed={seed} K={k} S")
        assert_parity(_np(H), ref["H"], what=f"directed unweighted seed={seed} K={k} H")


# ----------------------------------------------------------------- F == 1 column-blocked LDS kernel
@pytest.mark.parametrize("knobs", [dict(lds=0), dict(lds=1), dict(lds=1, lds_cb=2048), dict(lds=1, lds_cb=1024, lds_iter=2),
                                   dict(lds=1, lds_cb=4096, lds_iter=64, lds_wg=7),
                                   dict(lds=1, lds_cb=512, lds_maxnb=64), dict(lds=1, lds_cb=40704, lds_wg=1),
                                   dict(lds=2, lds_cb=2048), dict(lds=2, lds_cb=512, lds_maxnb=64),
                                   dict(lds=2, lds_wg=3), dict(lds=2, lds_cb=4096, lds_wg=1000),
                                   dict(lds=2, lds_depth=2, lds_k=1), dict(lds=2, lds_depth=8, lds_cb=1024, lds_k=1),
                                   dict(lds=2, lds_k=2), dict(lds=2, lds_k=2, lds_cb=1024),
                                   dict(lds=2, lds_k=4, lds_cb=512, lds_maxnb=64), dict(lds=2, lds_k=4, lds_wg=5),
                                   dict(lds=2, lds_perm=0), dict(lds=2, lds_perm=0, lds_k=1, lds_cb=1024),
                                   dict(lds=4), dict(lds=4, lds_cb=1024), dict(lds=4, lds_cb=32),
                                   dict(lds=4, lds_cb=4096, hub_iter=2, lds_wg=7), dict(lds=4, lds_cb=1024, lds_wg=1),
                                   dict(lds=4, lds_cb=2048, hub_iter=64), dict(lds=4, lds_cb=512, hub_iter=1),
                                   dict(lds=4, lds_cb=2048, hub_iter=3, hub_sell=0),
                                   dict(lds=4, hub_sell=0), dict(lds=4, lds_cb=4096, hub_sell=0),
                                   dict(lds=4, lds_cb=2048, hub_iter=3), dict(lds=4, lds_cb=1024, hub_iter=64, lds_wg=3)])
def test_lds1_plans_f1(knobs):
    """The LDS kernel (one and many column blocks, every team width, any
    workgroup split) and the gather kernel it replaces agree with the oracle."""
    _check_knobs(knobs, F=1)


def test_lds1_is_the_f1_path_and_deterministic():
    g = named_graph("pubmed")
    L = NormalizedLaplacian.from_graph(g)
    assert "lds1:" in L.describe(1)
    L.tune(lds=1, lds_cb=2048)
    assert "(+combine)" in L.describe(1)
    X = L.log1p_degree()
    H1, S1 = wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)
    H2, S2 = wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)
    assert torch.equal(S1, S2) and torch.equal(H1, H2)
    L.tune(lds=2, lds_cb=2048)
    assert "windows" in L.describe(1)
    X = L.log1p_degree()
    H1, S1 = wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)
    H2, S2 = wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)
    assert torch.equal(S1, S2) and torch.equal(H1, H2)


@pytest.mark.parametrize("seed", [0, 1])
def test_lds1_directed_isolated_selfloops(seed):
    """Unweighted directed graph with self loops and isolated nodes (L_hat_ii = -1
    rows that still have off-diagonal entries) through the LDS kernel."""
    g = random_graph(3000, 0.004, seed=seed, directed=True, weighted=False, self_loop_frac=0.05, isolated_frac=0.05)
    A = g.to_scipy()
    L = NormalizedLaplacian.from_graph(g)
    L.tune(lds=2 if seed else 3, lds_cb=512 if seed else 32768)  # auto picks row teams for one block
    assert "lds1:" in L.describe(1)
    X = np.random.default_rng(seed).standard_normal((g.n, 1)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=7, s=0.8, X0=X, return_all=True)
    H, S = wats_hip.graph_wavelet_features(L, k=7, X0=torch.from_numpy(X), return_S=True)
    assert_parity(_np(S), ref["S"], what="lds1 directed S")
    # H = S / (|S| + 1e-8) at F = 1 is ill-conditioned where |S| ~ 1e-8..1e-4 (a random
    # signal cancels there; float32 storage alone gives ~3e-5 on such rows): compare H
    # where |S| is not tiny, and check H is exactly the normalisation of the S we return
    Sg, Hg = _np(S).astype(np.float64), _np(H).astype(np.float64)
    ok = np.abs(ref["S"]) > 1e-3 * np.abs(ref["S"]).max()
    assert np.abs(Hg[ok] - ref["H"][ok]).max() <= 1e-5
    np.testing.assert_allclose(Hg, (Sg / (np.abs(Sg) + 1e-8)).astype(np.float32), rtol=1e-6, atol=1e-7)


def test_lds1_not_taken_for_weighted_graphs():
    g = random_graph(500, 0.02, seed=3, directed=False, weighted=True)
    L = NormalizedLaplacian.from_graph(g)
    assert "lds1:" not in L.describe(1)


def test_lds1_arxiv_f1_vs_oracle():
    """ogbn-arxiv-size at F = 1 (the reference signal) through the LDS kernel (3 blocks)."""
    g = named_graph("ogbn-arxiv")
    A = g.to_scipy()
    L = NormalizedLaplacian.from_graph(g)
    assert "lds1:" not in L.describe(1)  # auto: 3 blocks, short rows -> the gather kernel
    L.tune(lds=2)
    assert "windows" in L.describe(1)
    ref = O.graph_wavelet_features(A, k=16, s=0.8, return_all=True)
    H, S = wats_hip.graph_wavelet_features(L, k=16, return_S=True)
    assert_parity(_np(S), ref["S"], what="arxiv F=1 S")
    assert_parity(_np(H), ref["H"], what="arxiv F=1 H")


# ----------------------------------------------------------------- 8(f)-2: base-model propagation
def _dense_norm(A):
    adj = torch.tensor(A.toarray(), dtype=torch.float32, device="cuda")
    deg = adj.sum(dim=1, keepdim=True)
    deg[deg == 0] = 1
    return adj, adj / deg


@pytest.mark.parametrize("F", [1, 7, 64, 130, 500])
@pytest.mark.parametrize("kind", ["weighted_directed", "rmat"])
def test_rownorm_spmm_forward_backward_vs_dense_torch(F, kind):
    """adj_norm @ x (reference src/gnn/model.py:43-47) and its x-gradient
    against the dense torch fp32 product; rel tolerance 1e-5 of max|ref|."""
    if kind == "rmat":
        g = rmat_graph(3000, 30000, seed=F)
    else:
        g = random_graph(900, 0.01, seed=F, directed=True, weighted=True, self_loop_frac=0.1, isolated_frac=0.05)
    A = g.to_scipy()
    adj, norm = _dense_norm(A)
    op = wats_hip.RowNormalizedAdjacency.from_dense(adj)
    x = torch.randn(g.n, F, device="cuda", generator=torch.Generator("cuda").manual_seed(F), requires_grad=True)
    y = wats_hip.propagate(op, x)
    ref = norm.double() @ x.detach().double()
    assert_parity(_np(y), _np(ref), what=f"spmm F={F}")
    gy = torch.randn_like(y)
    (y * gy).sum().backward()
    gref = norm.double().t() @ gy.double()
    assert_parity(_np(x.grad), _np(gref), what=f"spmm grad F={F}")


def test_sparse_gcn_matches_dense_compatible_gcn():
    """SparseCompatibleGCN == the reference CompatibleGCN (same weights, eval mode):
    logits and parameter gradients."""
    from models import CompatibleGCN
    g = rmat_graph(2708, 10556, seed=3)
    adj, _ = _dense_norm(g.to_scipy() + __import__("scipy").sparse.eye(g.n))
    torch.manual_seed(0)
    x = torch.randn(g.n, 300, device="cuda")
    ref = CompatibleGCN(300, 7, nhid=64).cuda().eval()
    sp_model = wats_hip.SparseCompatibleGCN(300, nclass=7, nhid=64).cuda().eval()
    sp_model.load_state_dict(ref.state_dict())
    out_ref, out = ref(x, adj), sp_model(x, adj)
    assert_parity(_np(out), _np(out_ref).astype(np.float64), tol=1e-5, what="gcn logits")
    out_ref.square().sum().backward()
    out.square().sum().backward()
    for (n1, p1), (n2, p2) in zip(ref.named_parameters(), sp_model.named_parameters()):
        assert_parity(_np(p2.grad), _np(p1.grad).astype(np.float64), tol=1e-4, what=f"grad {n1}")
    with pytest.raises(NotImplementedError):
        sp_model(x, adj.clone().requires_grad_(True))


def test_wats_with_sparse_base_model_matches_reference_fixture():
    """The WATS drop-in over SparseCompatibleGCN reproduces the reference
    WATS.forward fixture (same head and base weights)."""
    d = load_golden("wats_forward120")
    n, nfeat = d["x"].shape
    ncls = d["base.gc2.weight"].shape[0]
    base = wats_hip.SparseCompatibleGCN(nfeat, nclass=ncls, nhid=d["base.gc1.weight"].shape[0])
    base.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in d.items() if k.startswith("base.")})
    base.eval()
    for p in base.parameters():
        p.requires_grad = False
    x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["y"])
    adj, val = torch.from_numpy(d["adj"]), torch.from_numpy(d["val_mask"])
    w = wats_hip.WATS(base, x, y, adj, val, verbose=False)
    w.net.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in d.items() if k.startswith("net.")})
    w.eval()
    with torch.no_grad():
        out = _np(w(x, adj))
    np.testing.assert_allclose(out, d["out"], rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------- 8(f)-3: fused temperature head
@pytest.mark.parametrize("F,C,n", [(1, 7, 2708), (1, 40, 5000), (40, 41, 3000), (3, 1, 17), (1, 130, 900)])
def test_fused_head_forward_backward_vs_torch(F, C, n):
    """wats_head == log_softmax(logits / log(exp(net(H)) + 1.1)) (WATS.py:124-130)
    in torch fp32, forward and all gradients."""
    from torch import nn
    torch.manual_seed(F * 100 + C)
    net = nn.Sequential(nn.Linear(F, 16), nn.ReLU(), nn.Linear(16, 1)).cuda()
    H = torch.randn(n, F, device="cuda")
    logits = (3 * torch.randn(n, C, device="cuda")).requires_grad_(True)
    out = wats_hip.wats_head(H, logits, net)
    t = net(H).squeeze(-1)
    T = torch.log(torch.exp(t) + 1.1)
    ref = torch.log_softmax(logits / T.unsqueeze(1), dim=1)
    assert_parity(_np(out), _np(ref).astype(np.float64), what="head forward")
    g = torch.randn_like(ref)
    grads = torch.autograd.grad((out * g).sum(), [logits] + list(net.parameters()))
    refg = torch.autograd.grad((ref * g).sum(), [logits] + list(net.parameters()))
    for a, b, name in zip(grads, refg, ["logits", "W1", "b1", "W2", "b2"]):
        assert_parity(_np(a).reshape(-1, 1), _np(b).reshape(-1, 1).astype(np.float64), tol=2e-5, what=f"d{name}")


def test_fused_head_deterministic_and_wats_trains_with_it():
    """Bitwise-reproducible backward; WATS calib_train with the fused head
    reaches the same loss as with the reference torch ops."""
    from models import CompatibleGCN
    d = load_golden("wats_forward120")
    n, nfeat = d["x"].shape
    ncls = d["base.gc2.weight"].shape[0]
    x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["y"])
    adj, val = torch.from_numpy(d["adj"]), torch.from_numpy(d["val_mask"])
    outs = []
    for fused in (True, False):
        base = CompatibleGCN(nfeat, ncls, nhid=d["base.gc1.weight"].shape[0])
        base.load_state_dict({k[5:]: torch.from_numpy(v) for k, v in d.items() if k.startswith("base.")})
        base.eval()
        torch.manual_seed(0)
        w = wats_hip.WATS(base, x, y, adj, val, verbose=False, fused_head=fused)
        w.eval()
        with torch.no_grad():
            outs.append(_np(w(x, adj)))
    np.testing.assert_allclose(outs[0], outs[1], rtol=2e-4, atol=2e-4)
    # determinism of the fused backward
    from torch import nn
    net = nn.Sequential(nn.Linear(1, 16), nn.ReLU(), nn.Linear(16, 1)).cuda()
    H = torch.randn(10000, 1, device="cuda")
    lg = torch.randn(10000, 7, device="cuda")
    g1 = torch.autograd.grad(wats_hip.wats_head(H, lg, net).sum(), list(net.parameters()))
    g2 = torch.autograd.grad(wats_hip.wats_head(H, lg, net).sum(), list(net.parameters()))
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))


def test_split_rows_inkernel_combine_bitwise_equals_combine_kernel():
    """Hub rows split over workgroups: the in-kernel last-arriver combine (sc1
    hand-off) sums the same partials in the same order as combine_kernel, so the
    two are bitwise identical, and stable over repeated calls."""
    g = named_graph("ogbn-arxiv")
    X = torch.randn(g.n, 40, generator=torch.Generator().manual_seed(5))
    L = NormalizedLaplacian.from_graph(g)
    L.tune(chunk_iter=4, block_iter=8)  # many split rows
    assert "split rows" in L.describe(40)
    outs = []
    for ink in (1, 0, 1):
        L.tune(inkernel_combine=ink)
        outs.append(wats_hip.graph_wavelet_features(L, k=16, X0=X, return_S=True)[1])
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


# ----------------------------------------------------------------- section 8(f)-4: ECE on the device
@pytest.mark.parametrize("logits,n,c", [(True, 5000, 7), (False, 3000, 40), (True, 169343, 40)])
def test_device_ece_vs_restatement(logits, n, c):
    """wats_hip.metrics on GPU tensors (utils/ece.py:8-89: 10 equal-width
    bins per class, np.digitize quirks) against oracle/ece_oracle.py (pinned
    bit for bit to the reference's own outputs, test_oracle.py)."""
    from oracle import ece_oracle as E
    from wats_hip import metrics as M
    rng = np.random.default_rng(n)
    out = (rng.standard_normal((n, c)) * 3).astype(np.float32)
    if not logits:
        out = np.exp(out) / np.exp(out).sum(1, keepdims=True)
        out[:7, 0] = 0.0
    y = rng.integers(0, c, n)
    ref = E.calculate_average_ece(out, y, c, logits=logits)
    o_d, y_d = torch.from_numpy(out).cuda(), torch.from_numpy(y).cuda()
    got = M.calculate_average_ece(o_d, y_d, c, logits=logits)
    assert abs(got - ref) < 1e-6
    for k in (0, c // 2, c - 1):
        assert abs(M.calculate_ece(o_d, y_d, k, logits=logits) - E.calculate_ece(out, y, k, logits=logits)) < 1e-6


def test_device_ece_vs_reference_fixtures():
    """wats_hip.metrics on device tensors against the reference's own
    calculate_ece / calculate_average_ece outputs (tests/golden/ece_cases.npz,
    tools/gen_ece_golden.py): every case, every class, within 1e-7."""
    from wats_hip import metrics as M
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "ece_cases.npz"))
    for nm in sorted({k.split("__")[0] for k in d.files}):
        o, y, (c, lg) = d[nm + "__outputs"], d[nm + "__labels"], d[nm + "__meta"]
        ot, yt = torch.from_numpy(o).cuda(), torch.from_numpy(y).cuda()
        per = np.array([M.calculate_ece(ot, yt, k, logits=bool(lg)) for k in range(c)])
        assert np.abs(per - d[nm + "__per_class"]).max() <= 1e-7, nm
        assert abs(M.calculate_average_ece(ot, yt, int(c), logits=bool(lg)) - d[nm + "__average"][0]) <= 1e-7, nm


# ----------------------------------------------------------------- small chains as a hipGraph
def _wf_call(L, X, S, H, K, s=0.8):
    lib = wats_hip._lib.load()
    wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), X.shape[1], K, s, S.data_ptr(), H.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream), "wavelet_features")


@pytest.mark.parametrize("F", [1, 8, 40])
def test_chain_graph_replay_bitwise(F):
    """wg_wavelet_features replayed as a hipGraph (tuning key graph = 1, the
    auto choice for PubMed-size chains): bitwise equal to the eager chain over
    repeated calls, picks up new signal contents behind the same pointer, and
    matches the oracle (WATS.py:39-74)."""
    g = rmat_graph(19717, 88648, seed=5)
    rng = np.random.default_rng(F)
    Xh = rng.standard_normal((g.n, F)).astype(np.float32)
    outs = {}
    for mode in (0, 1):
        L = NormalizedLaplacian.from_graph(g)
        L.tune(graph=mode)
        X = torch.from_numpy(Xh).cuda()
        S = torch.empty(g.n, F, device="cuda")
        H = torch.empty(g.n, F, device="cuda")
        res = []
        for i in range(5):   # eager, eager, capture + replay, replay, replay
            _wf_call(L, X, S, H, 16)
            res.append((S.clone(), H.clone()))
        X.mul_(-0.5)          # same pointer, new contents: a replay must read them
        _wf_call(L, X, S, H, 16)
        res.append((S.clone(), H.clone()))
        torch.cuda.synchronize()
        outs[mode] = res
        L.close()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert all(torch.equal(r[0], outs[1][0][0]) for r in outs[1][:5])
    ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=Xh, return_all=True)
    assert_parity(outs[1][4][0].cpu().numpy(), ref["S"], what=f"graph replay F={F} S")
    assert_parity(outs[1][5][0].cpu().numpy(), -0.5 * ref["S"], what=f"graph replay F={F} S (new X0)")


def test_chain_under_torch_graph_capture():
    """A caller may capture wg_wavelet_features into its own CUDA graph once
    the width was run uncaptured (plans and workspace exist); the replayed
    graph equals the eager chain."""
    g = rmat_graph(3000, 30000, seed=2)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(graph=0)
    X = torch.randn(g.n, 4, device="cuda")
    S0, H0 = torch.empty(g.n, 4, device="cuda"), torch.empty(g.n, 4, device="cuda")
    _wf_call(L, X, S0, H0, 8)     # uncaptured first call: builds plans and workspace
    S, H = torch.empty_like(S0), torch.empty_like(H0)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(cg, stream=side):
            _wf_call(L, X, S, H, 8)
    cg.replay()
    torch.cuda.synchronize()
    assert torch.equal(S, S0) and torch.equal(H, H0)
    L.close()


# ----------------------------------------------------------------- the one-launch chain (chain.hip)
@pytest.mark.parametrize("n,nnz,K,knobs", [(19717, 88648, 16, {}), (2708, 10556, 8, {}), (2708, 10556, 3, {"chain_wg": 1}),
                                           (19717, 88648, 1, {}), (19717, 88648, 2, {"chain_solo": 2}),
                                           (19717, 88648, 3, {"chain_solo": 2}), (19717, 88648, 16, {"chain_solo": 2}),
                                           (19717, 88648, 32, {"chain_solo": 2}), (2708, 10556, 1, {}),
                                           (19717, 88648, 2, {"chain_wg": 3}),
                                           (19717, 88648, 32, {"chain_wg": 16, "chain_xcd": 1}),
                                           (19717, 88648, 16, {"chain_solo": 0, "chain_xcd": 1}),
                                           (19717, 88648, 16, {"chain_solo": 0, "chain_direct": 1}),
                                           (19717, 88648, 2, {"chain_solo": 0, "chain_direct": 1}),
                                           (19717, 88648, 32, {"chain_wg": 16, "chain_direct": 1}),
                                           (6000, 150000, 16, {"chain_wg": 5}), (6000, 150000, 16, {})])
def test_chain1_vs_oracle(n, nnz, K, knobs):
    """F = 1 small graphs run the whole chain in one launch: one
    workgroup with the ids in registers (solo, the default where it fits: Cora
    and PubMed size) or P workers exchanging granules: PubMed-size K = 16 (the
    BASELINE configs[1] workload) and Cora-size K = 8, K = 1 / 2 / 3 / 32
    (every branch of the Clenshaw phase coefficients), 1 to 16 workers, XCD
    placement, against the oracle with the reference signal and a random one,
    repeated calls bitwise equal, no barrier timeout."""
    g = rmat_graph(n, nnz, seed=K)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(**knobs)
    rng = np.random.default_rng(n + K)
    for X in (None, rng.standard_normal((g.n, 1)).astype(np.float32)):
        Xt = None if X is None else torch.from_numpy(X)
        H1, S1 = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=Xt, return_S=True)
        H2, S2 = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=Xt, return_S=True)
        torch.cuda.synchronize()
        assert "chain1:" in L.describe(1), L.describe(1)
        solo = (not knobs and nnz <= 32768) or knobs.get("chain_solo") == 2
        assert ("(solo:" in L.describe(1)) == solo, L.describe(1)
        assert not L.chain_status(), "a chain barrier wait timed out"
        assert torch.equal(S1, S2) and torch.equal(H1, H2)
        X0 = L.log1p_degree().cpu().numpy() if X is None else X
        ref = O.graph_wavelet_features(g.to_scipy(), k=K, s=0.8, X0=X0, return_all=True)
        assert_parity(S1.cpu().numpy(), ref["S"], what=f"chain1 n={n} K={K} S")
        big = np.abs(ref["S"]) > 1e-3 * np.abs(ref["S"]).max()
        assert np.abs(H1.cpu().numpy()[big] - ref["H"][big]).max() <= 1e-5
    L.tune(chain=0)   # the multi-launch path gives the same result to rounding
    _, S0 = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=Xt, return_S=True)
    assert_parity(S1.cpu().numpy(), S0.cpu().numpy().astype(np.float64), what="chain1 vs multi-launch")
    L.close()


@pytest.mark.parametrize("wg", [4, 16, 64])
def test_chain1_directed_multi_worker(wg):
    """A directed graph through the one-launch chain with several workers: a worker
    that reads another need not be read by it, so each worker also waits on one
    granule of every worker that reads it (csrc/chain.hip build_chain_plan), or
    a fast worker could overwrite a granule buffer its reader has not finished
    (the reader would then wait for a tag that never comes)."""
    g = random_graph(12000, 0.0012, seed=wg, directed=True, weighted=False, self_loop_frac=0.05,
                     isolated_frac=0.05)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(chain_wg=wg)
    X = np.random.default_rng(wg).standard_normal((g.n, 1)).astype(np.float32)
    ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=X, return_all=True)
    out = {}
    for direct in (0, 1):   # staged u, or gathers straight from the granules (same sums, bitwise)
        L.tune(chain_direct=direct)
        for _ in range(3):
            H, S = wats_hip.graph_wavelet_features(L, k=16, s=0.8, X0=torch.from_numpy(X), return_S=True)
            torch.cuda.synchronize()
            assert "chain1:" in L.describe(1), L.describe(1)
            assert not L.chain_status(), "a chain wait timed out"
            assert_parity(_np(S), ref["S"], what=f"chain1 directed P={wg} direct={direct} S")
        out[direct] = _np(S)
    assert np.array_equal(out[0], out[1]), "direct gathers changed the sums"
    L.close()


@pytest.mark.parametrize("K", [16, 5])
def test_chain_solo_directed(K):
    """The one-workgroup chain (cheb_chain_solo_kernel) on a directed graph with self
    loops and isolated nodes: active rows with no entries, isolated-flag rows,
    long rows summed by lane teams;
    against the oracle, bitwise repeatable, and against the multi-worker chain
    and the multi-launch path to rounding."""
    g = random_graph(6000, 0.0015, seed=K, directed=True, weighted=False, self_loop_frac=0.05, isolated_frac=0.05)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(chain_solo=2)   # ~54 k entries: past the auto limit
    X = np.random.default_rng(K).standard_normal((g.n, 1)).astype(np.float32)
    ref = O.graph_wavelet_features(g.to_scipy(), k=K, s=0.8, X0=X, return_all=True)
    H1, S1 = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=torch.from_numpy(X), return_S=True)
    H2, S2 = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=torch.from_numpy(X), return_S=True)
    torch.cuda.synchronize()
    assert "(solo:" in L.describe(1), L.describe(1)
    assert torch.equal(S1, S2) and torch.equal(H1, H2)
    assert_parity(_np(S1), ref["S"], what=f"chain solo directed K={K} S")
    big = np.abs(ref["S"]) > 1e-3 * np.abs(ref["S"]).max()
    assert np.abs(_np(H1)[big] - ref["H"][big]).max() <= 1e-5
    for knobs in ({"chain_solo": 0, "chain_wg": 4}, {"chain": 0}):
        L.tune(**knobs)
        _, S0 = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=torch.from_numpy(X), return_S=True)
        torch.cuda.synchronize()
        assert "(solo:" not in L.describe(1)
        assert_parity(_np(S1), _np(S0).astype(np.float64), what=f"chain solo vs {knobs}")
    L.close()


def test_chain1_timeout_falls_back():
    """A worker that never publishes (fault injection: tuning key chain_fault)
    makes the one-launch chain give up its waits (the stand-in for a GPU shared
    with another process, where not every worker becomes resident): that
    launch's dependent S / H rows come out NaN, never silently wrong.  The
    Python drop-in detects it with an event wait (no device sync), reruns the
    call on the multi-launch path and returns oracle-equal features; the handle
    stays on that path (counted in describe) until the next tune.  Through the
    C ABI alone the failed launch returns WG_OK (asynchronous), the next call
    reports WG_ERR_TIMEOUT (-5) without launching, and the one after runs the
    multi-launch path."""
    g = rmat_graph(19717, 88648, seed=3)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(chain_wg=16)
    H0, S0 = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)
    torch.cuda.synchronize()
    assert "chain1:" in L.describe(1) and torch.isfinite(S0).all()
    ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=L.log1p_degree().cpu().numpy(), return_all=True)
    L.tune(chain_fault=3)
    H1, S1 = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)   # no exception
    torch.cuda.synchronize()
    assert torch.isfinite(S1).all() and torch.isfinite(H1).all()
    assert_parity(_np(S1), ref["S"], what="chain timeout -> multi-launch S")
    assert "chain1 timeouts=1 (off" in L.describe(1), L.describe(1)
    H2, S2 = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)   # stays on the multi-launch path
    torch.cuda.synchronize()
    assert torch.equal(S1, S2) and torch.equal(H1, H2)
    # the C ABI alone (a tune gives the one-launch chain another chance)
    L.tune(chain_fault=3)
    lib = wats_hip._lib.load()
    X = L.log1p_degree()
    S = torch.zeros(L.n, 1, device=X.device)
    H = torch.zeros(L.n, 1, device=X.device)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.wg_wavelet_features(L.handle, X.data_ptr(), 1, 16, 0.8, S.data_ptr(), H.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.isnan(S).any() and torch.isnan(H).any()
    assert lib.wg_wavelet_features(L.handle, X.data_ptr(), 1, 16, 0.8, S.data_ptr(), H.data_ptr(), st) == -5
    assert "gave up" in lib.wg_last_error().decode()
    assert lib.wg_wavelet_features(L.handle, X.data_ptr(), 1, 16, 0.8, S.data_ptr(), H.data_ptr(), st) == 0
    torch.cuda.synchronize()
    assert torch.equal(S, S1) and torch.equal(H, H1)
    L.tune(chain_fault=0)
    H3, S3 = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)
    torch.cuda.synchronize()
    assert not L.chain_status() and "timeouts" not in L.describe(1).split("chain1:")[0]
    assert torch.equal(S3, S0) and torch.equal(H3, H0)
    L.close()


def test_chain1_timeout_in_replayed_graph():
    """The one-launch chain captured into the handle's own hipGraph (tuning key
    graph=1: same X0 / S / H three calls in a row) and replayed with a fault:
    wg_chain_status waits for the replay itself (an event recorded after the
    graph launch), reports the timeout, and the handle's captured chain is
    dropped, so the next call with the same buffers runs the multi-launch path
    instead of replaying the faulted one-launch chain."""
    g = rmat_graph(19717, 88648, seed=3)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(chain_wg=16, graph=1)
    lib = wats_hip._lib.load()
    X = L.log1p_degree()
    ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=X.cpu().numpy(), return_all=True)
    S = torch.zeros(L.n, 1, device=X.device)
    H = torch.zeros(L.n, 1, device=X.device)
    st = torch.cuda.current_stream().cuda_stream
    call = lambda: lib.wg_wavelet_features(L.handle, X.data_ptr(), 1, 16, 0.8, S.data_ptr(), H.data_ptr(), st)
    for _ in range(4):   # eager, eager, captured + replayed, replayed: no fault
        assert call() == 0
    torch.cuda.synchronize()
    assert "chain1:" in L.describe(1)
    assert_parity(_np(S), ref["S"], what="replayed one-launch chain S")
    L.tune(chain_wg=16, graph=1, chain_fault=3)
    for _ in range(3):   # eager, eager, captured + replayed: every launch gives up a wait (0.5 s each)
        assert call() == 0
    t = ctypes.c_int32(0)
    assert lib.wg_chain_status(L.handle, ctypes.byref(t)) == 0 and t.value == 1
    assert torch.isnan(S).any()
    S.zero_()
    H.zero_()
    assert call() == 0    # same buffers: the captured (faulted) chain must not be replayed
    torch.cuda.synchronize()
    assert torch.isfinite(S).all() and torch.isfinite(H).all()
    assert_parity(_np(S), ref["S"], what="after a replayed timeout: multi-launch S")
    for _ in range(3):    # the multi-launch chain captured and replayed with the same buffers
        assert call() == 0
    torch.cuda.synchronize()
    assert lib.wg_chain_status(L.handle, ctypes.byref(t)) == 0 and t.value == 0
    assert_parity(_np(S), ref["S"], what="multi-launch chain replayed S")
    # the Python drop-in with results dropped between calls (the caching allocator hands back the
    # same S / H blocks, so the handle captures): every call's features are finite and oracle-equal
    L.tune(chain_wg=16, graph=1, chain_fault=3)
    for _ in range(4):
        H1, S1 = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)
        torch.cuda.synchronize()
        assert torch.isfinite(S1).all() and torch.isfinite(H1).all()
        assert_parity(_np(S1), ref["S"], what="drop-in after a timeout")
        del H1, S1
    L.close()


def test_chain1_workers_within_residency():
    """The one-launch chain's plan never asks for more workers than can be
    resident at once (one per CU, and what the occupancy query admits for its
    LDS): a graph that would need more takes the multi-launch path."""
    g = rmat_graph(19717, 88648, seed=5)
    L = NormalizedLaplacian.from_graph(g)
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    L.tune(chain_wg=n_cu * 2)   # more workers than CUs: refused, the multi-launch path runs
    H, S = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)
    torch.cuda.synchronize()
    assert "chain1:" not in L.describe(1)
    ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=L.log1p_degree().cpu().numpy(), return_all=True)
    assert_parity(_np(S), ref["S"], what="chain over-residency -> multi-launch S")
    L.tune(chain_wg=0)
    wats_hip.graph_wavelet_features(L, k=16, s=0.8)
    torch.cuda.synchronize()
    assert "chain1:" in L.describe(1)
    P = int(L.describe(1).split("chain1: one launch per chain, ")[1].split(" workers")[0])
    assert P <= n_cu
    L.close()


def test_chain1_golden_pubmed():
    """The reference's own PubMed-size K=16 vectors (tests/golden), through the one-launch chain."""
    d = load_golden("pubmed_rmat_k16")
    A = golden_csr(d)
    L = NormalizedLaplacian.from_scipy(A)
    H, S = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)
    torch.cuda.synchronize()
    assert "chain1:" in L.describe(1)
    assert_parity(S.cpu().numpy(), d["S"], what="chain1 golden pubmed S")
    L.close()


@pytest.mark.parametrize("team", [1, 0])
def test_split_row_counters_reset(team):
    """Long rows split over several waves (team kernel) or workgroups (step
    kernel) meet through per-row arrival counters; the arrival that completes a
    row resets its counter, so every launch starts from 0 and no combine depends
    on earlier launches (the old monotonic int32 counters and
    their `% parts` test broke at the 2^31 wrap for part counts that do not
    divide 2^32).  Rows with non-power-of-two part counts, 12 chains = 192
    launches: S bitwise equal every time, no counter left non-zero, oracle-equal."""
    g = rmat_graph(30000, 600000, seed=11)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(team=team)
    if not team:   # the workgroup kernel: rows over 384 entries split into chunks of 192
        L.tune(block_iter=16, chunk_iter=8)
    X = np.random.default_rng(7).standard_normal((g.n, 40)).astype(np.float32)
    Xt = torch.from_numpy(X)
    first = None
    for _ in range(12):
        _, S = wats_hip.graph_wavelet_features(L, k=16, s=0.8, X0=Xt, return_S=True)
        torch.cuda.synchronize()
        if first is None:
            first = S.clone()
        else:
            assert torch.equal(S, first)
    d = L.describe(40)
    if team:
        line = [ln for ln in d.splitlines() if ln.startswith("team:")][0]
        kv = dict(t.split("=") for t in line.split()[1:])
        assert int(kv["long_rows"]) > 0 and int(kv["npot_rows"]) > 0, line
    else:
        line = [ln for ln in d.splitlines() if ln.startswith("split rows:")][0]
    assert line.endswith("pending_arrivals=0"), line
    ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=X, return_all=True)
    assert_parity(_np(first), ref["S"], what=f"split rows team={team} S")
    L.close()


@pytest.mark.parametrize("K", [1, 2, 3, 16])
def test_fold_first_launch(K):
    """No permute-in pass (tuning key fold, default on): the chain's first
    team-kernel launch gathers the caller's X0 through caller-row ids scaled by
    dinv on the fly, reads its own X0 rows through perm, writes the internal X0
    for the later steps and finishes the closed-form rows.  u_0 is rounded as
    the pass rounded it, so S / H equal the permute-in path's bit for bit
    (K = 1: the final step is the first launch; K = 2 / 3: the implicit b_K
    branches), and both equal the oracle -- on the arxiv-size graph (45 % closed
    rows) and with no closed rows."""
    g = named_graph("ogbn-arxiv")
    for gg in (g, connect_isolated(g, seed=7)):
        X = np.random.default_rng(K).standard_normal((gg.n, 40)).astype(np.float32)
        L = NormalizedLaplacian.from_graph(gg)
        out = {}
        for fold in (1, 0):
            L.tune(fold=fold)
            H, S = wats_hip.graph_wavelet_features(L, k=K, X0=torch.from_numpy(X), return_S=True)
            torch.cuda.synchronize()
            out[fold] = (_np(S), _np(H))
        assert "team:" in L.describe(40)
        assert np.array_equal(out[1][0], out[0][0]) and np.array_equal(out[1][1], out[0][1]), "fold changed S / H"
        ref = O.graph_wavelet_features(gg.to_scipy(), k=K, s=0.8, X0=X, return_all=True)
        assert_parity(out[1][0], ref["S"], what=f"fold K={K} S")
        assert_parity(out[1][1], ref["H"], what=f"fold K={K} H")
        L.close()


def test_product_form_key_removed():
    """The opt-in product form (round 5, tuning key prod) missed the element-wise guard (2.0e-4 at K = 16
    on the connected graph, r05 s8) and left the library in round 6: the key is refused, and the
    Clenshaw chain is the only heat-sum path."""
    g = rmat_graph(2000, 20000, seed=1)
    L = NormalizedLaplacian.from_graph(g)
    with pytest.raises(Exception):
        L.tune(prod=1)
    L.close()
