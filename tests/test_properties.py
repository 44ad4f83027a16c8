"""Property tests: random small graphs -- directed or
not, weighted or not, with self loops and isolated nodes -- through the HIP
path against the oracle, with hypothesis drawing the shapes.  Each example
also runs the row-sharded chain's planning on the same graph (CPU, world 1).

The tolerance is the one of every parity test (tests/conftest.py): max|d| /
max|ref| <= 1e-5 per column."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from conftest import assert_parity

from oracle import wats_oracle as O

import wats_hip
from wats_hip.graphgen import random_graph

graphs = st.fixed_dictionaries({
    "n": st.integers(1, 80),
    "p": st.floats(0.0, 0.25),
    "directed": st.booleans(),
    "weighted": st.booleans(),
    "self_loop_frac": st.sampled_from([0.0, 0.1, 0.5]),
    "isolated_frac": st.sampled_from([0.0, 0.1, 0.4]),
    "seed": st.integers(0, 2 ** 31 - 1),
})


@pytest.mark.gpu
@settings(max_examples=60, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
@given(spec=graphs, F=st.sampled_from([1, 2, 3, 5, 8, 13]), K=st.integers(0, 7),
       s=st.sampled_from([0.8, 0.3, 1.5]))
def test_random_graphs_match_oracle(spec, F, K, s):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = random_graph(**spec)
    A = g.to_scipy()
    rng = np.random.default_rng(spec["seed"] % 1000)
    X = rng.standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=K, s=s, X0=X, return_all=True)
    L = wats_hip.NormalizedLaplacian.from_scipy(A)
    H, S = wats_hip.graph_wavelet_features(L, k=K, s=s, X0=torch.from_numpy(X), return_S=True)
    what = f"{spec} F={F} K={K} s={s}"
    assert_parity(S.cpu().numpy(), ref["S"], what=what + " S")
    # H = S / (|S|_1 + 1e-8) is ill-conditioned where a row's S cancels; compare it where |S|_1 is not tiny
    Sr = np.abs(ref["S"]).sum(axis=1)
    ok = Sr > 1e-3 * max(Sr.max(), 1e-30)
    if ok.any():
        assert np.abs(H.cpu().numpy()[ok] - ref["H"][ok]).max() <= 1e-5, what + " H"


@pytest.mark.gpu
@settings(max_examples=25, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
@given(spec=graphs, K=st.integers(1, 6), lds=st.sampled_from([1, 2, 4]))
def test_random_graphs_lds_kernels(spec, K, lds):
    """The F = 1 LDS kernels (teams, windows, hub teams) on random unweighted
    graphs, forced on, against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    spec = dict(spec, weighted=False)
    g = random_graph(**spec)
    A = g.to_scipy()
    rng = np.random.default_rng(spec["seed"] % 997)
    X = rng.standard_normal((g.n, 1)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=K, s=0.8, X0=X, return_all=True)
    L = wats_hip.NormalizedLaplacian.from_scipy(A)
    L.tune(lds=lds, lds_cb=64)   # small blocks / hub: several blocks and a tail even on tiny graphs
    _, S = wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=torch.from_numpy(X), return_S=True)
    assert_parity(S.cpu().numpy(), ref["S"], what=f"{spec} lds={lds} K={K} S")


# ------------------------------------------------------------ size-independent properties at the named sizes
def _colwise_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().amax(dim=0) / (b.abs().amax(dim=0) + 1e-30)).max().item()


def _features(L, X, k):
    H, S = wats_hip.graph_wavelet_features(L, k=k, s=0.8, X0=X, return_S=True)
    torch.cuda.synchronize()
    return H, S


@pytest.mark.gpu
def test_headline_linearity_relabelling_determinism():
    """The metric's config (ogbn-arxiv-size R-MAT, K=16, F=40: the team kernel with the folded first launch):
    S is linear in X0 (S(X + 2Y) = S(X) + 2 S(Y)), equivariant under a relabelling of the nodes
    (S(P A P^T, P X) = P S(A, X): a different internal order, so a different summation order), and bitwise
    reproducible -- column-wise within the parity tolerance, at the full size, without the oracle."""
    from wats_hip import NormalizedLaplacian
    from wats_hip.graphgen import CSRGraph, named_graph
    g = named_graph("ogbn-arxiv")
    n = g.n
    gen = torch.Generator().manual_seed(7)
    X = torch.randn(n, 40, generator=gen).cuda()
    Y = torch.randn(n, 40, generator=gen).cuda()
    L = NormalizedLaplacian.from_graph(g)
    _, SX = _features(L, X, 16)
    _, SY = _features(L, Y, 16)
    _, SZ = _features(L, X + 2 * Y, 16)
    assert "team:" in L.describe(40)
    assert _colwise_err(SZ, SX + 2 * SY) <= 1e-5
    _, SX2 = _features(L, X, 16)
    assert torch.equal(SX, SX2), "the chain must be bitwise reproducible"
    L.close()
    # relabel: new id of node v is p[v]
    p = np.random.default_rng(3).permutation(n)
    A = g.to_scipy().tocoo()
    import scipy.sparse as sp
    B = sp.csr_matrix((A.data, (p[A.row], p[A.col])), shape=A.shape)
    B.sort_indices()
    gp = CSRGraph(n, B.indptr.astype(np.int64), B.indices.astype(np.int32), None)
    Lp = NormalizedLaplacian.from_graph(gp)
    pt = torch.from_numpy(p).cuda()
    Xp = torch.empty_like(X)
    Xp[pt] = X
    Hp, Sp = _features(Lp, Xp, 16)
    assert _colwise_err(Sp[pt], SX) <= 1e-5
    Lp.close()


@pytest.mark.gpu
def test_reddit_f41_linearity_and_determinism():
    """Reddit-size K=16 F=41 (the fused hybrid step: dense blocks on the matrix cores, the tail's waves in the
    same launch): S linear in X0 and bitwise reproducible, at the full size."""
    from wats_hip import NormalizedLaplacian
    from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device
    n, nnz, _, _ = NAMED_CONFIGS["reddit"]
    ip, ix = rmat_graph_device(n, nnz, seed=0, device="cuda")
    L = NormalizedLaplacian(n, ip, ix)
    del ip, ix
    gen = torch.Generator().manual_seed(11)
    X = torch.randn(n, 41, generator=gen).cuda()
    Y = torch.randn(n, 41, generator=gen).cuda()
    _, SX = _features(L, X, 16)
    _, SY = _features(L, Y, 16)
    _, SZ = _features(L, X - 0.5 * Y, 16)
    d = L.describe(48)
    assert "tiles:" in d and "hybrid forms: fused=" in d, d
    assert _colwise_err(SZ, SX - 0.5 * SY) <= 1e-5
    _, SX2 = _features(L, X, 16)
    assert torch.equal(SX, SX2)
    L.close()
