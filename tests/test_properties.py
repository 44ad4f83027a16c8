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
