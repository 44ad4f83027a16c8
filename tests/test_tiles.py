"""The hybrid step (csrc/tiles.hip): dense (64-row, 32-column) blocks of an
unweighted graph summed on the matrix cores (three exact bf16 pieces of u per
block, float32 MFMA sums added in float64), the tail entries by the step
kernel's phase 2.  Checked against the oracle (reference calibration/WATS.py:29-74)
and against the all-gather chain (tiles = 0) on the same inputs."""
import numpy as np
import pytest
import torch

from conftest import assert_parity
from oracle import wats_oracle as O

pytestmark = pytest.mark.gpu

import wats_hip  # noqa: E402
from wats_hip import NormalizedLaplacian  # noqa: E402
from wats_hip.graphgen import connect_isolated, random_graph, rmat_graph  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _np(t):
    return t.detach().cpu().numpy()


def _run(L, X, k, **knobs):
    L.tune(**knobs)
    return wats_hip.graph_wavelet_features(L, k=k, X0=torch.from_numpy(X), return_S=True)


def _forms(describe):
    """The hybrid step's launches per form since the last tune ('hybrid forms:' line of describe)."""
    line = [x for x in describe.splitlines() if x.startswith("hybrid forms:")]
    assert line, describe
    return {k: int(v) for k, v in (t.split("=") for t in line[-1].split(":", 1)[1].split())}


def _close(a, b, what, tol=2e-6):
    a, b = _np(a).astype(np.float64), _np(b).astype(np.float64)
    scale = np.max(np.abs(b), axis=0) + 1e-30
    err = np.max(np.abs(a - b), axis=0) / scale
    assert np.all(err <= tol), f"{what}: hybrid vs gather max norm-wise err {err.max():.3e}"


@pytest.mark.parametrize("F", [16, 41, 48, 64, 32])
@pytest.mark.parametrize("k", [1, 2, 3, 16])
def test_tiles_vs_oracle_and_gather(F, k):
    """Every dense-block threshold / split shape against the oracle and the
    all-gather chain: tile_th 1 (every touched block dense), 8, 64; tile_max 1
    and 3 (long row blocks over many slots, combined in order); 64- and 128-row
    blocks, one or two 16-row groups per wave, or waves owning one 16-column block
    for four row groups (tile_rg = 4); the 32x32x16 MFMA shape (tile_mfma = 32,
    widths 48 / 64; narrower widths keep the 16x16x32 kernel); the first step
    gathers u_0 = X0 * dinv value-free (K = 1: the only step); the tail entries on
    the independent-wave kernel (csrc/team.hip; hyb_iter 8: long tails as part
    waves) and on the workgroup kernel (team = 0)."""
    g = rmat_graph(4000, 120000, seed=F + k)
    A = g.to_scipy()
    X = np.random.default_rng(F * 31 + k).standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=k, s=0.8, X0=X, return_all=True)
    L = NormalizedLaplacian.from_graph(g)
    H0, S0 = _run(L, X, k, tiles=0)
    for knobs in (dict(tile_th=64, tile_max=128, tile_rows=128, tile_rg=2), dict(tile_th=8, tile_max=3, tile_rows=64),
                  dict(tile_th=1, tile_max=1, tile_rows=128, tile_rg=1), dict(tile_th=16, tile_max=5, tile_rows=128, tile_rg=4),
                  dict(tile_th=1, tile_max=1, tile_rows=128, tile_mfma=32),
                  dict(tile_th=16, tile_max=5, tile_rows=128, tile_mfma=32),
                  dict(tile_th=16, tile_max=5, tile_rows=128, team_iter=8, hyb_iter=8),
                  dict(tile_th=8, tile_max=3, tile_rows=64, team=0, team_iter=96)):
        H1, S1 = _run(L, X, k, tiles=1, **knobs)
        assert "tiles:" in L.describe(F), f"hybrid step not planned: {L.describe(F)}"
        assert_parity(_np(S1), ref["S"], what=f"F={F} K={k} {knobs} S")
        assert_parity(_np(H1), ref["H"], what=f"F={F} K={k} {knobs} H")
        _close(S1, S0, f"F={F} K={k} {knobs} S")


def test_tiles_isolated_rows_and_no_closed_form():
    """Closed-form rows (never gathered) next to dense hubs, and the same graph with
    every isolated node attached (no closed-form rows: all rows in the chain)."""
    g = rmat_graph(6000, 150000, seed=5)
    for gg in (g, connect_isolated(g, seed=1)):
        A = gg.to_scipy()
        X = np.random.default_rng(7).standard_normal((gg.n, 48)).astype(np.float32)
        ref = O.graph_wavelet_features(A, k=8, s=0.8, X0=X, return_all=True)
        L = NormalizedLaplacian.from_graph(gg)
        H0, S0 = _run(L, X, 8, tiles=0)
        H1, S1 = _run(L, X, 8, tiles=1, tile_th=16)
        assert "tiles:" in L.describe(48)
        assert_parity(_np(S1), ref["S"], what="S")
        assert_parity(_np(H1), ref["H"], what="H")
        _close(S1, S0, "S")


def test_tiles_with_signal_tiles():
    """tile_f splits the step kernel's launch into column tiles (here 16 of the 48
    columns each) while the dense blocks run over all columns at once: every
    tile's tail sum meets its own columns of the blocks' sums."""
    g = rmat_graph(4000, 120000, seed=13)
    A = g.to_scipy()
    X = np.random.default_rng(3).standard_normal((g.n, 48)).astype(np.float32)
    ref = O.graph_wavelet_features(A, k=6, s=0.8, X0=X, return_all=True)
    L = NormalizedLaplacian.from_graph(g)
    H1, S1 = _run(L, X, 6, tiles=1, tile_th=8, tile_f=16)
    assert "tiles:" in L.describe(48)
    assert_parity(_np(S1), ref["S"], what="tile_f=16 S")
    assert_parity(_np(H1), ref["H"], what="tile_f=16 H")


@pytest.mark.parametrize("k", [1, 3, 16])
@pytest.mark.parametrize("F", [48, 16])
def test_tiles_tail_beside_blocks(F, k):
    """hyb_conc: the tail's row sums on a second stream beside the dense blocks and
    one epilogue pass after the join (csrc/step.hip hybrid_epilogue_kernel) give the
    same S and H as the sequential hybrid step, bit for bit (the same float64 sums
    in the same order), with and without closed-form rows and long tails split over
    part waves (hyb_iter 8); and the oracle's."""
    g = rmat_graph(6000, 150000, seed=F + k)
    for gg in (g, connect_isolated(g, seed=2)):
        X = np.random.default_rng(F + 7 * k).standard_normal((gg.n, F)).astype(np.float32)
        ref = O.graph_wavelet_features(gg.to_scipy(), k=k, s=0.8, X0=X, return_all=True)
        L = NormalizedLaplacian.from_graph(gg)
        for knobs in (dict(tile_th=16, tile_max=5, tile_rows=128), dict(tile_th=8, tile_max=3, tile_rows=64, team_iter=8, hyb_iter=8)):
            H0, S0 = _run(L, X, k, tiles=1, hyb_conc=0, **knobs)
            H1, S1 = _run(L, X, k, tiles=1, hyb_conc=2, **knobs)
            H2, S2 = _run(L, X, k, tiles=1, hyb_conc=2, **knobs)
            torch.cuda.synchronize()
            d = L.describe(F)
            assert "tiles:" in d
            # 128-row blocks: the one-launch form (hybrid_fused_kernel); 64-row blocks: two streams
            form = "fused" if knobs["tile_rows"] == 128 else "two_stream"
            assert _forms(d)[form] > 0 and _forms(d)["sequential"] == 0, d
            assert torch.equal(S0, S1) and torch.equal(H0, H1), f"F={F} K={k} {knobs}: concurrent tail differs"
            assert torch.equal(S1, S2) and torch.equal(H1, H2)
            assert_parity(_np(S1), ref["S"], what=f"F={F} K={k} {knobs} S")
        L.close()


def test_tiles_deterministic():
    g = rmat_graph(4000, 120000, seed=9)
    X = np.random.default_rng(1).standard_normal((g.n, 48)).astype(np.float32)
    L = NormalizedLaplacian.from_graph(g)
    _, S1 = _run(L, X, 16, tiles=1, tile_th=8, tile_max=2)
    _, S2 = _run(L, X, 16)
    assert torch.equal(S1, S2), "the hybrid chain must be bitwise reproducible"


def test_tiles_not_taken_for_weighted_or_narrow():
    """Weighted graphs (values read) and widths that are not a multiple of 16 keep
    the gather kernel."""
    g = random_graph(2000, 0.02, seed=3, directed=False, weighted=True)
    X = np.random.default_rng(2).standard_normal((g.n, 48)).astype(np.float32)
    L = NormalizedLaplacian.from_graph(g)
    _run(L, X, 4, tiles=1)
    assert "tiles:" not in L.describe(48)
    g = rmat_graph(4000, 120000, seed=2)
    X = np.random.default_rng(2).standard_normal((g.n, 8)).astype(np.float32)
    L = NormalizedLaplacian.from_graph(g)
    _run(L, X, 4, tiles=1)
    assert "tiles:" not in L.describe(8)


@pytest.mark.parametrize("F,tiles", [(48, 0), (48, 1), (6, 0)])
def test_clenshaw_step_abi(F, tiles):
    """wg_clenshaw_step (one step of the chain through the C ABI) against the
    per-step API: out = ck x0 + cacc (L_hat b1) - b2, valued (flags 0) on any
    graph, and value-free on u = b dinv (UIN | UPREV | UOUT) on an unweighted one
    -- the hybrid step when tiles = 1."""
    from wats_hip import _lib
    from wats_hip._lib import check, ptr
    g = rmat_graph(4000, 120000, seed=11)
    L = NormalizedLaplacian.from_graph(g)
    L.tune(tiles=tiles, tile_th=8)
    dev = L.device
    rng = np.random.default_rng(5)
    b1, b2, x0 = (torch.from_numpy(rng.standard_normal((g.n, F)).astype(np.float32)).to(dev) for _ in range(3))
    T1 = torch.empty_like(b1)
    L.step(1, b1, None, T1)                      # T_1 = L_hat b1 (internal order, like every vector here)
    ck, cacc = 0.3, 2.0
    ref = (ck * x0.double() + cacc * T1.double() - b2.double())
    lib = _lib.load()
    st = torch.cuda.current_stream(dev).cuda_stream
    out = torch.empty_like(b1)
    check(lib.wg_clenshaw_step(L.handle, F, ptr(b1), ptr(b2), ptr(x0), ptr(out), ck, cacc, 0, st), "clenshaw_step")
    torch.cuda.synchronize()
    _close(out, ref.float(), f"valued F={F}", tol=1e-6)
    # value-free: b1, b2 given as u = b * dinv; out comes back as u
    iperm_deg = torch.from_numpy(np.diff(g.indptr).astype(np.float64))   # column degrees: the graph is symmetric
    deg_int = L.permute(iperm_deg.float().reshape(-1, 1).to(dev), to_internal=True).double()
    dinv = torch.where(deg_int > 0, 1.0 / torch.sqrt(deg_int), torch.ones_like(deg_int))
    u1, u2 = (b1.double() * dinv).float(), (b2.double() * dinv).float()
    outu = torch.empty_like(b1)
    check(lib.wg_clenshaw_step(L.handle, F, ptr(u1), ptr(u2), ptr(x0), ptr(outu), ck, cacc, 1 | 2 | 4, st),
          "clenshaw_step u")
    torch.cuda.synchronize()
    _close((outu.double() / dinv).float(), ref.float(), f"value-free F={F} tiles={tiles}", tol=2e-6)
    if tiles:
        assert "tiles:" in L.describe(F)


def test_tiles_duplicate_entries_keep_the_gather_kernel():
    """A CSR with a repeated entry (outside the canonical-input precondition) cannot be
    a 0/1 row mask: the hybrid step declines and the gather kernel runs, unchanged."""
    g = rmat_graph(3000, 90000, seed=4)
    indptr, indices = g.indptr.copy(), g.indices.copy()
    r = int(np.argmax(np.diff(indptr)))                 # repeat the first entry of the longest row
    pos = indptr[r]
    indices = np.insert(indices, pos, indices[pos])
    indptr[r + 1:] += 1
    X = np.random.default_rng(8).standard_normal((g.n, 48)).astype(np.float32)
    L = NormalizedLaplacian.from_csr(indptr, indices, None, n=g.n)
    H0, S0 = _run(L, X, 6, tiles=0)
    H1, S1 = _run(L, X, 6, tiles=1, tile_th=4)
    assert "tiles:" not in L.describe(48)
    assert torch.equal(S0, S1) and torch.equal(H0, H1)


@pytest.mark.parametrize("F", [48, 64])
def test_tiles_auto_items_default_form(F):
    """The shipped defaults on a graph large enough for long fused items (~n_plan / 310 blocks per item,
    past the former 256 cap): at width 48 the step runs in the fused form with its own item list, at
    width 64 (32x32x16 MFMA, never fused) the sequential step keeps the sequential rule's 128-block items
    (one plan serves every width).  Both against the oracle and the forced sequential step
    (hyb_conc = 0); with an explicit tile_max the default form (fused at 48, two streams at 64: fewer
    items than two per CU) and the sequential one walk the same items and agree bit for bit."""
    g = rmat_graph(150000, 3_600_000, seed=21)
    X = np.random.default_rng(F).standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(g.to_scipy(), k=4, s=0.8, X0=X, return_all=True)
    L = NormalizedLaplacian.from_graph(g)
    H1, S1 = _run(L, X, 4, tiles=1)                      # defaults: tile_max auto, hyb_conc auto
    d1 = L.describe(F)
    items = d1.split("tiles:")[1]
    n_seq = int(items.split(" items,")[0].split()[-1])
    n_fus = int(items.split("fused launch: ")[1].split(" items")[0])
    n_act = int(d1.split("active_rows=")[1].split()[0])
    assert n_act // 310 > 256, d1
    if F == 48:
        assert _forms(d1) == {"fused": 4, "two_stream": 0, "sequential": 0}, d1
        assert n_fus < n_seq, d1                         # longer items in the fused launch
    else:   # not the fused shape: sequential, or two streams when the items leave the GPU half idle
        assert _forms(d1)["fused"] == 0 and _forms(d1)["two_stream"] + _forms(d1)["sequential"] == 4, d1
    H0, S0 = _run(L, X, 4, tiles=1, hyb_conc=0)
    d0 = L.describe(F)
    assert _forms(d0) == {"fused": 0, "two_stream": 0, "sequential": 4}, d0
    assert_parity(_np(S1), ref["S"], what=f"auto items F={F} S")
    assert_parity(_np(H1), ref["H"], what=f"auto items F={F} H")
    _close(S1, S0, f"auto items F={F} vs sequential")
    H2, S2 = _run(L, X, 4, tiles=1, tile_max=1024, hyb_conc=1)
    if F == 48:
        assert _forms(L.describe(F))["fused"] == 4
    H3, S3 = _run(L, X, 4, tiles=1, tile_max=1024, hyb_conc=0)
    torch.cuda.synchronize()
    assert torch.equal(S2, S3) and torch.equal(H2, H3), f"F={F}: default form vs hyb_conc=0 differ bitwise"
    assert_parity(_np(S2), ref["S"], what=f"tile_max=1024 F={F} S")
    L.close()
