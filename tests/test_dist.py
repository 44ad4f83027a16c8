"""Row-sharded path: partition, halo plan, column-degree
all-reduce and the per-step halo exchange.

CPU tests run world_size 2 and 3 with the gloo backend and drive the chain with
the oracle's float64 local mat-vec, so they check the index plumbing against
the single-process oracle.  The GPU test runs the HIP sharded chain with
several ranks sharing one GPU (host-staged exchange over gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, assert_parity

from oracle import wats_oracle as O
from wats_hip.dist import build_halo_plan, global_column_degree, halo_exchange, partition_rows
from wats_hip.graphgen import random_graph, rmat_graph


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _graph(kind):
    if kind == "rmat":
        return rmat_graph(1500, 12000, seed=5)
    return random_graph(400, 0.02, seed=3, directed=True, weighted=True, self_loop_frac=0.1, isolated_frac=0.05)


def test_partition_rows_balanced():
    g = rmat_graph(5000, 60000, seed=1)
    for world in (1, 2, 3, 8):
        b = partition_rows(g.indptr, world)
        assert b[0] == 0 and b[-1] == g.n and np.all(np.diff(b) >= 0) and len(b) == world + 1
        w = np.diff(g.indptr[b]) + np.diff(b)
        assert w.max() <= (g.nnz + g.n) / world + np.diff(g.indptr).max() + 1


def _cpu_worker(rank, world, port, kind, K, F, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _graph(kind)
        A = g.to_scipy()
        bounds = partition_rows(g.indptr, world)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        lo, hi = g.indptr[r0], g.indptr[r1]
        indptr_l = g.indptr[r0:r1 + 1] - lo
        cols_g = g.indices[lo:hi]
        vals_l = None if g.values is None else g.values[lo:hi]
        # rmat: the halo groups in descending global degree (what ShardedWavelet passes)
        col_degree = np.bincount(g.indices, minlength=g.n) if kind == "rmat" else None
        plan = build_halo_plan(indptr_l, cols_g, bounds, None, col_degree=col_degree)
        assert len(plan.recv_counts) == len(plan.send_counts) == world
        owner = np.searchsorted(bounds, plan.halo_global, side="right") - 1
        assert np.all(np.diff(owner) >= 0), "halo not grouped by owner"
        assert np.array_equal(np.bincount(owner, minlength=world), plan.recv_counts)
        if col_degree is not None:
            for peer in range(world):
                dq = col_degree[plan.halo_global[owner == peer]]
                assert np.all(np.diff(dq) <= 0), "halo group not in descending degree"
        # partial column degrees of this shard (the GPU path does this with wg_column_degree)
        cs = np.zeros(g.n)
        dg = np.zeros(g.n)
        v = np.ones(hi - lo) if vals_l is None else vals_l.astype(np.float64)
        np.add.at(cs, cols_g, v)
        rows_g = np.repeat(np.arange(r0, r1), np.diff(indptr_l))
        np.add.at(dg, rows_g[rows_g == cols_g], v[rows_g == cols_g])
        w_cols = global_column_degree(torch.from_numpy(cs), torch.from_numpy(dg), plan, None).numpy()
        # oracle column degree for the same columns
        full_w = (np.asarray(A.sum(axis=0)).ravel().astype(np.float32) - A.diagonal().astype(np.float32))
        ids = np.concatenate([np.arange(r0, r1), plan.halo_global])
        w_ok = np.allclose(w_cols, full_w[ids], rtol=1e-6, atol=0)
        # local block of the oracle L_hat with columns renumbered [own | halo]
        Lg = O.rescaled_laplacian(A)[r0:r1].tocoo()
        col_map = np.full(g.n, -1, np.int64)
        col_map[r0:r1] = np.arange(r1 - r0)
        col_map[plan.halo_global] = (r1 - r0) + np.arange(plan.n_halo)
        assert np.all(col_map[Lg.col] >= 0), "L_hat column outside [own | halo]"
        import scipy.sparse as sp
        Ll = sp.csr_matrix((Lg.data, (Lg.row, col_map[Lg.col])), shape=(r1 - r0, plan.n_cols))
        rng = np.random.default_rng(0)
        X = rng.standard_normal((g.n, F)).astype(np.float32)
        ext = torch.zeros(plan.n_cols, F, dtype=torch.float64)
        ext[: plan.n_own] = torch.from_numpy(X[r0:r1].astype(np.float64))
        send_idx = torch.from_numpy(plan.send_rows.astype(np.int64))
        sendbuf = torch.empty(len(send_idx), F, dtype=torch.float64)
        pack = lambda e, out: out.copy_(e.index_select(0, send_idx))
        S = ext[: plan.n_own].clone()
        prev = ext.clone()
        prevprev = None
        for k in range(1, K + 1):
            halo_exchange(prev, plan, pack, sendbuf, None)
            y = torch.from_numpy(Ll @ prev.numpy())
            t = y if k == 1 else 2 * y - prevprev[: plan.n_own]
            S += np.exp(-0.8 * k) * t
            nxt = torch.zeros_like(prev)
            nxt[: plan.n_own] = t
            prevprev, prev = prev, nxt
        ref = O.graph_wavelet_features(A, k=K, s=0.8, X0=X, return_all=True)["S"][r0:r1]
        q.put((rank, w_ok, float(np.max(np.abs(S.numpy() - ref)) / max(1e-30, np.max(np.abs(ref)))),
               plan.stats))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "rmat"), (3, "rmat"), (2, "weighted"), (3, "weighted"), (8, "rmat")])
def test_sharded_chain_cpu_gloo(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, world, port, kind, 5, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, w_ok, err, stats in res:
        assert w_ok, f"rank {rank}: column degree mismatch"
        assert err < 1e-12, f"rank {rank}: sharded chain differs from oracle ({err:.2e})"
        assert stats["n_halo"] > 0


# ------------------------------------------------------------------ GPU, ranks share one device
def _gpu_worker(rank, world, port, kind, K, F, q, lds=2, exchange="host", tiles=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wats_hip.dist import ShardedWavelet
        g = _graph(kind)
        bounds = partition_rows(g.indptr, world)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        lo, hi = g.indptr[r0], g.indptr[r1]
        sw = ShardedWavelet(g.indptr[r0:r1 + 1] - lo, g.indices[lo:hi],
                            None if g.values is None else g.values[lo:hi], g.n, bounds, exchange=exchange,
                            device="cuda:0")
        # lds 4 (hub teams) with a 256-column hub: the shard's hub mixes its own top columns
        # with every peer group's (halo groups in descending degree), the rest is gathered
        sw.L.tune(lds=lds, **({"lds_cb": 256} if lds == 4 else {}))
        # tiles = 1: the hybrid step on every shard, exchange-then-step, u_0
        # exchanged; tiles = 2: the same except rank 1, whose shard keeps the gather kernel (ADVICE
        # r2: ranks that disagree on the plan must still exchange u_0 in one format)
        hybrid = bool(tiles) and not (tiles == 2 and rank == 1)
        if tiles:
            sw.L.tune(tiles=1 if hybrid else 0, tile_th=8, tile_max=3)
        q_path = "u" if (F == 1 and sw.u_len() > 0) else "t"
        rng = np.random.default_rng(0)
        X = rng.standard_normal((g.n, F)).astype(np.float32)
        runs = 3 if exchange in ("ipc", "sdma") else 1   # native: eager, captured, replayed
        outs = [sw.wavelet_features(torch.from_numpy(X[r0:r1]), k=K, s=0.8) for _ in range(runs)]
        H, S = outs[0]
        same = all(torch.equal(o[1], S) and torch.equal(o[0], H) for o in outs)
        if exchange in ("ipc", "sdma"):
            if tiles:
                assert ("tiles:" in sw.L.describe(F + (-F) % 16)) == hybrid, sw.L.describe(F)
            assert sw.info()["exchange"] == exchange
            sw.check_exchange()
            sw.close()
        q.put((rank, S.cpu().numpy(), H.cpu().numpy(), q_path, same))
    except Exception as exc:  # noqa: BLE001 -- reported to the parent at once, not by its queue timeout
        import traceback
        q.put((rank, None, None, f"{exc!r}\n{traceback.format_exc()}", False))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,kind,F,lds,exchange,tiles", [
    (2, "rmat", 1, 2, "host", 0), (4, "rmat", 1, 2, "host", 0), (2, "rmat", 1, 0, "host", 0), (3, "rmat", 40, 2, "host", 0),
    (2, "weighted", 4, 2, "host", 0), (2, "weighted", 1, 2, "host", 0),
    (2, "rmat", 1, 2, "ipc", 0), (4, "rmat", 1, 2, "ipc", 0), (2, "rmat", 1, 0, "ipc", 0), (3, "rmat", 40, 2, "ipc", 0),
    (2, "weighted", 4, 2, "ipc", 0), (3, "weighted", 1, 2, "ipc", 0), (2, "rmat", 1, 4, "ipc", 0), (2, "rmat", 1, 4, "host", 0),
    (4, "rmat", 1, 2, "ipc", 0), (3, "rmat", 8, 2, "host", 0), (8, "rmat", 40, 2, "ipc", 0), (8, "rmat", 1, 2, "ipc", 0),
    (8, "weighted", 4, 2, "ipc", 0), (2, "rmat", 48, 2, "ipc", 1), (3, "rmat", 41, 2, "ipc", 1),
    (4, "rmat", 48, 2, "ipc", 1), (3, "rmat", 48, 2, "ipc", 2), (2, "rmat", 41, 2, "ipc", 2),
    (2, "rmat", 1, 2, "sdma", 0), (3, "rmat", 40, 2, "sdma", 0), (4, "weighted", 4, 2, "sdma", 0),
    (8, "rmat", 40, 2, "sdma", 0), (8, "rmat", 1, 2, "sdma", 0), (4, "rmat", 48, 2, "sdma", 1),
    (3, "rmat", 41, 2, "sdma", 2)])
def test_sharded_chain_gpu_multi_rank(world, kind, F, lds, exchange, tiles):
    """Several ranks on one GPU: the Python exchange over gloo host copies, or
    the native chain with the one-sided IPC exchange (ranks pull from each
    other's memory; same-device IPC stands in for xGMI peers), or with the
    packed-block copies (sdma: hipMemcpyAsync from the owners' IPC-mapped send
    buffers on a copy stream, behind the same phase flags).  tiles = 1: the
    hybrid step on every shard (dense blocks over [own | halo] columns); tiles = 2:
    on every shard but rank 1's (the ranks disagree on the plan)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    K = 8
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, kind, K, F, q, lds, exchange, tiles))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            res.append(q.get(timeout=150))
            if res[-1][1] is None:
                pytest.fail(f"rank {res[-1][0]}: {res[-1][3]}")
    finally:
        for p in procs:
            p.join(timeout=60 if len(res) == world and res[-1][1] is not None else 5)
            if p.is_alive():
                p.kill()
    res.sort(key=lambda t: t[0])
    assert all(p.exitcode == 0 for p in procs)
    g = _graph(kind)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(g.to_scipy(), k=K, s=0.8, X0=X, return_all=True)
    S = np.concatenate([r[1] for r in res])
    H = np.concatenate([r[2] for r in res])
    # F == 1 on an unweighted graph with lds on: the LDS kernel with the u halo exchange
    assert all(r[3] == ("u" if (F == 1 and kind == "rmat" and lds) else "t") for r in res)
    assert all(r[4] for r in res), "repeated calls differ (graph capture / replay)"
    assert_parity(S, ref["S"], what=f"sharded world={world} S")
    if F > 1:
        assert_parity(H, ref["H"], what=f"sharded world={world} H")
    else:  # H = S / (|S| + 1e-8) is ill-conditioned where a random signal cancels (|S| ~ 1e-8..1e-4)
        ok = np.abs(ref["S"]) > 1e-3 * np.abs(ref["S"]).max()
        assert np.abs(H[ok] - ref["H"][ok]).max() <= 1e-5


# ------------------------------------------------------------------ GPU, native chain (csrc/dist.hip)
def _native_graph(kind):
    if kind == "dense-rmat":   # avg degree ~ 80: the F = 1 LDS window kernel applies
        return rmat_graph(3000, 240000, seed=7)
    return _graph(kind)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,F,lds", [("rmat", 1, 3), ("dense-rmat", 1, 2), ("rmat", 40, 3), ("weighted", 4, 3),
                                        ("weighted", 1, 3)])
def test_native_chain_world1(kind, F, lds):
    """wg_dist_* at world 1 (its own one-rank RCCL communicator, no halo):
    eager first call, captured second, replayed after -- all equal the oracle
    and each other bit for bit."""
    from wats_hip.dist import ShardedWavelet
    g = _native_graph(kind)
    sw = ShardedWavelet(g.indptr, g.indices, g.values, g.n, np.array([0, g.n]), exchange="rccl", device="cuda:0")
    sw.L.tune(lds=lds)
    rng = np.random.default_rng(2)
    X = torch.from_numpy(rng.standard_normal((g.n, F)).astype(np.float32)).cuda()
    K = 8
    outs = [sw.wavelet_features(X, k=K, s=0.8) for _ in range(3)]
    ref = O.graph_wavelet_features(g.to_scipy(), k=K, s=0.8, X0=X.cpu().numpy(), return_all=True)
    for H, S in outs:
        assert torch.equal(S, outs[0][1]) and torch.equal(H, outs[0][0])
    S, H = outs[0][1].cpu().numpy(), outs[0][0].cpu().numpy()
    assert_parity(S, ref["S"], what=f"native world=1 {kind} F={F} S")
    ok = np.abs(ref["S"]) > 1e-3 * np.abs(ref["S"]).max(axis=0, keepdims=True) if F == 1 else np.ones_like(S, bool)
    assert np.abs(H[ok] - ref["H"][ok]).max() <= 1e-5
    sw.close()


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 2, 3, 5])
def test_native_chain_clenshaw_small_orders(K):
    """The sharded chain's Clenshaw heat sum (F > 1) at the orders whose
    first / second phases carry the implicit b_K: against the oracle and
    against the forward recurrence (clenshaw = 0)."""
    from wats_hip.dist import ShardedWavelet
    g = _native_graph("weighted")
    sw = ShardedWavelet(g.indptr, g.indices, g.values, g.n, np.array([0, g.n]), exchange="rccl", device="cuda:0")
    X = torch.from_numpy(np.random.default_rng(K).standard_normal((g.n, 6)).astype(np.float32)).cuda()
    ref = O.graph_wavelet_features(g.to_scipy(), k=K, s=0.8, X0=X.cpu().numpy(), return_all=True)
    H1, S1 = sw.wavelet_features(X, k=K, s=0.8)
    sw.L.tune(clenshaw=0)
    H0, S0 = sw.wavelet_features(X, k=K, s=0.8)
    for S, H, tag in ((S1, H1, "clenshaw"), (S0, H0, "forward")):
        assert_parity(S.cpu().numpy(), ref["S"], what=f"native K={K} {tag} S")
        assert_parity(H.cpu().numpy(), ref["H"], what=f"native K={K} {tag} H")
    sw.close()


@pytest.mark.gpu
@pytest.mark.parametrize("F,lds,graph,clen,tiles", [
    (1, 2, 1, 1, 0), (1, 0, 1, 1, 0), (8, 3, 1, 1, 0), (8, 3, 0, 1, 0), (40, 3, 1, 1, 0), (40, 3, 0, 0, 0),
    (8, 3, 1, 0, 0), (1, 0, 1, 0, 0), (12, 3, 1, 1, 0), (48, 3, 1, 1, 1), (41, 3, 0, 1, 1), (48, 3, 0, 1, 1)])
def test_native_chain_loopback_exchange(F, lds, graph, clen, tiles):
    """The native exchange with real RCCL traffic on one GPU: a one-rank shard
    whose column space is [own | halo] where the halo columns are copies of own
    rows (every entry (i, j) with j % 3 == 0 and (i + j) odd reads the copy).
    Per step the pack kernel + ncclSend/ncclRecv to self must refresh the
    copies, so the result equals the unsharded chain, with the Clenshaw or the
    forward chain (clen).  tiles = 1: the hybrid step (csrc/tiles.hip, dense blocks on the
    matrix cores) over the [own | halo] column space, exchange-then-step."""
    import ctypes
    import wats_hip
    from wats_hip import _lib
    from wats_hip._lib import check, ptr
    g = _native_graph("dense-rmat")
    n = g.n
    J = np.arange(0, n, 3)
    slot = np.full(n, -1, np.int64)
    slot[J] = np.arange(J.size)
    rows = np.repeat(np.arange(n), np.diff(g.indptr))
    cols = g.indices.astype(np.int64).copy()
    move = (slot[cols] >= 0) & ((rows + cols) % 2 == 1)
    cols[move] = n + slot[cols[move]]
    deg = np.bincount(g.indices, minlength=n).astype(np.float32)   # unweighted, symmetric, no loops: w = degree
    w_ext = np.concatenate([deg, deg[J]])
    L = wats_hip.NormalizedLaplacian(n, torch.from_numpy(g.indptr), torch.from_numpy(cols.astype(np.int32)), None,
                                     n_cols=n + J.size, w_cols=torch.from_numpy(w_ext), device="cuda:0")
    L.tune(lds=lds, clenshaw=clen)
    if tiles:
        L.tune(tiles=1, tile_th=8, tile_max=4)
    lib = _lib.load()
    dev = torch.device("cuda:0")
    caller = torch.from_numpy(J.astype(np.int32)).to(dev)
    internal = torch.empty_like(caller)
    st = torch.cuda.current_stream(dev).cuda_stream
    check(lib.wg_laplacian_map_rows(L.handle, 0, ptr(caller), caller.numel(), ptr(internal), st), "map_rows")
    uid = (ctypes.c_uint8 * 128)()
    check(lib.wg_dist_unique_id(uid), "unique_id")
    counts = np.array([J.size], np.int64)
    h = ctypes.c_void_p()
    check(lib.wg_dist_create(L.handle, uid, 0, 1, ptr(internal), counts.ctypes.data, counts.ctypes.data,
                             ctypes.byref(h)), "dist_create")
    try:
        check(lib.wg_dist_set_graph(h, graph), "set_graph")
        rng = np.random.default_rng(4)
        X = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
        S = torch.empty(n, F, device=dev)
        H = torch.empty(n, F, device=dev)
        K = 8
        res = []
        for _ in range(3):
            S.fill_(float("nan"))
            check(lib.wg_dist_wavelet_features(h, ptr(X), F, K, 0.8, ptr(S), ptr(H), st), "dist_wavelet_features")
            res.append(S.cpu().numpy().copy())
        ref = O.graph_wavelet_features(g.to_scipy(), k=K, s=0.8, X0=X.cpu().numpy(), return_all=True)
        for r in res:
            assert np.array_equal(r, res[0])
        assert_parity(res[0], ref["S"], what=f"loopback F={F} lds={lds} graph={graph}")
        info = (ctypes.c_int64 * 8)()
        check(lib.wg_dist_info(h, info), "dist_info")
        if tiles:
            assert "tiles:" in L.describe(F), L.describe(F)
            # the tail beside the dense blocks (hyb_conc): off and forced on, bitwise the same
            for conc in (0, 2, 1):
                L.tune(hyb_conc=conc)
                for _ in range(2):   # eager, then replayed (or eager again where the tail runs beside)
                    S.fill_(float("nan"))
                    check(lib.wg_dist_wavelet_features(h, ptr(X), F, K, 0.8, ptr(S), ptr(H), st), "dist_wavelet_features")
                    assert np.array_equal(S.cpu().numpy(), res[0]), f"hyb_conc={conc}"
        assert info[0] == 0 and info[5] == 2 and info[7] == 1, list(info)
        L.profile_enable(True)
        check(lib.wg_dist_wavelet_features(h, ptr(X), F, K, 0.8, ptr(S), ptr(H), st), "dist_wavelet_features")
        tot, cnt = ctypes.c_double(0), ctypes.c_int64(0)
        check(lib.wg_dist_profile_collect(h, ctypes.byref(tot), ctypes.byref(cnt)), "profile_collect")
        L.profile_collect()
        L.profile_enable(False)
        assert cnt.value == K and tot.value > 0
    finally:
        lib.wg_dist_destroy(h)


def _gather_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wats_hip.dist import gather_rows
        g = rmat_graph(700, 5000, seed=2)
        b = partition_rows(g.indptr, world)
        full = np.arange(g.n * 3, dtype=np.float32).reshape(g.n, 3)
        got = gather_rows(torch.from_numpy(full[b[rank]:b[rank + 1]].copy()), b)
        q.put((rank, bool(np.array_equal(got.numpy(), full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rows_cpu_gloo(world):
    """The optional final gather of row-sharded outputs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


@pytest.mark.gpu
def test_native_chain_recaptures_after_tune():
    """the captured hipGraph must not outlive wg_laplacian_tune
    (which frees the plans its kernels point at and changes launch knobs).
    Three calls (eager, captured, replayed), a plan-shaping tune, then more
    calls: every result equals the oracle."""
    from wats_hip.dist import ShardedWavelet
    g = _native_graph("rmat")
    sw = ShardedWavelet(g.indptr, g.indices, g.values, g.n, np.array([0, g.n]), exchange="rccl", device="cuda:0")
    X = torch.from_numpy(np.random.default_rng(6).standard_normal((g.n, 8)).astype(np.float32)).cuda()
    ref = O.graph_wavelet_features(g.to_scipy(), k=6, s=0.8, X0=X.cpu().numpy(), return_all=True)
    for _ in range(3):
        H, S = sw.wavelet_features(X, k=6, s=0.8)
    assert_parity(S.cpu().numpy(), ref["S"], what="before tune")
    for knobs in ({"iter": 3, "block_iter": 2, "chunk_iter": 2}, {"clenshaw": 0}, {"waves": 8}):
        sw.L.tune(**knobs)
        for _ in range(3):
            H, S = sw.wavelet_features(X, k=6, s=0.8)
            assert_parity(S.cpu().numpy(), ref["S"], what=f"after tune {knobs}")
    sw.close()


def _empty_shard_worker(rank, world, port, bounds, F, q, exchange="ipc"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wats_hip.dist import ShardedWavelet
        g = _graph("rmat")
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        lo, hi = g.indptr[r0], g.indptr[r1]
        sw = ShardedWavelet(g.indptr[r0:r1 + 1] - lo, g.indices[lo:hi], None, g.n, np.asarray(bounds),
                            exchange=exchange, device="cuda:0", max_features=F)
        X = np.random.default_rng(0).standard_normal((g.n, F)).astype(np.float32)
        outs = [sw.wavelet_features(torch.from_numpy(X[r0:r1]), k=5, s=0.8) for _ in range(3)]
        sw.check_exchange()
        sw.close()
        q.put((rank, outs[0][1].cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("F,exchange", [(1, "ipc"), (4, "ipc"), (4, "sdma")])
def test_ipc_chain_with_an_empty_shard(F, exchange):
    """a rank that owns no rows runs the native chain too (it must
    take part in every exchange phase); before, it took the Python path and
    its peers hung.  Bounds [0, 600, 600, 1100, n]: rank 1 is empty."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = _graph("rmat")
    bounds = [0, 600, 600, 1100, g.n]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_empty_shard_worker, args=(r, 4, port, bounds, F, q, exchange)) for r in range(4)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=170) for _ in range(4)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1][1].shape == (0, F)
    X = np.random.default_rng(0).standard_normal((g.n, F)).astype(np.float32)
    ref = O.graph_wavelet_features(g.to_scipy(), k=5, s=0.8, X0=X, return_all=True)
    assert_parity(np.concatenate([r[1] for r in res]), ref["S"], what=f"empty shard F={F}")


def _width_worker(rank, world, port, widths, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wats_hip.dist import ShardedWavelet
        g = rmat_graph(4000, 120000, seed=9)
        bounds = partition_rows(g.indptr, world)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        lo, hi = g.indptr[r0], g.indptr[r1]
        sw = ShardedWavelet(g.indptr[r0:r1 + 1] - lo, g.indices[lo:hi], None, g.n, bounds, exchange="ipc",
                            device="cuda:0", max_features=max(widths))
        sw.L.tune(tiles=1, tile_th=8, tile_max=3)
        out = []
        for F in widths:
            X = np.random.default_rng(F).standard_normal((g.n, F)).astype(np.float32)
            H, S = sw.wavelet_features(torch.from_numpy(X[r0:r1]), k=6, s=0.8)
            torch.cuda.synchronize()
            out.append(S.cpu().numpy())
        sw.check_exchange()
        sw.close()
        q.put((rank, out))
    except Exception as exc:  # noqa: BLE001
        import traceback
        q.put((rank, f"{exc!r}\n{traceback.format_exc()}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_ipc_chain_width_changes():
    """The IPC pull moves only a signal's own columns (F = 41: 44 of the 48 exchanged, the halo rows' pad
    columns zeroed once per width), and a full-width pull (F = 48) invalidates those zeros: one handle runs
    F = 41, 48, 41, 16 in turn on 2 ranks sharing the GPU (the hybrid step on both shards), every result
    against the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    widths = [41, 48, 41, 16]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_width_worker, args=(r, 2, port, widths, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(2):
            res.append(q.get(timeout=170))
            if isinstance(res[-1][1], str):
                pytest.fail(f"rank {res[-1][0]}: {res[-1][1]}")
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    res.sort(key=lambda t: t[0])
    g = rmat_graph(4000, 120000, seed=9)
    for i, F in enumerate(widths):
        X = np.random.default_rng(F).standard_normal((g.n, F)).astype(np.float32)
        ref = O.graph_wavelet_features(g.to_scipy(), k=6, s=0.8, X0=X, return_all=True)
        assert_parity(np.concatenate([r[1][i] for r in res]), ref["S"], what=f"IPC width change F={F} (call {i})")
