"""Full-size, column-sensitive parity: the Reddit-size
(233k nodes / 114.6M nonzeros, K=16) and 8M R-MAT (8.4M / 268M, K=32)
configurations of BASELINE.json, with RANDOM signals -- a wrong gathered
column or a wrong halo row changes the result, unlike the eigenvector KAT
(X0 = sqrt(degree) makes every gathered u_j equal).

The checker is the C restatement of the reference path (oracle/wats_chain.c,
pinned bit for bit to the numpy oracle and to the reference's golden vectors
by tests/test_oracle.py), run on the GPU box's host cores.  Columns of the
chain are independent, so the F=41 run is checked on a subset of its
columns; H (which couples the columns) is checked against S in float64.
Every row-sharded run (2 and 4 ranks sharing the one GPU, the native IPC
exchange) is compared with the same oracle on every rank's rows.

Graphs come from the GPU generator (wats_hip.graphgen.rmat_graph_device), as
in bench.py.  Reference: calibration/WATS.py:29-37 (the recurrence),
WATS.py:65-72 (heat sum, normalisation)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import REPO, assert_parity

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

import wats_hip  # noqa: E402
from wats_hip import NormalizedLaplacian  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402

ORACLE_THREADS = 16   # the GPU box's CPU share (os.cpu_count() reports the whole machine there)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    wats_hip._lib.load()


def _log(msg):
    import sys
    import time
    print(f"[fullsize {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _oracle(indptr, indices, X, k, cols=None):
    from oracle import wats_oracle_c as C
    import time
    Xs = X if cols is None else np.ascontiguousarray(X[:, cols])
    t0 = time.perf_counter()
    S, H = C.graph_wavelet_features(indptr, indices, None, Xs, k, 0.8, threads=ORACLE_THREADS)
    _log(f"oracle: n={len(indptr) - 1} nnz={len(indices)} K={k} F={Xs.shape[1]}: {time.perf_counter() - t0:.1f} s")
    return S, H


_GRAPHS = {}


def _graph(config, seed=0):
    """(indptr int64, indices int32) host arrays of the named config, generated
    on the GPU (cached per module)."""
    key = (config, seed)
    if key not in _GRAPHS:
        n, nnz, _, _ = NAMED_CONFIGS[config]
        _log(f"generating {config}")
        ip, ix = rmat_graph_device(n, nnz, seed=seed, device="cuda")
        _GRAPHS.clear()
        _GRAPHS[key] = (ip.cpu().numpy(), ix.cpu().numpy())
        del ip, ix
        torch.cuda.empty_cache()
    return _GRAPHS[key]


def _forms(describe):
    """The hybrid step's launches per form, from wg_laplacian_describe's 'hybrid forms:' line."""
    line = [x for x in describe.splitlines() if x.startswith("hybrid forms:")]
    assert line, describe
    return {k: int(v) for k, v in (t.split("=") for t in line[-1].split(":", 1)[1].split())}


def _check_H(H, S):
    """H = S / (|S|_1 + 1e-8) (WATS.py:71-72), recomputed from S in float64."""
    Sd = S.astype(np.float64)
    Hd = Sd / (np.abs(Sd).sum(axis=1, keepdims=True) + 1e-8)
    big = np.abs(Sd).sum(axis=1) > 1e-4 * np.abs(Sd).sum(axis=1).max()
    assert np.abs(H[big] - Hd[big]).max() <= 1e-5


# ------------------------------------------------------------------ one GPU
@pytest.mark.parametrize("F,cols", [(1, None), (41, [0, 17, 40])])
def test_reddit_random_signal_vs_oracle(F, cols):
    """Reddit-size K=16, auto plan: the F=1 chunk-window LDS kernel
    (csrc/lds1.hip) and, at F=41, the hybrid step (width padded
    to 48, dense blocks on the bf16 MFMA tile kernel, the rest of each row
    gathered by the step kernel with the >= 8 M-nonzero tail plan) -- asserted,
    so a change of the auto rule cannot move the only full-size test of the
    MFMA kernel back onto the gather kernel."""
    indptr, indices = _graph("reddit")
    n = len(indptr) - 1
    L = NormalizedLaplacian(n, torch.from_numpy(indptr), torch.from_numpy(indices))
    if F == 1:
        info = L.lds_plan_info(active_only=True)
        assert info is not None and info["mode"] == 2, info     # chunk windows
    X = np.random.default_rng(11 + F).standard_normal((n, F)).astype(np.float32)
    H, S = wats_hip.graph_wavelet_features(L, k=16, X0=torch.from_numpy(X), return_S=True)
    S, H = S.cpu().numpy(), H.cpu().numpy()
    if F == 41:
        d = L.describe(48)
        assert "tiles:" in d, "the hybrid step did not run: " + d
        # the shipped form: dense blocks and the tail's waves in one launch (hybrid_fused_kernel), every step
        assert _forms(d) == {"fused": 16, "two_stream": 0, "sequential": 0}, d
    L.close()
    S_ref, H_ref = _oracle(indptr, indices, X, 16, cols)
    got = S if cols is None else S[:, cols]
    assert_parity(got, S_ref, what=f"reddit F={F} S")
    if F == 1:
        ok = np.abs(S_ref[:, 0]) > 1e-3 * np.abs(S_ref).max()
        assert np.abs(H[ok, 0] - H_ref[ok, 0]).max() <= 1e-5
    else:
        _check_H(H, S)


def test_rmat8m_random_signal_vs_oracle():
    """8M R-MAT K=32 F=1: the hub-teams kernel (cheb_hub1_kernel, lds mode 4)."""
    indptr, indices = _graph("rmat-8m")
    n = len(indptr) - 1
    L = NormalizedLaplacian(n, torch.from_numpy(indptr), torch.from_numpy(indices))
    info = L.lds_plan_info(active_only=True)
    assert info is not None and info["mode"] == 4, info
    X = np.random.default_rng(5).standard_normal((n, 1)).astype(np.float32)
    H, S = wats_hip.graph_wavelet_features(L, k=32, X0=torch.from_numpy(X), return_S=True)
    S = S.cpu().numpy()
    L.close()
    S_ref, _ = _oracle(indptr, indices, X, 32)
    assert_parity(S, S_ref, what="rmat-8m S")


@pytest.mark.parametrize("F", [1, 40, 41])
def test_large_graph_defaults_random_signal(F):
    """The >= 16 M-nonzero defaults (chunk_iter 128, int4 index loads at F=1,
    8 entries per lane, vidx) on a 20 M-nonzero R-MAT graph with a random
    signal, against the oracle (was an eigenvector KAT, blind to column
    errors)."""
    ip, ix = rmat_graph_device(400_000, 20_000_000, seed=3)
    L = NormalizedLaplacian(400_000, ip, ix)
    indptr, indices = ip.cpu().numpy(), ix.cpu().numpy()
    X = np.random.default_rng(F).standard_normal((400_000, F)).astype(np.float32)
    H, S = wats_hip.graph_wavelet_features(L, k=16, X0=torch.from_numpy(X), return_S=True)
    S, H = S.cpu().numpy(), H.cpu().numpy()
    L.close()
    cols = None if F == 1 else [0, F // 2, F - 1]
    S_ref, _ = _oracle(indptr, indices, X, 16, cols)
    assert_parity(S if cols is None else S[:, cols], S_ref, what=f"20M R-MAT F={F} S")
    if F > 1:
        _check_H(H, S)


# ------------------------------------------------------------------ row-sharded, ranks sharing the GPU
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_worker(rank, world, port, config, F, K, seed_x, q, graph_dir):
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(120, exit=False)   # where a stuck rank is, before the parent gives up
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["WATS_DIST_LOG"] = "1"
    os.environ["RANK"] = str(rank)
    sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from wats_hip.dist import ShardedWavelet, partition_rows
        n, nnz, _, _ = NAMED_CONFIGS[config]
        # the graph the parent generated (ranks generating it concurrently on the one shared GPU
        # stalled for minutes inside torch.unique's radix sort), memory-mapped
        indptr = np.load(os.path.join(graph_dir, "indptr.npy"))
        ix = np.load(os.path.join(graph_dir, "indices.npy"), mmap_mode="r")
        bounds = partition_rows(indptr, world)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        lo, hi = int(indptr[r0]), int(indptr[r1])
        cols = np.ascontiguousarray(ix[lo:hi])
        del ix
        sw = ShardedWavelet(indptr[r0:r1 + 1] - lo, cols, None, n, bounds, exchange="ipc", device="cuda:0",
                            max_features=F)
        X = np.random.default_rng(seed_x).standard_normal((n, F)).astype(np.float32)[r0:r1]
        outs = []
        for i in range(3):   # eager, captured, replayed
            outs.append(sw.wavelet_features(torch.from_numpy(X), k=K, s=0.8))
            torch.cuda.synchronize()
            _log(f"rank {rank}: chain {i} done")
        H, S = outs[0]
        same = all(torch.equal(o[1], S) for o in outs)
        path = "u" if (F == 1 and sw.u_len() > 0) else "t"
        d = sw.L.describe(F + (-F) % 16)
        if F > 1 and "tiles:" in d:
            path = "tiles"   # the hybrid step ran on this shard
            f = _forms(d)
            if f["fused"] > 0 and f["two_stream"] == 0 and f["sequential"] == 0:
                path = "tiles-fused"   # every step in the one-launch form (hybrid_fused_kernel)
        sw.check_exchange()
        sw.close()
        q.put((rank, r0, r1, S.cpu().numpy(), H.cpu().numpy(), same, path))
    except Exception as exc:  # noqa: BLE001
        q.put((rank, None, None, None, None, False, repr(exc)))
        raise
    finally:
        dist.destroy_process_group()


def _run_sharded(world, config, F, K, seed_x, graph_dir):
    indptr, indices = _graph(config)
    np.save(os.path.join(graph_dir, "indptr.npy"), indptr)
    np.save(os.path.join(graph_dir, "indices.npy"), indices)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, config, F, K, seed_x, q, graph_dir),
                         daemon=True) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = sorted([q.get(timeout=170) for _ in range(world)], key=lambda t: t[0])
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("world,config,F,cols", [(2, "reddit", 1, None), (4, "reddit", 1, None),
                                                 (4, "reddit", 41, [0, 21, 40]), (2, "rmat-8m", 1, None)])
def test_sharded_full_size_vs_oracle(world, config, F, cols, tmp_path):
    """The row-sharded chain (nnz-balanced shards, [own | halo] columns, the
    one-sided IPC exchange, the chain captured and replayed as a hipGraph) on
    the full-size graph with a random signal: every rank's rows against the
    oracle, eager == captured == replayed bit for bit."""
    K = NAMED_CONFIGS[config][2]
    res = _run_sharded(world, config, F, K, 100 + F, str(tmp_path))
    for r in res:
        assert r[1] is not None, f"rank {r[0]} failed: {r[6]}"
        assert r[5], f"rank {r[0]}: eager / captured / replayed chains differ"
    if F == 1 and config == "reddit":
        assert all(r[6] == "u" for r in res), "Reddit F=1 shards should run the LDS kernel"
    if F == 41:
        assert all(r[6] == "tiles-fused" for r in res), \
            f"every Reddit F=41 shard should run the fused hybrid step: {[r[6] for r in res]}"
    S = np.concatenate([r[3] for r in res])
    H = np.concatenate([r[4] for r in res])
    indptr, indices = _graph(config)
    n = len(indptr) - 1
    assert S.shape == (n, F)
    X = np.random.default_rng(100 + F).standard_normal((n, F)).astype(np.float32)
    S_ref, H_ref = _oracle(indptr, indices, X, K, cols)
    assert_parity(S if cols is None else S[:, cols], S_ref, what=f"sharded {config} world={world} F={F} S")
    if F > 1:
        _check_H(H, S)
