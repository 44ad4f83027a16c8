"""Per-rank cost of one shard of the sharded chain with its halo exchange, on one GPU
(run on the GPU box, with a timing-probe build of the library).

One rank's shard of a row-sharded graph ([own | halo] columns, as wats_hip.dist
builds it) runs the native chain (csrc/dist.hip) at world 1 with a loopback
exchange: the halo rows are refreshed from own rows by RCCL send/recv to self,
then a spinning wave holds the stream for `xdelay` microseconds per exchange
(the link time an N-GPU run has and one GPU does not).  Prints the chain time
per Chebyshev step at each simulated link time (exchange, then the step).

    make -C efficient-gnn_amd/csrc VARIANT=probes EXTRA_FLAGS=-DWG_TIMING_PROBES
    WATS_HIP_LIB=$PWD/efficient-gnn_amd/wats_hip/libwats_hip_probes.so \\
        python tools/tier_probe.py --config reddit --world 8 --F 48 --delays 0,30,60
"""
import argparse
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip import _lib  # noqa: E402
from wats_hip._lib import check, ptr  # noqa: E402
from wats_hip.dist import partition_rows  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402


def shard(indptr, ix, deg, b, rank, dev):
    """[own | halo] local columns, halo ordered (owner, -degree, id) as build_halo_plan does."""
    r0, r1 = int(b[rank]), int(b[rank + 1])
    cols = ix[int(indptr[r0]):int(indptr[r1])].to(torch.int64)
    own = (cols >= r0) & (cols < r1)
    remote = cols[~own]
    halo_t = torch.unique(remote, sorted=True)
    halo_sorted = halo_t.cpu().numpy()
    owner_sorted = np.searchsorted(b, halo_sorted, side="right") - 1
    order = np.lexsort((halo_sorted, -deg[halo_sorted].astype(np.float64), owner_sorted))
    rank_of = np.empty(halo_sorted.size, np.int64)
    rank_of[order] = np.arange(halo_sorted.size)
    local = cols - r0
    local[~own] = (r1 - r0) + torch.from_numpy(rank_of).to(dev)[torch.searchsorted(halo_t, remote)]
    return r0, r1, local.to(torch.int32), halo_sorted[order]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="reddit")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--F", type=int, default=48)
    ap.add_argument("--delays", default="0,30,60")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--graph", type=int, default=1, help="replay the chain as a hipGraph (1) or run it eagerly (0)")
    ap.add_argument("--knobs", default="", help="tuning keys for the shard's handle, e.g. 'hyb_conc=1'")
    a = ap.parse_args()
    n, nnz_t, K, _ = NAMED_CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    ip, ix = rmat_graph_device(n, nnz_t, seed=0, device=dev)
    indptr = ip.cpu().numpy()
    deg = np.diff(indptr).astype(np.float32)
    b = partition_rows(indptr, a.world)
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    r0, r1, local, halo = shard(indptr, ix, deg, b, a.rank, dev)
    n_own, n_cols = r1 - r0, (r1 - r0) + int(halo.size)
    w = torch.from_numpy(np.concatenate([deg[r0:r1], deg[halo]]))
    L = wats_hip.NormalizedLaplacian(n_own, torch.from_numpy(indptr[r0:r1 + 1] - indptr[r0]), local, None,
                                     n_cols=n_cols, w_cols=w, device=dev)
    if a.knobs:
        L.tune(**{kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.knobs.split(",")})
    # loopback: halo row h is refreshed from own row h % n_own
    caller = torch.from_numpy((np.arange(halo.size) % n_own).astype(np.int32)).to(dev)
    internal = torch.empty_like(caller)
    check(lib.wg_laplacian_map_rows(L.handle, 0, ptr(caller), caller.numel(), ptr(internal), st), "map_rows")
    uid = (ctypes.c_uint8 * 128)()
    check(lib.wg_dist_unique_id(uid), "unique_id")
    h = ctypes.c_void_p()
    counts = np.array([halo.size], np.int64)
    check(lib.wg_dist_create(L.handle, uid, 0, 1, ptr(internal), counts.ctypes.data, counts.ctypes.data,
                             ctypes.byref(h)), "dist_create")
    check(lib.wg_dist_set_graph(h, a.graph), "set_graph")
    X = torch.randn(n_own, a.F, device=dev)
    S = torch.empty(n_own, a.F, device=dev)
    H = torch.empty(n_own, a.F, device=dev)
    print(f"shard {a.rank}/{a.world} rows {n_own} halo {halo.size} nnz {L.nnz} knobs {a.knobs or '-'}", flush=True)
    res = []
    for d in [int(x) for x in a.delays.split(",")]:
        L.tune(xdelay=d)   # a timing-probe build only (rejected as an unknown key otherwise)
        run = lambda: check(lib.wg_dist_wavelet_features(h, ptr(X), a.F, K, 0.8, ptr(S), ptr(H), st),
                            "dist_wavelet_features")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
        ev[0].record()
        t0 = time.perf_counter()
        for i in range(a.reps):
            run()
            ev[i + 1].record()
        host_ms = (time.perf_counter() - t0) * 1e3 / a.reps
        torch.cuda.synchronize()
        ms = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps))[a.reps // 2]
        r = dict(xdelay_us=d, chain_ms=ms, us_per_step=ms * 1e3 / K, host_ms_per_chain=host_ms)
        res.append(r)
        print(r, flush=True)
    lib.wg_dist_destroy(h)
    L.close()
    b0 = res[0]["us_per_step"]
    for r in res:
        print(f"  xdelay {r['xdelay_us']:4d}: {r['us_per_step']:8.1f} us/step, over xdelay {res[0]['xdelay_us']}: "
              f"{r['us_per_step'] - b0:7.1f}")


if __name__ == "__main__":
    main()
