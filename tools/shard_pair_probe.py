"""Does one 8-way shard's hybrid step fill the GPU?  Two ranks' shards stepped together on two
streams (run on the GPU box) against each alone: if two together take little more than one,
the step leaves most of the GPU idle and running its tile and tail kernels side by side could pay.

    python tools/shard_pair_probe.py --config reddit --world 8 --ranks 0,1 --F 48
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from shard_probe import build_shard  # noqa: E402
from wats_hip import _lib  # noqa: E402
from wats_hip._lib import check, ptr  # noqa: E402
from wats_hip.dist import partition_rows  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="reddit")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", default="0,1")
    ap.add_argument("--F", type=int, default=48)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lds", type=int, default=3)
    ap.add_argument("--groups", type=int, default=1)
    a = ap.parse_args()
    n, nnz_t, K, _ = NAMED_CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    ip, ix = rmat_graph_device(n, nnz_t, seed=0, device=dev)
    indptr = ip.cpu().numpy()
    deg = np.diff(indptr).astype(np.float32)
    b = partition_rows(indptr, a.world)
    lib = _lib.load()
    F = a.F
    shards = []
    for rk in [int(x) for x in a.ranks.split(",")]:
        a.rank = rk
        L, n_own, n_cols = build_shard(a, b, ip, ix, indptr, deg, dev)
        L.tune(lds=a.lds)
        X = [torch.rand(n_cols, F, device=dev), torch.rand(n_own, F, device=dev), torch.rand(n_own, F, device=dev)]
        shards.append((L, X, torch.cuda.Stream()))

    def step(sh):
        L, X, s = sh
        check(lib.wg_clenshaw_step(L.handle, F, ptr(X[0]), ptr(X[1]), ptr(X[2]), ptr(X[1]), 0.3, 2.0, 1 | 2 | 4,
                                   s.cuda_stream), "clenshaw_step")

    def timed(which):
        for _ in range(3):
            for sh in which:
                step(sh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for sh in which:
            sh[2].wait_stream(torch.cuda.current_stream())
        for _ in range(a.reps):
            for sh in which:
                step(sh)
        for sh in which:
            torch.cuda.current_stream().wait_stream(sh[2])
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    for i, sh in enumerate(shards):
        print(f"shard {i} alone: {timed([sh]):.1f} us per step", flush=True)
    print(f"all {len(shards)} together on {len(shards)} streams: {timed(shards):.1f} us per step of each", flush=True)
    for L, _, _ in shards:
        L.close()


if __name__ == "__main__":
    main()
