"""Chain time with and without the hipGraph replay of wg_wavelet_features
(tuning key "graph"), per graph size: back-to-back throughput (chains queued
without a sync) and single-chain latency (sync after each), HIP events and
host wall clock.  Usage: python tools/graph_probe.py [--configs pubmed,ogbn-arxiv-f1]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, named_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="pubmed,ogbn-arxiv-f1,cora")
ap.add_argument("--reps", type=int, default=200)
ap.add_argument("--modes", default="graph=0;graph=1",
                help="';'-separated knob sets, each 'key=value,key=value' (tuning keys of wg_laplacian_tune)")
args = ap.parse_args()
lib = wats_hip._lib.load()
for cfg in args.configs.split(","):
    n, nnz, K, F = NAMED_CONFIGS[cfg]
    g = named_graph(cfg.replace("-f1", ""), seed=0)
    modes = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in m.split(",") if kv) for m in args.modes.split(";")]
    for mode in modes + modes:
        L = wats_hip.NormalizedLaplacian.from_graph(g)
        L.tune(**mode)
        X = L.log1p_degree() if F == 1 else torch.randn(g.n, F, device="cuda")
        S = torch.empty(g.n, F, device="cuda")
        H = torch.empty(g.n, F, device="cuda")
        st = torch.cuda.current_stream().cuda_stream

        def run():
            wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), F, K, 0.8, S.data_ptr(),
                                                        H.data_ptr(), st), "wf")
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        for _ in range(args.reps):
            run()
        b.record()
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        thr = a.elapsed_time(b) / args.reps * 1e3
        lat = []
        for _ in range(50):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t1) * 1e6)
        lat.sort()
        print(f"{cfg} K={K} F={F} {mode}: back-to-back {thr:.1f} us/chain (host enqueue {t_host / args.reps * 1e6:.1f} "
              f"us/chain, wall {t_all / args.reps * 1e6:.1f}); single chain median {lat[25]:.1f} us", flush=True)
        L.close()
