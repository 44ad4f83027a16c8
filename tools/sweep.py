"""GPU tuning sweep for the step kernel (run on the GPU box).

For a named config: time graph_wavelet_features' step kernels for a grid of
(iter, chunk_iter) knobs, and (--segments, a -DWG_TIMING_PROBES build: the
"seg_mask" key) attribute time per plan segment.
Writes one JSON line per measurement to stdout."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, named_graph  # noqa: E402


REPS = 10


def time_chain(L, X, K, reps=None):
    reps = reps or REPS
    n, F = X.shape
    S = torch.empty_like(X)
    H = torch.empty_like(X)
    lib = wats_hip._lib.load()
    st = torch.cuda.current_stream().cuda_stream
    run = lambda: wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), F, K, 0.8, S.data_ptr(),
                                                               H.data_ptr(), st))
    for _ in range(1 if reps <= 2 else 2):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):   # no per-launch events: the chain as the bench times it
        run()
    e1.record()
    torch.cuda.synchronize()
    chain_us = e0.elapsed_time(e1) / reps * 1e3
    L.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    p = L.profile_collect()
    L.profile_enable(False)
    return dict(chain_us=chain_us, step_us=p["sum_ms"] / max(1, p["launches"]) * 1e3, max_us=p["max_ms"] * 1e3,
                call_ms=wall * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ogbn-arxiv")
    ap.add_argument("--F", type=int, default=None)
    ap.add_argument("--K", type=int, default=None)
    ap.add_argument("--grid", default="iter=24;chunk_iter=128",
                    help="knob grid, e.g. 'iter=16,24;chunk_iter=64,128;nt=0,7'")
    ap.add_argument("--segments", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm-s", type=float, default=1.0, help="seconds of untimed chains before the grid")
    ap.add_argument("--keep-order", action="store_true", help="WG_FLAG_KEEP_COLUMN_ORDER (no per-row column sort)")
    a = ap.parse_args()
    global REPS
    REPS = a.reps
    import itertools
    n, nnz, K, F = NAMED_CONFIGS[a.config]
    F = a.F or F
    K = a.K or K
    if nnz > 20_000_000:   # numpy generator too slow: same recipe on the GPU
        from wats_hip.graphgen import rmat_graph_device
        ip, ix = rmat_graph_device(n, nnz, seed=0)
        L = wats_hip.NormalizedLaplacian(n, ip, ix, sort_columns=not a.keep_order)
        del ip, ix
    else:
        g = named_graph(a.config)
        L = wats_hip.NormalizedLaplacian.from_graph(g, sort_columns=not a.keep_order)
    X = torch.randn(L.n, F, device="cuda") if F > 1 else L.log1p_degree()
    n_act = L.n - int(L.info["n_closed_form"])
    bstep = 8 * L.nnz + 4 * (n_act + 1) + 20 * n_act * F
    # knobs separated by ';' or '/' (the latter survives a shell command line unquoted)
    grid = [(kv.split("=")[0], [int(v) for v in kv.split("=")[1].split(",")])
            for kv in a.grid.replace("/", ";").split(";") if kv]
    names = [k for k, _ in grid]
    # Clock ramp: without ~1 s of load first, the first grid entry reads 2-3 us slow
    # on arxiv F=40 (profiles/r01/s48_ab.log round 0, s51_iter_sweep.log).
    t_end = time.perf_counter() + a.warm_s
    while time.perf_counter() < t_end:
        time_chain(L, X, K, reps=2)
    first = None
    for combo in itertools.product(*[v for _, v in grid]):
        knobs = dict(zip(names, combo))
        first = first or knobs
        L.tune(**knobs)
        r = time_chain(L, X, K)
        r.update(config=a.config, keep_order=a.keep_order, F=F, K=K, GBs=bstep / (r["step_us"] * 1e-6) / 1e9, **knobs)
        print(json.dumps(r), flush=True)
    if a.segments:
        L.tune(**first)
        plan = L.describe(F)
        print(plan, flush=True)
        nseg = int(plan.split("segments=")[1].split()[0])
        for i in range(nseg):
            L.tune(seg_mask=1 << i)
            r = time_chain(L, X, K)
            r.update(segment=i)
            print(json.dumps(r), flush=True)
        L.tune(seg_mask=-1)


if __name__ == "__main__":
    main()
