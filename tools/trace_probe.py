"""Per-wave timeline of one step launch (probe build, tuning key "trace"; GPU box).

Runs the arxiv-size F = 40 chain (or --config) with WATS_HIP_LIB pointing at the
-DWG_TIMING_PROBES build, records launch --launch of the chain (1-based) and saves
{trace (n, 4) uint64, plan text} to --out (.npz) for offline analysis
(tools/trace_report.py).  Each trace row: [block | wave << 24 | xcc << 28 |
hw_id << 32, start, end (100 MHz wall clock), shader cycles]."""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, named_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ogbn-arxiv")
    ap.add_argument("--launch", type=int, default=8)
    ap.add_argument("--knobs", default="", help="extra tuning keys, e.g. 'gather4=0,iter=96'")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    n, nnz, K, F = NAMED_CONFIGS[a.config]
    g = named_graph(a.config)
    L = wats_hip.NormalizedLaplacian.from_graph(g)
    knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.knobs.split(",") if kv)
    if knobs:
        L.tune(**knobs)
    X = torch.randn(L.n, F, device="cuda")
    lib = wats_hip._lib.load()
    fn = lib.wg_probe_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    for _ in range(20):   # warm, clock ramp
        wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=X)
    torch.cuda.synchronize()
    out = {}
    for rep in range(3):
        L.tune(trace=a.launch, **knobs)
        wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=X)
        torch.cuda.synchronize()
        got = ctypes.c_int64(0)
        buf = np.zeros(1 << 22, np.uint64)
        wats_hip._lib.check(fn(L.handle, buf.ctypes.data, buf.size, ctypes.byref(got)))
        tr = buf[:got.value].reshape(-1, 4)
        out[f"trace{rep}"] = tr
        st = tr[tr[:, 1] > 0]
        span = (st[:, 2].max() - st[:, 1].min()) * 10e-3
        print(f"rep {rep}: {len(st)} waves, span {span:.2f} us, mean wave {(st[:, 2] - st[:, 1]).mean() * 10:.0f} ns",
              flush=True)
    np.savez(a.out, plan=np.array(L.describe(F)), **out)
    L.tune(trace=0)
    print(L.describe(F))


if __name__ == "__main__":
    main()
