"""Hybrid-step probe (csrc/tiles.hip) on a named config generated on the GPU:
per knob set the mean step time (HIP events around each step launch, both
kernels of a hybrid step), the chain time and S's max relative difference
against the first set.  Run on the GPU box:

    python tools/tiles_probe.py --config reddit-f41 --sets "tiles=0;tiles=1,tile_th=64;tiles=1,tile_th=32"
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

import wats_hip  # noqa: E402
from sweep import time_chain  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="reddit-f41")
    ap.add_argument("--F", type=int, default=None)
    ap.add_argument("--sets", required=True)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n, nnz, K, F = NAMED_CONFIGS[a.config]
    F = a.F or F
    indptr, indices = rmat_graph_device(n, nnz, seed=0, device="cuda")
    L = wats_hip.NormalizedLaplacian.from_csr(indptr, indices, None, n=n)
    del indptr, indices
    torch.manual_seed(1)
    X = torch.randn(L.n, F, device="cuda")
    sets = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv) for s in a.sets.split(";")]
    ref = None
    for rnd in range(a.rounds):
        for s in sets:
            L.tune(**s)
            H, S = wats_hip.graph_wavelet_features(L, X0=X, k=K, s=0.8, return_S=True)
            torch.cuda.synchronize()
            if ref is None:
                ref = S.clone()
            ds = ((S - ref).abs().max(dim=0).values / ref.abs().max(dim=0).values).max().item()
            r = time_chain(L, X, K, a.reps)
            plan = [ln for ln in L.describe(F).splitlines() if ln.startswith("tiles:")]
            r.update(round=rnd, config=a.config, F=F, K=K, S_rel_vs_first=ds, plan=plan[0] if plan else "", **s)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
