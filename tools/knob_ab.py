"""A/B of step-kernel knob sets on one named config (run on the GPU box):
per set, the mean step-kernel time and the max relative difference of S and H
against the first set (the reference numbering is unchanged by any knob).

    python tools/knob_ab.py --config ogbn-arxiv --sets "clenshaw=0;clenshaw=1" [--rounds 2]
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
from wats_hip.graphgen import NAMED_CONFIGS, named_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ogbn-arxiv")
    ap.add_argument("--F", type=int, default=None)
    ap.add_argument("--sets", required=True)
    ap.add_argument("--rounds", type=int, default=2, help="alternate the sets this many times")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    n, nnz, K, F = NAMED_CONFIGS[a.config]
    F = a.F or F
    g = named_graph(a.config)
    L = wats_hip.NormalizedLaplacian.from_graph(g)
    torch.manual_seed(1)
    X = torch.randn(L.n, F, device="cuda") if F > 1 else L.log1p_degree()
    sets = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in s.split(",") if kv) for s in a.sets.split(";")]
    keys = sorted({k for s in sets for k in s})
    if any(set(s) != set(keys) for s in sets):
        raise SystemExit("every set must name the same knobs (the handle keeps the last value of a knob)")
    ref = None
    for rnd in range(a.rounds):
        for s in sets:
            L.tune(**s)
            H, S = wats_hip.graph_wavelet_features(L, X0=X, k=K, s=0.8, return_S=True)
            torch.cuda.synchronize()
            if ref is None:
                ref = (S.clone(), H.clone())
            ds = ((S - ref[0]).abs().max() / ref[0].abs().max()).item()
            dh = ((H - ref[1]).abs().max()).item()
            r = time_chain(L, X, K, a.reps)
            r.update(round=rnd, config=a.config, F=F, K=K, S_rel_vs_first=ds, H_abs_vs_first=dh, **s)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
