"""How much of a Chebyshev step is its own-row streams (run on the GPU box):
time wg_cheb_step (all rows, internal order) with and without the T_k store
and the S read/write, at the named config's F.  Timing only: the variants
without S / T_k do not compute the chain.

    python tools/stream_probe.py [--config ogbn-arxiv] [--reps 20]
"""
import argparse
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, named_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ogbn-arxiv")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n, nnz, K, F = NAMED_CONFIGS[a.config]
    L = wats_hip.NormalizedLaplacian.from_graph(named_graph(a.config))
    torch.manual_seed(1)
    T = [torch.randn(L.n, F, device="cuda") for _ in range(3)]
    S = torch.randn(L.n, F, device="cuda")
    variants = {"T_k + S": (True, True), "T_k only": (True, False), "S only": (False, True), "neither": (False, False)}
    for rnd in range(2):
        for name, (wt, ws) in variants.items():
            run = lambda k: L.step(k, T[0], T[1], T[2] if wt else None, S=S if ws else None, alpha0=1.0,
                                   alpha_k=math.exp(-0.8 * k))
            for k in range(2, 5):
                run(k)
            torch.cuda.synchronize()
            L.profile_enable(True)
            for _ in range(a.reps):
                run(2)
            p = L.profile_collect()
            L.profile_enable(False)
            print(json.dumps(dict(round=rnd, variant=name, step_us=p["sum_ms"] / p["launches"] * 1e3,
                                  config=a.config, F=F)), flush=True)


if __name__ == "__main__":
    main()
