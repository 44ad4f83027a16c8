"""Product-form chain (tuning key prod) against the oracle and Clenshaw: precision per K on the
arxiv-size graph and its connected variant, F = 40 (run on the GPU box)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from oracle import wats_oracle as O  # noqa: E402
from wats_hip.graphgen import connect_isolated, named_graph  # noqa: E402

g0 = named_graph("ogbn-arxiv")
for gname, g in (("arxiv", g0), ("arxiv-connected", connect_isolated(g0, seed=7))):
    A = g.to_scipy()
    X = np.random.default_rng(1).standard_normal((g.n, 40)).astype(np.float32)
    L = wats_hip.NormalizedLaplacian.from_graph(g)
    for K in (1, 2, 3, 5, 16, 32):
        ref = O.graph_wavelet_features(A, k=K, s=0.8, X0=X, return_all=True)
        out = {}
        for prod in (0, 1):
            L.tune(prod=prod)
            H, S = wats_hip.graph_wavelet_features(L, k=K, X0=torch.from_numpy(X), return_S=True)
            torch.cuda.synchronize()
            S = S.cpu().numpy().astype(np.float64)
            d = np.abs(S - ref["S"])
            big = np.abs(ref["S"]) > 1e-3 * np.abs(ref["S"]).max()
            out[prod] = dict(norm=float(d.max() / np.abs(ref["S"]).max()),
                             col=float(max(d[:, j].max() / np.abs(ref["S"][:, j]).max() for j in range(40))),
                             elem=float((d[big] / np.abs(ref["S"][big])).max()),
                             H=float(np.abs(H.cpu().numpy() - ref["H"])[big].max()))
        print(json.dumps(dict(graph=gname, K=K, clenshaw=out[0], prod=out[1])), flush=True)
    L.close()
