"""One PubMed-size one-launch chain with the given tuning keys, checked against the oracle (diagnostics)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from oracle import wats_oracle as O  # noqa: E402
from wats_hip.graphgen import named_graph  # noqa: E402

knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[1:])
g = named_graph("pubmed", seed=0)
L = wats_hip.NormalizedLaplacian.from_graph(g)
L.tune(**knobs)
print(knobs, flush=True)
H, S = wats_hip.graph_wavelet_features(L, k=16, s=0.8, return_S=True)
torch.cuda.synchronize()
print(L.describe(1), flush=True)
ref = O.graph_wavelet_features(g.to_scipy(), k=16, s=0.8, X0=L.log1p_degree().cpu().numpy(), return_all=True)
print("rel err", float(np.abs(S.cpu().numpy() - ref["S"]).max() / np.abs(ref["S"]).max()), flush=True)
