"""Run N chains of a named config (for rocprofv3 traces of the one-launch chain)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, named_graph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "pubmed"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in sys.argv[3:])
n, nnz, K, F = NAMED_CONFIGS[cfg]
g = named_graph(cfg, seed=0)
L = wats_hip.NormalizedLaplacian.from_graph(g)
L.tune(**knobs)
X = L.log1p_degree()
for _ in range(reps):
    wats_hip.graph_wavelet_features(L, k=K, s=0.8, X0=X)
torch.cuda.synchronize()
print(L.describe(1))
