"""8(f)-2 measurement: one CompatibleGCN propagation adj_norm @ x (reference
src/gnn/model.py:43-47, dense torch.mm in fp32) vs the HIP CSR SpMM
(wats_hip.RowNormalizedAdjacency), on synthetic R-MAT graphs with self loops.
One JSON line per (graph, F)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip.graphgen import rmat_graph  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


for name, n, nnz in [("cora", 2708, 10556), ("pubmed", 19717, 88648), ("subsampled-20k", 20000, 400000)]:
    g = rmat_graph(n, nnz, seed=0)
    A = (g.to_scipy() + sp.eye(n)).tocsr()
    adj = torch.tensor(A.toarray(), dtype=torch.float32, device="cuda")
    deg = adj.sum(dim=1, keepdim=True)
    deg[deg == 0] = 1
    norm = adj / deg
    op = wats_hip.RowNormalizedAdjacency.from_dense(adj)
    for F in (64, 500, 1433):
        x = torch.randn(n, F, device="cuda")
        t_dense = timed(lambda: torch.mm(norm, x))
        t_sp = timed(lambda: wats_hip.propagate(op, x))
        err = ((wats_hip.propagate(op, x) - torch.mm(norm.double(), x.double()).float()).abs().max()
               / torch.mm(norm.double(), x.double()).abs().max()).item()
        print(json.dumps(dict(graph=name, n=n, nnz=int(A.nnz), F=F, dense_mm_us=t_dense * 1e6, spmm_us=t_sp * 1e6,
                              speedup=t_dense / t_sp, max_rel_err=err)), flush=True)
