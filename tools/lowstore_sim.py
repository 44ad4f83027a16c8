"""CPU model (a checker, not product code): the Clenshaw chain with the b_k of tiny weight c_k stored
in bfloat16 (the rest float32, sums float64), against the oracle -- the precision side of a
16-bit storage of the first vectors (not kept)."""
import os, sys, numpy as np, scipy.sparse as sp, scipy.sparse.csgraph as cg, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd")); sys.path.insert(0, REPO)
from wats_hip.graphgen import named_graph, connect_isolated
from oracle import wats_oracle as O
def bf16(x): return torch.from_numpy(np.ascontiguousarray(x,dtype=np.float32)).to(torch.bfloat16).float().numpy().astype(np.float64)
f32=lambda v: v.astype(np.float32).astype(np.float64)
g=connect_isolated(named_graph("ogbn-arxiv"),seed=7); A=g.to_scipy(); F=8
X=np.random.default_rng(0).standard_normal((A.shape[0],F)).astype(np.float32)
L=sp.csr_matrix(cg.laplacian(A.astype(np.float32),normed=True),dtype=np.float64)-sp.identity(A.shape[0],format="csr")
for K,s in ((16,0.8),(32,0.8),(16,0.3)):
    c=np.exp(-s*np.arange(K+1))
    ref=O.graph_wavelet_features(A,k=K,s=s,X0=X,return_all=True)["S"]
    def err(S):
        big=np.abs(ref)>1e-3*np.abs(ref).max(0)
        return float(np.max(np.abs(S-ref).max(0)/np.abs(ref).max(0))), float(np.max(np.abs(S-ref)[big]/np.abs(ref)[big]))
    def runb(th):
        X0=X.astype(np.float64); b1=np.zeros_like(X0); b2=np.zeros_like(X0); n16=0
        for k in range(K,0,-1):
            b=c[k]*X0+2*(L@b1)-b2
            if c[k]<=th and k<K: b=bf16(b); n16+=1
            else: b=f32(b)
            b2=b1; b1=b
        return c[0]*X0+L@b1-b2, n16
    print(K,s,"fp32",err(runb(0)[0]))
    for th in (2e-5,5e-6):
        S,n16=runb(th); print(K,s,"bf16 c_k<=",th,"vectors",n16,err(S))
