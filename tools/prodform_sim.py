"""CPU model of the product-form chain's float32 rounding (tuning key prod): the
heat polynomial's quadratic factors applied to an arxiv-size graph with every stored vector rounded to
float32 (sums in float64), in three factor orders, against the oracle; plus the forward recurrence with
float32 storage.  r05: natural 1.05e-4, reversed 1.12e-4, interleaved 3.5e-7, greedy 2.7e-7, forward
1.4e-8 (max |err| / max |ref|); element-wise interleaved 4.3e-5.

    python tools/prodform_sim.py
"""
import sys, numpy as np, numpy.polynomial.chebyshev as C, scipy.sparse as sp
import os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd")); sys.path.insert(0, REPO)
from wats_hip.graphgen import named_graph
from oracle import wats_oracle as O
g=named_graph("ogbn-arxiv"); A=g.to_scipy()
K=16; s=0.8; F=8
X=np.random.default_rng(0).standard_normal((A.shape[0],F)).astype(np.float32)
ref=O.graph_wavelet_features(A,k=K,s=s,X0=X,return_all=True)["S"]
Lh=O.compute_normalized_laplacian(A) if hasattr(O,'compute_normalized_laplacian') else None
import scipy.sparse.csgraph as cg
L=cg.laplacian(A.astype(np.float32),normed=True)
L=sp.csr_matrix(L,dtype=np.float64)-sp.identity(A.shape[0],format="csr")
c=np.exp(-s*np.arange(K+1)); r=C.chebroots(c); alpha=c[-1]*2**(K-1)
quads=[];used=np.zeros(len(r),bool)
for i,z in enumerate(r):
    if used[i]: continue
    j=[k for k in range(len(r)) if not used[k] and k!=i and abs(r[k]-np.conj(z))<1e-9][0]
    used[i]=used[j]=True; quads.append((2*z.real,abs(z)**2))
def run(order, scale_each=True):
    v=X.astype(np.float64)
    # distribute alpha over factors
    f=alpha**(1.0/len(order))
    for (a,b) in order:
        w=(L@v).astype(np.float32).astype(np.float64)          # half 1: w = L v, stored fp32
        v=(L@w - a*w + b*v)*f                                   # half 2
        v=v.astype(np.float32).astype(np.float64)
    return v
def err(S): return np.max(np.abs(S-ref))/np.max(np.abs(ref))
print("natural", err(run(quads)))
print("reversed", err(run(quads[::-1])))
inter=[]; q=list(quads)
while q:
    inter.append(q.pop(0))
    if q: inter.append(q.pop(-1))
print("interleaved", err(run(inter)))
# forward chebyshev with fp32 storage for comparison
T0=X.astype(np.float64); T1=(L@T0).astype(np.float32).astype(np.float64); S=c[0]*T0+c[1]*T1
for k in range(2,K+1):
    T2=(2*(L@T1)-T0).astype(np.float32).astype(np.float64); S+=c[k]*T2; T0,T1=T1,T2
print("forward fp32 storage", err(S))
# greedy: keep the partial product's range on [-1,1] closest to p's scale
x=np.linspace(-1,1,401); pv=C.chebval(x,c)
f=alpha**(1.0/len(quads))
rem=list(quads); cur=np.ones_like(x); greedy=[]
for step in range(len(quads)):
    best=None
    for qd in rem:
        t=cur*(x*x-qd[0]*x+qd[1])*f
        score=np.max(np.abs(t))/np.min(np.abs(t))
        if best is None or score<best[0]: best=(score,qd)
    greedy.append(best[1]); rem.remove(best[1]); cur=cur*(x*x-best[1][0]*x+best[1][1])*f
Sg=run(greedy); print("greedy-ratio", err(Sg), [round(q[0],2) for q in greedy])
def elem(S):
    big=np.abs(ref)>1e-3*np.abs(ref).max()
    return np.max(np.abs(S-ref)[big]/np.abs(ref)[big])
Si=run(inter)
print("elementwise interleaved", elem(Si), "greedy", elem(Sg))
