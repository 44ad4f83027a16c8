"""Generate golden vectors for the WATS graph-wavelet path FROM THE REFERENCE.

Run only in the build container, where the reference is mounted read-only at
/root/reference:

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py

It imports ``calibration/WATS.py`` (and, for the forward fixture,
``src/gnn/model.py``) through a stub package so that only those files execute
(``calibration/__init__.py`` pulls in seaborn / torch_geometric, which are not
installed -- SURVEY.md section 8(c)).  Outputs are DATA only: input graphs,
signals and the reference's outputs, written as ``tests/golden/*.npz`` plus
``tests/golden/manifest.json`` (versions, seeds, sha256).  Nothing of the
reference's source travels with the fixtures.
"""
from __future__ import annotations

import hashlib
import importlib
import importlib.util
import json
import os
import sys
import types

import numpy as np
import scipy
import scipy.sparse as sp
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))

from wats_hip.graphgen import CSRGraph, random_graph, rmat_graph  # noqa: E402


def import_reference():
    pkg = types.ModuleType("calibration")
    pkg.__path__ = [os.path.join(REF, "calibration")]
    sys.modules["calibration"] = pkg
    W = importlib.import_module("calibration.WATS")
    spec = importlib.util.spec_from_file_location("ref_gnn_model", os.path.join(REF, "src", "gnn", "model.py"))
    M = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(M)
    return W, M


def csr_of(A) -> sp.csr_matrix:
    A = sp.csr_matrix(A, dtype=np.float32)
    A.sort_indices()
    return A


def save(name: str, manifest: dict, **arrays):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    with open(path, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    manifest["files"][name + ".npz"] = dict(sha256=digest, keys=sorted(arrays.keys()))
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def ref_case(W, A: sp.csr_matrix, k: int, s: float, X0=None, keep_T=True, keep_L=True):
    """Run the reference functions on A.  With X0=None the reference's own
    composite ``graph_wavelet_features(A, k, s)`` is also called and its H
    stored as ``H_ref_fn`` (it only supports the built-in signal)."""
    n = A.shape[0]
    L = W.compute_normalized_laplacian(A)
    L_resc = (2 / 2.0) * L - sp.identity(n)          # WATS.py:55 (composition step)
    if X0 is None:
        degrees = np.array(A.sum(axis=1)).flatten()  # WATS.py:58-59
        X0 = np.log1p(degrees).reshape(-1, 1)
        H_fn = W.graph_wavelet_features(A, k=k, s=s)
    else:
        H_fn = None
    T = W.chebyshev_polynomials(L_resc, k, X0)
    alpha = [np.exp(-s * i) for i in range(k + 1)]   # WATS.py:65-72 (composition step)
    S = sum(alpha[i] * T[i] for i in range(k + 1))
    row_sums = np.linalg.norm(S, ord=1, axis=1, keepdims=True) + 1e-8
    H = S / row_sums
    out = dict(indptr=A.indptr.astype(np.int64), indices=A.indices.astype(np.int32),
               values=A.data.astype(np.float32), n=np.int64(n), k=np.int64(k), s=np.float64(s),
               X0=np.asarray(X0, dtype=np.float32), S=np.asarray(S, np.float64),
               H=np.asarray(H, np.float64))
    if H_fn is not None:
        out["H_ref_fn"] = np.asarray(H_fn, np.float64)
    if keep_T:
        out["T"] = np.stack([np.asarray(t, np.float64) for t in T])
    if keep_L:
        Lc = sp.csr_matrix(L_resc)
        Lc.sort_indices()
        out["L_indptr"] = Lc.indptr.astype(np.int64)
        out["L_indices"] = Lc.indices.astype(np.int32)
        out["L_values"] = Lc.data.astype(np.float64)
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    W, M = import_reference()
    manifest = dict(generator="tools/gen_golden.py", reference="/root/reference calibration/WATS.py (2026-02-06)",
                    numpy=np.__version__, scipy=scipy.__version__, torch=torch.__version__, files={})

    # 1. 4-node edge-case KAT: self loop, directed edge,
    #    in-degree-0 node, isolated node.
    A4 = csr_of(np.array([[1, 1, 0, 0], [1, 0, 1, 0], [0, 0, 0, 0], [0, 0, 1, 0]], np.float32))
    for k in (0, 1, 2, 3):
        save(f"kat4_k{k}", manifest, **ref_case(W, A4, k, 0.8))

    # 2. Zachary karate club (networkx built-in), K=3 and K=8
    import networkx as nx
    Ak = csr_of(nx.to_scipy_sparse_array(nx.karate_club_graph(), weight=None, dtype=np.float32))
    for k in (3, 8):
        save(f"karate_k{k}", manifest, **ref_case(W, Ak, k, 0.8))

    # 3. Cora-size R-MAT, harness convention (no self loops), K=8 (config 0) and K=3 (WATS default)
    g = rmat_graph(2708, 10556, seed=0)
    Ac = csr_of(g.to_scipy())
    save("cora_rmat_k8", manifest, **ref_case(W, Ac, 8, 0.8, keep_L=False))
    save("cora_rmat_k3", manifest, **ref_case(W, Ac, 3, 0.8, keep_L=False))

    # 4. attack convention: symmetrised + self loops = 1 (ugca_calib_attack.py:42-47)
    g = rmat_graph(500, 4000, seed=3, self_loops=True)
    Aa = csr_of(g.to_scipy())
    for k in (3, 16):
        save(f"attack500_k{k}", manifest, **ref_case(W, Aa, k, 0.8))

    # 5. directed, weighted, self loops and isolated nodes (exercises column-sum
    #    degree != row-sum degree, w==0 handling and float32 divisions)
    g = random_graph(300, 0.02, seed=5, directed=True, weighted=True, self_loop_frac=0.1, isolated_frac=0.05)
    Ad = csr_of(g.to_scipy())
    for k in (1, 5):
        save(f"directed_weighted300_k{k}", manifest, **ref_case(W, Ad, k, 0.8))
    # weighted symmetric, different heat scale
    g = random_graph(200, 0.05, seed=6, directed=False, weighted=True, isolated_frac=0.1)
    Aw = csr_of(g.to_scipy())
    save("sym_weighted200_k6_s05", manifest, **ref_case(W, Aw, 6, 0.5))

    # 6. multi-column signal (F=3 and F=40) through the reference recurrence
    rng = np.random.default_rng(1)
    X3 = rng.standard_normal((Ak.shape[0], 3)).astype(np.float32)
    save("karate_f3_k4", manifest, **ref_case(W, Ak, 4, 0.8, X0=X3))
    g = rmat_graph(1000, 8000, seed=7)
    Ar = csr_of(g.to_scipy())
    X40 = rng.standard_normal((1000, 40)).astype(np.float32)
    save("rmat1000_f40_k16", manifest, **ref_case(W, Ar, 16, 0.8, X0=X40, keep_T=False, keep_L=False))
    X40k = rng.standard_normal((Ak.shape[0], 40)).astype(np.float32)
    save("karate_f40_k16", manifest, **ref_case(W, Ak, 16, 0.8, X0=X40k))

    # 7. PubMed-size, K=16 (config 1), F=1: S and H only
    g = rmat_graph(19717, 88648, seed=0)
    Ap = csr_of(g.to_scipy())
    save("pubmed_rmat_k16", manifest, **ref_case(W, Ap, 16, 0.8, keep_T=False, keep_L=False))

    # 8. degenerate graphs: no edges at all, single node, single self loop
    save("empty10_k3", manifest, **ref_case(W, csr_of(np.zeros((10, 10), np.float32)), 3, 0.8))
    save("single_k3", manifest, **ref_case(W, csr_of(np.zeros((1, 1), np.float32)), 3, 0.8))
    save("selfloop1_k3", manifest, **ref_case(W, csr_of(np.ones((1, 1), np.float32)), 3, 0.8))

    # 9. WATS forward fixture: reference WATS constructed on CPU on a small graph,
    #    its trained temperature head + base model weights + forward output.
    torch.manual_seed(42)
    np.random.seed(42)
    n, nfeat, ncls = 120, 16, 4
    g = rmat_graph(n, 600, seed=11)
    adj = torch.tensor(g.to_scipy().toarray(), dtype=torch.float32)
    x = torch.randn(n, nfeat)
    y = torch.randint(0, ncls, (n,))
    val_mask = torch.zeros(n, dtype=torch.bool)
    val_mask[::3] = True
    base = M.CompatibleGCN(nfeat=nfeat, nclass=ncls, nhid=32, dropout=0.5)
    base.eval()
    for p in base.parameters():
        p.requires_grad = False
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        wats = W.WATS(base, x, y, adj, val_mask)
    wats.eval()
    with torch.no_grad():
        out = wats(x, adj)
    arrays = dict(adj=adj.numpy(), x=x.numpy(), y=y.numpy(), val_mask=val_mask.numpy(),
                  wavelet_feats=wats.wavelet_feats.cpu().numpy(), out=out.numpy())
    for name, t in base.state_dict().items():
        arrays["base." + name] = t.cpu().numpy()
    for name, t in wats.net.state_dict().items():
        arrays["net." + name] = t.cpu().numpy()
    save("wats_forward120", manifest, **arrays)

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("manifest written")


if __name__ == "__main__":
    main()
