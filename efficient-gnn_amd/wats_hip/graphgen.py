"""Synthetic graph inputs of the named sizes (host side, numpy).

The reference runs WATS on PyG/OGB datasets (Planetoid Cora, ogbn-arxiv,
Reddit; ``benchmark_calibration_methods.py:46-55``,
``exp/ablation/ugca_full_multi_dataset.py:61-148``) which cannot be downloaded
here, so benchmarks and parity tests use Graph500-style R-MAT graphs of the same
node/edge counts:

* R-MAT (a=.57, b=c=.19, d=.05) edges over ``2^ceil(log2 N)`` ids, a random
  vertex permutation, ids >= N rejected;
* symmetrised ``A + A^T``, clamped to 1, self loops removed (the ablation
  loaders' convention, ``ugca_full_multi_dataset.py:137-139``), optionally
  with self loops = 1 (the attack convention, ``ugca_calib_attack.py:42-47``);
* over-sampled until nnz is within +0..5 % of the target.

All outputs are canonical CSR (sorted column indices, no duplicates) with
int64 ``indptr`` and int32 ``indices``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# name -> (nodes, target nnz of the symmetrised off-diagonal adjacency, K, F)
NAMED_CONFIGS = {
    "cora": (2_708, 10_556, 8, 1),
    "pubmed": (19_717, 88_648, 16, 1),
    "ogbn-arxiv": (169_343, 2_315_598, 16, 40),
    "ogbn-arxiv-f1": (169_343, 2_315_598, 16, 1),
    "reddit": (232_965, 114_615_892, 16, 1),
    "reddit-f41": (232_965, 114_615_892, 16, 41),
    "rmat-8m": (8_388_608, 268_435_456, 32, 1),
}


@dataclass
class CSRGraph:
    """Host CSR adjacency (canonical, float32 values or None = all ones)."""
    n: int
    indptr: np.ndarray   # int64 (n+1,)
    indices: np.ndarray  # int32 (nnz,)
    values: np.ndarray | None = None  # float32 (nnz,) or None

    @property
    def nnz(self) -> int:
        return int(self.indptr[-1])

    def to_scipy(self):
        import scipy.sparse as sp
        vals = self.values if self.values is not None else np.ones(self.nnz, np.float32)
        return sp.csr_matrix((vals, self.indices, self.indptr), shape=(self.n, self.n))

    def stats(self) -> dict:
        deg = np.diff(self.indptr)
        rows = np.repeat(np.arange(self.n, dtype=np.int64), deg)
        offdiag = int(np.count_nonzero(rows != self.indices))
        return dict(n=self.n, nnz=self.nnz, nnz_offdiag=offdiag,
                    isolated=int(np.count_nonzero(deg == 0)),
                    max_degree=int(deg.max()) if self.n else 0)


def _rmat_edges(rng: np.random.Generator, scale: int, m: int, a=0.57, b=0.19, c=0.19):
    """Graph500 R-MAT endpoint bits, vectorised over m edges."""
    src = np.zeros(m, dtype=np.int64)
    dst = np.zeros(m, dtype=np.int64)
    ab = a + b
    c_norm = c / (1.0 - ab)
    a_norm = a / ab
    for lvl in range(scale):
        r1 = rng.random(m, dtype=np.float32)
        r2 = rng.random(m, dtype=np.float32)
        src_bit = r1 > ab
        dst_bit = np.where(src_bit, r2 > c_norm, r2 > a_norm)
        src |= src_bit.astype(np.int64) << lvl
        dst |= dst_bit.astype(np.int64) << lvl
    return src, dst


def coo_to_csr(n: int, src: np.ndarray, dst: np.ndarray, values=None) -> CSRGraph:
    """Build canonical CSR from (possibly duplicated) COO pairs; duplicate
    values are summed (``values=None`` -> pattern only, duplicates collapse)."""
    key = src.astype(np.int64) * n + dst.astype(np.int64)
    if values is None:
        key = np.unique(key)
        vals = None
    else:
        order = np.argsort(key, kind="stable")
        key = key[order]
        v = np.asarray(values, dtype=np.float64)[order]
        uniq, start = np.unique(key, return_index=True)
        vals = np.add.reduceat(v, start).astype(np.float32) if len(key) else np.zeros(0, np.float32)
        key = uniq
    rows = key // n
    cols = (key % n).astype(np.int32)
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=indptr[1:])
    return CSRGraph(n, indptr, cols, vals)


def rmat_graph(n: int, target_nnz: int, seed: int = 0, self_loops: bool = False,
               max_rounds: int = 64) -> CSRGraph:
    """Symmetrised, clamped R-MAT graph with ``n`` nodes and nnz (off-diagonal,
    both directions) within +0..5 % of ``target_nnz``."""
    rng = np.random.default_rng(seed)
    scale = max(1, math.ceil(math.log2(max(n, 2))))
    perm = rng.permutation(1 << scale)
    keys = np.zeros(0, dtype=np.int64)
    want = target_nnz
    m = max(16, int(target_nnz // 2 * 1.05))
    for _ in range(max_rounds):
        s, d = _rmat_edges(rng, scale, m)
        s = perm[s]
        d = perm[d]
        ok = (s < n) & (d < n) & (s != d)
        s, d = s[ok], d[ok]
        k1 = s * n + d
        k2 = d * n + s
        keys = np.unique(np.concatenate([keys, k1, k2]))
        have = keys.size
        if have >= want:
            break
        # estimate how many more raw edges are needed (duplicates make this sub-linear)
        gain = max(1.0, 2.0 * ok.sum() / max(1, m))
        m = max(16, int((want - have) / gain * 1.15) + 16)
    if keys.size > int(want * 1.05):
        # drop a random subset of undirected pairs to land inside +0..5 %
        rows = keys // n
        cols = keys % n
        upper = keys[rows < cols]
        n_pairs = int(math.ceil(want * 1.02 / 2))
        sel = rng.choice(upper.size, size=min(n_pairs, upper.size), replace=False)
        up = upper[sel]
        r, c = up // n, up % n
        keys = np.unique(np.concatenate([r * n + c, c * n + r]))
    rows = keys // n
    cols = keys % n
    if self_loops:
        diag = np.arange(n, dtype=np.int64)
        rows = np.concatenate([rows, diag])
        cols = np.concatenate([cols, diag])
    return coo_to_csr(n, rows, cols)


def named_graph(name: str, seed: int = 0) -> CSRGraph:
    n, nnz, _, _ = NAMED_CONFIGS[name]
    return rmat_graph(n, nnz, seed=seed)


def connect_isolated(g: CSRGraph, seed: int = 0) -> CSRGraph:
    """The same graph with every isolated node attached (both directions) to
    one uniformly random other node: an arxiv-shaped input with no
    closed-form rows (R-MAT at the ogbn-arxiv size leaves 44.6 % of the nodes
    isolated; the real ogbn-arxiv has none).  Unweighted graphs only."""
    if g.values is not None:
        raise ValueError("connect_isolated: unweighted graphs only")
    rng = np.random.default_rng(seed)
    deg = np.diff(g.indptr)
    iso = np.flatnonzero(deg == 0)
    if iso.size == 0 or g.n < 2:
        return g
    other = rng.integers(0, g.n - 1, size=iso.size)
    other = other + (other >= iso)            # never a self loop
    rows = np.repeat(np.arange(g.n, dtype=np.int64), deg)
    src = np.concatenate([rows, iso, other])
    dst = np.concatenate([g.indices.astype(np.int64), other, iso])
    return coo_to_csr(g.n, src, dst)


def random_graph(n: int, p: float, seed: int = 0, directed: bool = True, weighted: bool = False,
                 self_loop_frac: float = 0.0, isolated_frac: float = 0.0) -> CSRGraph:
    """Small Erdos-Renyi-style graph with optional weights / self loops /
    forced isolated nodes -- the edge cases the reference's scipy path handles."""
    rng = np.random.default_rng(seed)
    m = rng.binomial(n * n, p) if n else 0
    src = rng.integers(0, n, size=m) if n else np.zeros(0, np.int64)
    dst = rng.integers(0, n, size=m) if n else np.zeros(0, np.int64)
    if not directed:
        src, dst = np.concatenate([src, dst]), np.concatenate([dst, src])
    keep = src != dst
    src, dst = src[keep], dst[keep]
    if self_loop_frac > 0 and n:
        loops = rng.choice(n, size=max(1, int(n * self_loop_frac)), replace=False)
        src = np.concatenate([src, loops])
        dst = np.concatenate([dst, loops])
    if isolated_frac > 0 and n:
        iso = rng.choice(n, size=max(1, int(n * isolated_frac)), replace=False)
        bad = np.isin(src, iso) | np.isin(dst, iso)
        src, dst = src[~bad], dst[~bad]
    g = coo_to_csr(n, src, dst)
    if weighted:
        g.values = rng.uniform(0.1, 2.0, size=g.nnz).astype(np.float32)
        if not directed:
            # keep weights symmetric: w_ij = w_ji
            A = g.to_scipy()
            A = ((A + A.T) * 0.5).tocsr()
            A.sort_indices()
            g = CSRGraph(n, A.indptr.astype(np.int64), A.indices.astype(np.int32),
                         A.data.astype(np.float32))
    return g


def rmat_graph_device(n: int, target_nnz: int, seed: int = 0, device="cuda", max_rounds: int = 16):
    """R-MAT graph generated on the GPU with torch ops (same recipe as
    :func:`rmat_graph`: a=.57, b=c=.19, random vertex permutation, ids >= n
    rejected, symmetrised, clamped to 1, no self loops, nnz within +0..5 %
    of the target).  Deterministic for a given seed, so every rank of a
    sharded run builds the identical graph.  Used for the Reddit / 8M R-MAT
    sizes, where the numpy generator takes minutes.  Returns
    (indptr int64, indices int32) device tensors.
    (Not bit-identical to the numpy generator: a different random stream.)"""
    import torch
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    scale = max(1, math.ceil(math.log2(max(n, 2))))
    perm = torch.randperm(1 << scale, generator=gen, device=device)
    a, b, c = 0.57, 0.19, 0.19
    ab = a + b
    c_norm = c / (1.0 - ab)
    a_norm = a / ab
    keys = torch.zeros(0, dtype=torch.int64, device=device)
    m = max(16, int(target_nnz // 2 * 1.05))
    for _ in range(max_rounds):
        src = torch.zeros(m, dtype=torch.int64, device=device)
        dst = torch.zeros(m, dtype=torch.int64, device=device)
        for lvl in range(scale):
            r1 = torch.rand(m, generator=gen, device=device)
            r2 = torch.rand(m, generator=gen, device=device)
            sb = r1 > ab
            db = torch.where(sb, r2 > c_norm, r2 > a_norm)
            src |= sb.to(torch.int64) << lvl
            dst |= db.to(torch.int64) << lvl
        src, dst = perm[src], perm[dst]
        ok = (src < n) & (dst < n) & (src != dst)
        src, dst = src[ok], dst[ok]
        keys = torch.unique(torch.cat([keys, src * n + dst, dst * n + src]))
        del src, dst, ok
        if keys.numel() >= target_nnz:
            break
        m = max(16, int((target_nnz - keys.numel()) / 2 * 1.3) + 16)
    if keys.numel() > int(target_nnz * 1.05):
        rows, cols = keys // n, keys % n
        upper = keys[rows < cols]
        n_pairs = int(math.ceil(target_nnz * 1.02 / 2))
        sel = torch.randperm(upper.numel(), generator=gen, device=device)[:n_pairs]
        up = upper[sel]
        r, cc = up // n, up % n
        keys = torch.unique(torch.cat([r * n + cc, cc * n + r]))
    rows = keys // n
    cols = (keys % n).to(torch.int32)
    counts = torch.bincount(rows, minlength=n)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return indptr, cols
