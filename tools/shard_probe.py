"""Time one rank's shard of a row-sharded graph on one GPU (run on the GPU box):
the per-step compute a rank of an N-GPU run does, without the exchange.

    python tools/shard_probe.py --config reddit --world 8 [--rank 0] [--lds 3]
"""
import argparse
import ctypes
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import wats_hip  # noqa: E402
from wats_hip import _lib  # noqa: E402
from wats_hip._lib import check, ptr  # noqa: E402
from wats_hip.dist import partition_rows  # noqa: E402
from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="reddit")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--ranks", default="", help="comma-separated ranks to probe one after another (one graph)")
    ap.add_argument("--lds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--F", type=int, default=1, help="signal width (F > 1: the gather kernel at this width)")
    ap.add_argument("--groups", type=int, default=1, help="hand the degree-ordered halo groups to the handle "
                                                          "(the F = 1 hub kernel applies to the shard)")
    ap.add_argument("--clen", type=int, default=1, help="F > 1: the value-free Clenshaw step of the sharded chain "
                                                       "(wg_clenshaw_step; the hybrid step where it applies); 0 = wg_cheb_step")
    ap.add_argument("--grid", default="", help="';'-separated knob sets to time, e.g. 'lds_wg=64;lds_wg=128,lds_k=2'")
    a = ap.parse_args()
    n, nnz_t, K, _ = NAMED_CONFIGS[a.config]
    dev = torch.device("cuda", 0)
    ip, ix = rmat_graph_device(n, nnz_t, seed=0, device=dev)
    indptr = ip.cpu().numpy()
    deg = np.diff(indptr).astype(np.float32)
    b = partition_rows(indptr, a.world)
    for rk in ([int(x) for x in a.ranks.split(",")] if a.ranks else [a.rank]):
        a.rank = rk
        one_rank(a, b, ip, ix, indptr, deg, dev, K)


def one_rank(a, b, ip, ix, indptr, deg, dev, K):
    L, n_own, n_cols = build_shard(a, b, ip, ix, indptr, deg, dev)
    lib = _lib.load()
    for knobs in (a.grid.split(";") if a.grid else [""]):
        kv = dict(lds=a.lds)
        kv.update({x.split("=")[0]: int(x.split("=")[1]) for x in knobs.split(",") if x})
        L.tune(**kv)
        probe(L, lib, n_own, n_cols, K, a, dev, kv)
    L.close()
    torch.cuda.empty_cache()


def build_shard(a, b, ip, ix, indptr, deg, dev):
    """Rank a.rank's shard as wats_hip.dist builds it; returns (handle, own rows, columns)."""
    r0, r1 = int(b[a.rank]), int(b[a.rank + 1])
    cols = ix[int(indptr[r0]):int(indptr[r1])].to(torch.int64)
    # the shard as wats_hip.dist builds it: [own | halo], halo grouped by owner, each group in
    # descending degree (build_halo_plan with col_degree), group offsets handed to the handle
    plan_bounds = np.asarray(b)
    own = (cols >= r0) & (cols < r1)
    halo_sorted = torch.unique(cols[~own], sorted=True).cpu().numpy()
    owner_sorted = np.searchsorted(plan_bounds, halo_sorted, side="right") - 1
    order = np.lexsort((halo_sorted, -deg[halo_sorted].astype(np.float64), owner_sorted))
    rank_of = np.empty(halo_sorted.size, np.int64)
    rank_of[order] = np.arange(halo_sorted.size)
    local = cols - r0
    local[~own] = (r1 - r0) + torch.from_numpy(rank_of).to(dev)[
        torch.searchsorted(torch.from_numpy(halo_sorted).to(dev), cols[~own])]
    halo = halo_sorted[order]
    counts = np.bincount(owner_sorted[order], minlength=a.world)
    n_own, n_cols = r1 - r0, (r1 - r0) + int(halo.size)
    w = torch.from_numpy(np.concatenate([deg[r0:r1], deg[halo]]))
    L = wats_hip.NormalizedLaplacian(n_own, torch.from_numpy(indptr[r0:r1 + 1] - indptr[r0]),
                                     local.to(torch.int32), None, n_cols=n_cols, w_cols=w, device=dev)
    if a.groups and a.world > 1:
        offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        check(_lib.load().wg_laplacian_set_halo_groups(L.handle, a.world, offs.ctypes.data), "set_halo_groups")
    del cols, local
    return L, n_own, n_cols


def probe(L, lib, n_own, n_cols, K, a, dev, kv):
    st = torch.cuda.current_stream().cuda_stream
    ulen = ctypes.c_int64(0)
    check(lib.wg_cheb_u_len(L.handle, ctypes.byref(ulen)), "u_len")
    print(f"shard {a.rank}/{a.world}: rows {n_own}, cols {n_cols}, nnz {L.nnz}, u_len {ulen.value}", flush=True)
    T = [torch.rand(n_own, device=dev) for _ in range(3)]
    S = torch.zeros(n_own, device=dev)
    if a.F > 1:
        F = a.F
        X = [torch.rand(n_cols, F, device=dev), torch.rand(n_own, F, device=dev), torch.rand(n_own, F, device=dev)]
        SF = torch.zeros(n_own, F, device=dev)
        if a.clen:
            flags = 1 | 2 | 4   # WG_CLEN_UIN | UPREV | UOUT: b1 (own + halo rows of u), b2 = u, out = u over b2
            run = lambda k: check(lib.wg_clenshaw_step(L.handle, F, ptr(X[0]), ptr(X[1]), ptr(X[2]), ptr(X[1]), 0.3,
                                                       2.0, flags, st), "clenshaw_step")
            info = f"value-free Clenshaw step F={F}; " + "; ".join(ln for ln in L.describe(F).splitlines()
                                                                      if ln.startswith("tiles:"))
        else:
            run = lambda k: L.step(k, X[0], X[1], X[2], S=SF, alpha0=1.0, alpha_k=math.exp(-0.8 * k))
            info = f"gather kernel F={F}"
    elif ulen.value:
        U = [torch.rand(ulen.value, device=dev) for _ in range(2)]
        run = lambda k: check(lib.wg_cheb_step_u(L.handle, k, ptr(U[0]), ptr(T[0]), ptr(T[1]), ptr(T[2]), ptr(U[1]),
                                                 ptr(S), 1.0, math.exp(-0.8 * k), st), "step_u")
        info = L.lds_plan_info(active_only=False)
    else:
        X = [torch.rand(n_cols, 1, device=dev), torch.rand(n_own, 1, device=dev), torch.rand(n_own, 1, device=dev)]
        run = lambda k: L.step(k, X[0], X[1], X[2], S=S.view(-1, 1), alpha0=1.0, alpha_k=math.exp(-0.8 * k))
        info = None
    for k in range(2, 6):
        run(k)
    torch.cuda.synchronize()
    if a.F > 1 and a.clen:   # the plan text once the first step has built it
        info = f"value-free Clenshaw step F={a.F}; " + "; ".join(ln for ln in L.describe(a.F).splitlines()
                                                                  if ln.startswith("tiles:"))
    L.profile_enable(True)
    for _ in range(a.reps):
        for k in range(2, K + 1):
            run(k)
    p = L.profile_collect()
    L.profile_enable(False)
    print(f"{kv}: step kernel(s) {p['sum_ms'] / p['launches'] * 1e3:.2f} us per step (plan {info})", flush=True)


if __name__ == "__main__":
    main()
