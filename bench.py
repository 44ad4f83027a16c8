#!/usr/bin/env python3
"""Benchmark: Chebyshev SpMM-chain edges*K/s on MI355X (BASELINE.json metric).

One "step" = one full ``graph_wavelet_features`` pass (reference
calibration/WATS.py:39-74) over a device-resident graph: permute the signal
into the internal order, K fused SpMM steps evaluating S = sum_k alpha_k
T_k(L_hat) X0 by Clenshaw's recurrence (value-free gathers on
an unweighted graph), the last one writing S / H in caller order.  The Laplacian
prologue (a1-a3) is built once before timing, as the reference builds it once
per WATS construction.

Headline workload by GPU count (BASELINE.json configs):
  N = 1  configs[2], the one the metric is quoted on: ogbn-arxiv-size synthetic
         R-MAT graph (N=169,343, nnz~2.32M symmetrised), K=16, F=40
         random-normal signal columns, s=0.8.
  N > 1  configs[3]: the Reddit-size graph (232,965 nodes / 114.6M nonzeros),
         K=16, F=41 (the 41-class logit-shaped RHS of SURVEY 8(d)), ONE graph
         row-sharded over the N ranks (nnz-balanced row blocks, [own | halo]
         columns) with a halo exchange per Chebyshev step -- strong scaling.
         Exchange (--exchange ipc,rccl,sdma, --pick-exchange 1): the headline
         is timed with the one-sided IPC pull AND with RCCL grouped
         ncclSend/ncclRecv (north_star's all-to-all-v, each peer's rows straight
         into the halo), and the line is the FASTER of the two whose check
         passed (both attached; an RCCL error or hang falls back to IPC on every
         rank); the peer-DMA exchange (sdma) is timed beside them.  So the N > 1
         line may well be the IPC pull, not RCCL: whichever measured faster on
         that node.  The same Reddit run at one
         rank is the N = 1 line's `sharded` object, so the Reddit curve is
         complete across the driver's 1/2/4/8 lines.
value = total edges*K processed by all ranks / max-over-ranks wall time, where
edges = nnz of the off-diagonal L_hat (= symmetrised adjacency without loops).

Also printed in the same JSON line:
  roofline      -- SURVEY.md 8(d)'s algorithmic bytes per launch (B_step =
                   8 nnz + 4 (N+1) + 20 N F over the launched rows) / the step
                   kernel's mean duration from HIP events recorded live around
                   every step launch; kernel_bytes_frac: the fewer bytes the
                   kernel's own algorithm needs (clenshaw_bytes);
  cpu_baseline  -- the oracle (scipy/numpy restatement of the reference, one
                   thread) on the same graph, rank 0 at N=1 only; its `check`
                   compares the benchmarked pass's S (all columns) with the C
                   restatement of the oracle (oracle/wats_chain.c);
  sharded runs  -- `check`: every rank's rows of S for a random signal against
                   the unsharded chain on the same GPU (max over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "efficient-gnn_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
CHECK_TOL = 1e-5       # north_star: <= 1e-5 relative (max|dS| / max|S| per column)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-s", type=float, default=0.5,
                    help="seconds of untimed passes after the W warmup passes (clock ramp); reported as settle_s")
    ap.add_argument("--config", default="ogbn-arxiv", help="the N = 1 headline workload")
    ap.add_argument("--scale-config", default="reddit-f41",
                    help="the N > 1 headline: this config row-sharded over all ranks (strong scaling)")
    ap.add_argument("--K", type=int, default=None)
    ap.add_argument("--F", type=int, default=None)
    ap.add_argument("--s", type=float, default=0.8)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--traffic-json", default="auto",
                    help="per-launch HBM bytes of the step kernel from a rocprofv3 --pmc pass (tools/pmc_traffic.py); "
                         "'auto': the committed PMC summary of the default workload (profiles/r06/s13_traffic.json, "
                         "tools/pmc_legs.sh arxiv + tools/traffic_json.py) when the workload is the default one; 'none' to omit")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--sharded-extra", default="reddit-f41,reddit,rmat-8m,ogbn-arxiv",
                    help="comma-separated configs also measured row-sharded over all ranks (halo exchange), attached "
                         "as 'sharded' (first) and 'sharded_<config>' objects of the line; 'none' to skip.  At N > 1 "
                         "the --scale-config run is the headline and is not repeated here")
    ap.add_argument("--sharded-steps", type=int, default=5)
    ap.add_argument("--headline-timeout", type=float, default=900.0,
                    help="N > 1: seconds the row-sharded headline may take before an error line is printed")
    ap.add_argument("--sharded-timeout", type=float, default=420.0,
                    help="seconds the extras may take before the line is printed without the unfinished ones")
    ap.add_argument("--exchange", default="ipc,rccl,sdma",
                    help="comma-separated sharded halo exchanges: native chain with grouped ncclSend/ncclRecv "
                         "(rccl), the one-sided IPC pull (ipc), packed blocks copied by peer DMA (sdma), or torch "
                         "all_to_all_single per step (nccl); the "
                         "first is the headline's (N > 1) and the extras'; the others are timed for the first "
                         "sharded config only, as 'sharded_<config>_<exchange>'")
    ap.add_argument("--pick-exchange", type=int, default=1,
                    help="N > 1: time the headline with the first two --exchange kinds and report the faster "
                         "(both attached)")
    ap.add_argument("--cold-reps", type=int, default=5,
                    help="chains timed after writing a 512 MiB scratch buffer (cold Infinity Cache / L2); 0 = skip")
    ap.add_argument("--f1-companion", type=int, default=1,
                    help="also time the same graph with the F=1 log1p-degree signal (SURVEY 8(d) 'also report F=1')")
    ap.add_argument("--connected-companion", type=int, default=1,
                    help="N = 1: also time an arxiv-shaped graph without isolated rows (graphgen.connect_isolated)")
    ap.add_argument("--pubmed-companion", type=int, default=1,
                    help="N = 1: also time the PubMed-size K=16 F=1 chain (BASELINE configs[1], launch-bound)")
    ap.add_argument("--replicas", type=int, default=1,
                    help="N > 1: also time one independent arxiv-size graph per rank (no collective) as 'replicas'")
    ap.add_argument("--mode", default="auto", choices=["auto", "graphs", "sharded"],
                    help="auto: graphs at N = 1, sharded (--scale-config) at N > 1; graphs: one independent graph "
                         "per rank; sharded: --config row-sharded over all ranks")
    return ap.parse_args()


def algorithmic_bytes(n: int, nnz: int, F: int) -> int:
    """CSR indices+values 8 B/nnz, int32 row pointers, read
    T_{k-1} once, read T_{k-2}, write T_k, read+write S (fp32)."""
    return 8 * nnz + 4 * (n + 1) + 20 * n * F


def clenshaw_bytes(n: int, nnz: int, F: int, unit: bool = False) -> int:
    """The wavelet chain's heat sum by Clenshaw's recurrence:
    CSR 8 B/nnz, int32 row pointers, gather b_{k+1} once, read b_{k+2} and X0,
    write b_k (fp32) -- no S stream.  On an unweighted graph (`unit`) the chain
    carries u = b * dinv and reads no CSR values: 4 B/nnz plus the float64
    dinv of each row.  Reported as kernel_bytes_frac beside the roofline's
    SURVEY 8(d) forward-recurrence model (algorithmic_bytes)."""
    if unit:
        return 4 * nnz + 4 * (n + 1) + 16 * n * F + 8 * n
    return 8 * nnz + 4 * (n + 1) + 16 * n * F


def _byte_model(info) -> str:
    if not info:
        return "SURVEY 8(d)"
    if info["mode"] == 4:
        return "hub teams (int32 ids, no values; DESIGN.md 4.5)"
    return "lds (16-bit ids, no values; DESIGN.md 4.4)"


def lds_kernel_name(info, chain1: bool = False, team: bool = False) -> str:
    if chain1:
        return "cheb_chain1_kernel (the whole chain in one launch; per-step time = launch / K)"
    if not info:
        return "cheb_team4_kernel" if team else "cheb_step_kernel"
    return {1: "cheb_lds1_kernel", 2: "cheb_lds3_kernel + combine_lds2_kernel",
            4: "cheb_hub1_kernel"}.get(info["mode"], "lds mode %d" % info["mode"])


def lds_algorithmic_bytes(info: dict) -> int:
    """Bytes one step of the F == 1 column-blocked LDS kernel must move
    (its entries carry 16-bit column ids and no values):
    ids 2 B/nnz; float32 block partials written + read (8 B per non-empty
    (row, block) segment); segment map 4 B per (block, row); per row: T_{k-1}
    (isolated diagonal), T_{k-2}, T_k, u_k = T_k*dinv (4 B each), S read+write
    (8 B), dinv (8 B, float64), iso (1 B); the gathered u read once (4 B/column;
    the per-workgroup LDS fills are L2 hits).  Chunk padding is excluded here
    (it is real traffic, visible in the PMC `traffic`)."""
    n, nb, nnz, segs, cols = info["rows"], info["blocks"], info["nnz"], info["segments"], info["cols"]
    if info["mode"] == 4:   # hub teams: the operator's int32 columns and row pointers, no values
        return 4 * nnz + 4 * (n + 1) + 33 * n + 4 * cols
    if info["mode"] == 2:
        return 2 * nnz + 8 * segs + 4 * nb * n + 33 * n + 4 * cols
    return 2 * nnz + 4 * (nb * n + 1) + (8 * nb * n if nb > 1 else 0) + 33 * n + 4 * cols


def cpu_baseline(g, K, F, s, X, seconds, S_gpu):
    """The reference's CPU path, restated (oracle/wats_oracle.py: scipy
    csgraph.laplacian + single-threaded sparsetools CSR mat-vecs, as
    WATS.py:53-72 runs), timed on a bounded sample of passes; then the parity
    check of the benchmarked pass: S_gpu (all columns) against the C
    restatement of the oracle (oracle/wats_chain.c, 16 threads)."""
    from oracle import wats_oracle as O
    from oracle import wats_oracle_c as C
    A = g.to_scipy()
    t0 = time.perf_counter()
    L_hat = O.rescaled_laplacian(A)  # prologue: outside the chain's time (as on the GPU), reported
    prologue_s = time.perf_counter() - t0
    nnz = int(L_hat.nnz - np.count_nonzero(L_hat.diagonal()))
    reps, t_total = 0, 0.0
    while t_total < seconds and reps < 50:
        t0 = time.perf_counter()
        T = O.chebyshev_polynomials(L_hat, K, X)
        S = O.heat_kernel_combine(T, s)
        O.row_l1_normalize(np.asarray(S))
        t_total += time.perf_counter() - t0
        reps += 1
        del T, S
    out = dict(value=nnz * K * reps / t_total, unit="edges*K/s", cores=1, kind="port", prologue_s=prologue_s,
               sample=f"{reps} full graph_wavelet_features passes (chain + heat sum + L1 norm, prologue excluded) "
                      f"of the same graph/signal, scipy {__import__('scipy').__version__} single-threaded CSR "
                      f"matvecs, {t_total:.1f} s")
    t0 = time.perf_counter()
    S_ref, _ = C.graph_wavelet_features(g.indptr, g.indices, g.values, X, K, s, threads=16, return_H=False)
    t_c = time.perf_counter() - t0
    # a second CPU figure beside the reference's own (single-threaded scipy) path: the C
    # restatement (float64, OpenMP over rows, 16 threads = the box's CPU share) on the same pass
    out["c_oracle_16_threads"] = {"value": nnz * K / t_c, "unit": "edges*K/s", "cores": 16, "seconds": t_c,
                                  "what": "oracle/wats_chain.c: the same pass (its own Laplacian build included, chain, heat sum, L1 norm), "
                                          "float64, rows split over 16 OpenMP threads"}
    err = _rel_err(S_gpu, S_ref)
    out["check"] = {"max_rel_err": err, "tol": CHECK_TOL, "ok": bool(err <= CHECK_TOL),
                    "what": f"the benchmarked pass's S (all {F} columns, this signal) vs the C restatement of the "
                            f"oracle (oracle/wats_chain.c, float64, {time.perf_counter() - t0:.1f} s on 16 threads); "
                            f"max over columns of max|dS| / max|S|"}
    return out


def _rel_err(got, ref) -> float:
    got = np.asarray(got, np.float64).reshape(ref.shape)
    scale = np.abs(ref).max(axis=0)
    err = np.abs(got - ref).max(axis=0)
    ok = scale > 0
    return float((err[ok] / scale[ok]).max()) if ok.any() else float(err.max(initial=0.0))


# ----------------------------------------------------------------------------- row-sharded runs
_GRAPHS: dict = {}


def shared_graph(config, seed, world, rank, device):
    """The row-sharded runs' graph (GPU R-MAT generator), generated ONCE, by
    rank 0, and broadcast to every rank: (indptr int64, indices int32) on this
    rank's device, cached per (config, seed).  Ranks used to generate it each
    for themselves; with several ranks on ONE device (the one-GPU rehearsal of
    the N > 1 bench) the concurrent generators sat in torch.unique's radix sort
    for minutes (profiles/r03/s49_rehearse, DESIGN.md 7: its onesweep passes
    spin on their predecessors' look-back, and kernels of several processes
    time-share one device's queues), so no rank depends on that any more."""
    key = (config, seed)
    if key in _GRAPHS:
        return _GRAPHS[key]
    from wats_hip.graphgen import NAMED_CONFIGS, rmat_graph_device
    n_t, nnz_t = NAMED_CONFIGS[config][:2]
    if world == 1:
        ip, ix = rmat_graph_device(n_t, nnz_t, seed=seed, device=device)
    else:
        on = device if dist.get_backend() == "nccl" else torch.device("cpu")
        size = torch.zeros(1, dtype=torch.int64, device=on)
        if rank == 0:
            ip, ix = rmat_graph_device(n_t, nnz_t, seed=seed, device=device)
            size[0] = ix.numel()
            ip, ix = ip.to(on), ix.to(on)
        dist.broadcast(size, 0)
        if rank != 0:
            ip = torch.empty(n_t + 1, dtype=torch.int64, device=on)
            ix = torch.empty(int(size.item()), dtype=torch.int32, device=on)
        dist.broadcast(ip, 0)
        dist.broadcast(ix, 0)
        ip, ix = ip.to(device), ix.to(device)
        _log(f"graph {config}: {ix.numel()} nonzeros generated on rank 0, broadcast to {world} ranks")
    _GRAPHS[key] = (ip, ix)
    return ip, ix


def run_sharded(config, K, F, steps, warmup, seed, s_heat, world, rank, device, exchange="rccl",
                median_reps: int = 0, check: bool = True, min_time: float = 0.0):
    """One graph (generated identically on every rank, on the GPU) split into
    nnz-balanced row blocks; per Chebyshev step one halo exchange (`exchange`:
    RCCL send/recv or IPC pull in the native chain, or torch
    all_to_all_single) + the step kernel.  Strong scaling (fixed graph).
    Returns the result dict (meaningful on rank 0)."""
    from wats_hip import NormalizedLaplacian, graph_wavelet_features
    from wats_hip.dist import ShardedWavelet, partition_rows
    from wats_hip.graphgen import NAMED_CONFIGS

    n_t, nnz_t, K_def, F_def = NAMED_CONFIGS[config]
    K = K if K is not None else K_def
    F = F if F is not None else F_def
    _log(f"sharded {config} ({exchange}): generating")
    indptr_d, indices_d = shared_graph(config, seed, world, rank, device)
    indptr = indptr_d.cpu().numpy()
    _log(f"sharded {config} ({exchange}): generated; building the shard")
    bounds = partition_rows(indptr, world)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    lo, hi = int(indptr[r0]), int(indptr[r1])
    cols = indices_d[lo:hi].cpu().numpy()
    nnz_global = int(indptr[-1])
    torch.cuda.empty_cache()
    with _stdout_to_stderr():   # RCCL prints its version banner at communicator init: keep stdout one JSON line
        sw = ShardedWavelet(indptr[r0:r1 + 1] - lo, cols, None, n_t, bounds, exchange=exchange, device=device,
                            max_features=F)
    if F == 1:
        X = sw.L.log1p_degree()
    else:
        g = torch.Generator(device=device)
        g.manual_seed(1 + rank)
        X = torch.randn(r1 - r0, F, generator=g, device=device)
    out = (torch.empty(r1 - r0, F, device=device), torch.empty(r1 - r0, F, device=device))
    if exchange in ("rccl", "ipc", "sdma") and sw._dist is not None:
        # the signal already in the chain's input buffer (as graph_wavelet_features reads the
        # caller's X0 in place): no per-chain copy into it
        xb = sw._buf("X", r1 - r0, X.shape[1] if X.dim() == 2 else 1)
        xb.copy_(X.reshape(xb.shape))
        X = xb
    _log(f"sharded {config} ({exchange}): shard ready ({r1 - r0} rows, {sw.plan.n_halo} halo rows); warmup")
    run = (lambda: sw.wavelet_features(X, k=K, s=s_heat, out=out)) if exchange in ("rccl", "ipc", "sdma") else \
        (lambda: sw.wavelet_features(X, k=K, s=s_heat))
    for i in range(max(2, warmup)):   # the native chain is captured into a hipGraph on its 2nd call
        run()
        torch.cuda.synchronize(device)
    _log(f"sharded {config} ({exchange}): warm")
    if min_time > 0:
        # extras: at least min_time s of chains in the timed region -- a few 1-ms chains (Reddit
        # F = 1) read 2x slow on one ms-scale hiccup (profiles/r02/s36_bench: 5 chains 2.19 ms
        # each vs 1.03 alone, s37).  The headline times exactly the driver's steps.
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        run()
        torch.cuda.synchronize(device)
        one = time.perf_counter() - t1
        if world > 1:
            one = _allreduce(one, dist.ReduceOp.MAX, device)
        steps = max(steps, min(200, int(min_time / max(one, 1e-6))))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _log(f"sharded {config} ({exchange}): timed {steps} chains in {elapsed:.3f} s")
    med = None
    if median_reps > 0:   # per-chain times (HIP events on the launch stream), median over ranks' max
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(median_reps + 1)]
        if world > 1:
            dist.barrier()
        evs[0].record()
        for i in range(median_reps):
            run()
            evs[i + 1].record()
        torch.cuda.synchronize(device)
        per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(median_reps))
        med = per[len(per) // 2]
        if world > 1:
            med = _allreduce(med, dist.ReduceOp.MAX, device)
    # kernel / exchange attribution: one more pass, eager, with HIP events (outside the timed region)
    dinfo = sw.info()   # after the timed chains: was the chain replayed as a hipGraph?
    sw.profile_start()
    run()
    prof = sw.profile_collect()
    chk = None
    if check:
        chk = _check_vs_unsharded(sw, indptr_d, indices_d, n_t, r0, r1, F, K, s_heat, world, device,
                                  NormalizedLaplacian, graph_wavelet_features)
    del indptr_d, indices_d
    if world > 1:
        elapsed = _allreduce(elapsed, dist.ReduceOp.MAX, device)
    nnz_lhat = _allreduce(float(sw.L.nnz), dist.ReduceOp.SUM, device) if world > 1 else float(sw.L.nnz)
    p = sw.plan
    # SURVEY 8(d) over the rows the step launches: a shard's purely isolated own rows are closed-form
    # and never launched, as in the unsharded line
    n_launch = p.n_own - int(sw.L.info["n_closed_form"])
    b_8d = algorithmic_bytes(n_launch, sw.L.nnz, F)
    lds_info = sw.L.lds_plan_info(active_only=False) if (F == 1 and sw.u_len() > 0) else None
    b_step = lds_algorithmic_bytes(lds_info) if lds_info else b_8d
    plan_text = sw.L.describe(F)
    kernel = lds_kernel_name(lds_info, team="team:" in plan_text) + " (rank 0 shard)"
    tiles_plan = [ln for ln in plan_text.splitlines() if ln.startswith("tiles:")]
    if tiles_plan:   # the hybrid step: dense blocks on MFMA + the tail, in the form that ran
        forms = [ln for ln in plan_text.splitlines() if ln.startswith("hybrid forms:")]
        f = dict(t.split("=") for t in forms[-1].split(":", 1)[1].split()) if forms else {}
        if int(f.get("fused", 0)) > 0 and int(f.get("two_stream", 0)) == 0 and int(f.get("sequential", 0)) == 0:
            kernel = ("hybrid step, fused form: hybrid_fused_kernel (dense-block items + the tail's team waves in "
                      "one launch) + tiles_combine_kernel + hybrid_epilogue_kernel (rank 0 shard)")
        else:
            kernel = ("hybrid step: cheb_tiles_kernel + tiles_combine_kernel + the tail on the step kernel "
                      f"(forms run: {forms[-1] if forms else 'unknown'}; rank 0 shard)")
    avg_ms = prof["step_ms"]
    sw.close()
    del sw
    torch.cuda.empty_cache()
    return {
        "metric": f"Chebyshev SpMM-chain edges*K/s ({config}-size, K={K}, row-sharded)",
        "value": nnz_lhat * K * steps / elapsed,
        "unit": "edges*K/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "median_step_ms": med,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"{config}-size R-MAT (GPU generator, seed {seed}), one graph row-sharded over "
                               f"{world} ranks, halo exchange per Chebyshev step "
                               + {"rccl": "(native: grouped ncclSend/ncclRecv",
                                  "ipc": "(native: one-sided pull from IPC-mapped peer memory, flag-ordered phases",
                                  "sdma": "(native: owners pack, receivers copy the packed blocks from "
                                          "IPC-mapped peer memory by hipMemcpyAsync on a copy stream, "
                                          "flag-ordered phases",
                                  "nccl": "(torch all_to_all_single, RCCL",
                                  "host": "(torch all_to_all_single on host copies, gloo"}[exchange]
                               + (", chain replayed as a hipGraph)" if dinfo and dinfo.get("captured")
                                  else ", chain launched eagerly)" if dinfo else ")")
                               + f"; K={K} F={F}",
                   "exchange": exchange,
                   "N": n_t, "nnz_input": nnz_global, "nnz_lhat": nnz_lhat, "K": K, "F": F,
                   "rank0_rows": p.n_own, "rank0_halo_rows": p.n_halo, "parallelism": f"rows x{world}"},
        "roofline": {"bound": "hbm", "achieved": b_step / (avg_ms * 1e-3) / 1e9 if avg_ms else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (b_step / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if avg_ms else None,
                     "traffic": None, "kernel": kernel,
                     "algorithmic_bytes_per_launch": b_step, "avg_launch_us": avg_ms * 1e3,
                     "avg_exchange_us": prof["exchange_ms"] * 1e3,
                     "graph_replayed": bool(dinfo.get("captured")) if dinfo else None,
                     "byte_model": _byte_model(lds_info),
                     "lds_plan": lds_info,
                     "tiles_plan": tiles_plan[0] if tiles_plan else None,
                     "rows_per_launch": n_launch, "closed_form_rows": p.n_own - n_launch},
        "check": chk,
    }


def _check_vs_unsharded(sw, indptr_d, indices_d, n, r0, r1, F, K, s_heat, world, device, NormalizedLaplacian,
                        graph_wavelet_features) -> dict:
    """Column-sensitive check of the sharded chain: a random signal (same on
    every rank, seeded), the sharded S on this rank's rows against the
    unsharded chain of the whole graph on this rank's GPU (the product path
    twice: every halo row and gathered column must be right); max over ranks."""
    gen = torch.Generator(device=device)
    gen.manual_seed(12345)
    X = torch.randn(n, F, generator=gen, device=device)
    _, S_sh = sw.wavelet_features(X[r0:r1].contiguous(), k=K, s=s_heat)
    L = NormalizedLaplacian(n, indptr_d, indices_d, device=device)
    _, S_full = graph_wavelet_features(L, k=K, s=s_heat, X0=X, return_S=True)
    L.close()
    ref = S_full[r0:r1].double()
    err = (S_sh.double() - ref).abs().amax(dim=0) if r1 > r0 else torch.zeros(F, dtype=torch.float64, device=device)
    scale = S_full.double().abs().amax(dim=0)
    rel = float((err / scale.clamp_min(1e-300)).max())
    if world > 1:
        rel = _allreduce(rel, dist.ReduceOp.MAX, device)
    return {"max_rel_err": rel, "tol": CHECK_TOL, "ok": bool(rel <= CHECK_TOL),
            "what": "random signal (all F columns): every rank's rows of the sharded S vs the unsharded chain on "
                    "the same GPU; max over ranks and columns of max|dS| / max|S|"}


def one_gpu_chain(config, K, F, steps, seed, s_heat, device, world=1, rank=0) -> dict:
    """The N > 1 headline's workload unsharded on ONE GPU (every rank runs it on
    its own device, no collective; rank 0's is reported): the same graph
    (GPU generator, same seed), K, F and s through wg_wavelet_features, so the
    row-sharded curve can be read against the same config's one-GPU chain
    (VERDICT r2 item 6)."""
    import wats_hip
    from wats_hip import NormalizedLaplacian
    from wats_hip.graphgen import NAMED_CONFIGS
    n_t, nnz_t, K_def, F_def = NAMED_CONFIGS[config]
    K = K if K is not None else K_def
    F = F if F is not None else F_def
    ip, ix = shared_graph(config, seed, world, rank, device)
    L = NormalizedLaplacian(n_t, ip, ix, device=device)
    del ip, ix
    gen = torch.Generator(device=device)
    gen.manual_seed(1)
    X = L.log1p_degree() if F == 1 else torch.randn(n_t, F, generator=gen, device=device)
    S = torch.empty(n_t, F, device=device)
    H = torch.empty(n_t, F, device=device)
    lib = wats_hip._lib.load()
    stream = torch.cuda.current_stream(device).cuda_stream

    def run():
        wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), F, K, s_heat, S.data_ptr(),
                                                    H.data_ptr(), stream), "wavelet_features")
    for _ in range(3):
        run()
    torch.cuda.synchronize(device)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    evs[0].record()
    for i in range(steps):
        run()
        evs[i + 1].record()
    torch.cuda.synchronize(device)
    per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    total = evs[0].elapsed_time(evs[-1])
    plan = [ln for ln in L.describe(F).splitlines() if ln.startswith("tiles:")]
    nnz = L.nnz
    L.close()
    del S, H, X
    torch.cuda.empty_cache()
    return {"config": config, "K": K, "F": F, "nnz": nnz, "steps": steps, "ms_per_step": total / steps,
            "median_step_ms": per[len(per) // 2], "value": float(nnz) * K * steps / (total * 1e-3),
            "unit": "edges*K/s", "hybrid_step": bool(plan),
            "what": "the same graph / K / F unsharded through wg_wavelet_features on one GPU (HIP events over "
                    "the chains; each rank on its own device, rank 0 reported): divide the headline's value by "
                    "this value for the row-sharded speed-up on the same config"}


# ----------------------------------------------------------------------------- single-GPU measurement
def cold_chains(step, L, reps, device):
    """SURVEY.md 8(d) 'cold' protocol: before each timed pass, write a 512 MiB
    scratch buffer (evicts the 256 MiB Infinity Cache and every L2), then time
    the pass alone (HIP events on the stream it runs on)."""
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device=device)
    ms, launch_ms, launches = [], 0.0, 0
    for _ in range(reps):
        scratch.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        L.profile_enable(True)
        a.record()
        step()
        b.record()
        torch.cuda.synchronize(device)
        p = L.profile_collect()
        L.profile_enable(False)
        ms.append(a.elapsed_time(b))
        launch_ms += p["sum_ms"]
        launches += p["launches"]
    del scratch
    torch.cuda.empty_cache()
    ms.sort()
    return {"reps": reps, "step_ms": ms[len(ms) // 2], "avg_launch_us": launch_ms / max(1, launches) * 1e3,
            "protocol": "512 MiB scratch write before each pass; median pass time"}


def f1_companion(lib, L, K, s_heat, steps, device, unit=False):
    """The same graph with the reference's own F = 1 signal log1p(rowsum)
    (WATS.py:58-59): the kernel auto-selection's choice and its step time."""
    import wats_hip
    X = L.log1p_degree()
    n = L.n
    S = torch.empty(n, 1, dtype=torch.float32, device=device)
    H = torch.empty(n, 1, dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream

    def run():
        wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), 1, K, s_heat, S.data_ptr(),
                                                    H.data_ptr(), stream), "wavelet_features")
    for _ in range(3):
        run()
    torch.cuda.synchronize(device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):     # passes alone, then again with per-launch events for the kernel time
        run()
    b.record()
    torch.cuda.synchronize(device)
    ms = a.elapsed_time(b) / steps
    L.profile_enable(True)
    for _ in range(steps):
        run()
    p = L.profile_collect()
    L.profile_enable(False)
    avg_ms = p["sum_ms"] / max(1, p["launches"])
    n_active = n - int(L.info["n_closed_form"])
    info = L.lds_plan_info(active_only=True)
    b_step = lds_algorithmic_bytes(info) if info else clenshaw_bytes(n_active, L.nnz, 1, unit)
    b_8d = algorithmic_bytes(n_active, L.nnz, 1)
    b_roof = b_step if info else b_8d   # as the main line: SURVEY 8(d) unless an LDS format runs
    return {"F": 1, "signal": "log1p(rowsum) (WATS.py:58-59)", "value": float(L.nnz) * K / (ms * 1e-3),
            "unit": "edges*K/s", "ms_per_step": ms, "avg_launch_us": avg_ms * 1e3,
            "kernel": lds_kernel_name(info),
            "byte_model": _byte_model(info),
            "algorithmic_bytes_per_launch": b_roof, "frac": b_roof / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "kernel_byte_model": _byte_model(info) if info else "Clenshaw heat sum (DESIGN.md 4.1)",
            "kernel_bytes_frac": b_step / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}


def prologue_timing(g, L, device, reps: int = 5) -> dict:
    """the prologue (a1-a3: degrees, dinv, isolated flags, the
    length-ordered column-sorted operator, log1p(rowsum)) reported beside the
    chain, not in it: wg_laplacian_create from a CSR already on the device
    (graph upload excluded), median of `reps`; and the log1p-degree signal."""
    import wats_hip
    ipd = torch.from_numpy(np.asarray(g.indptr, np.int64)).to(device)
    ixd = torch.from_numpy(np.asarray(g.indices, np.int32)).to(device)
    vd = None if g.values is None else torch.from_numpy(np.asarray(g.values, np.float32)).to(device)
    ms = []
    for _ in range(reps + 1):   # the first also loads kernels
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        Lp = wats_hip.NormalizedLaplacian(g.n, ipd, ixd, vd, device=device)
        torch.cuda.synchronize(device)
        ms.append((time.perf_counter() - t0) * 1e3)
        Lp.close()
    ms = sorted(ms[1:])
    sig = []
    for _ in range(reps):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        L.log1p_degree()
        torch.cuda.synchronize(device)
        sig.append((time.perf_counter() - t0) * 1e3)
    sig.sort()
    del ipd, ixd, vd
    return {"create_ms": ms[len(ms) // 2], "log1p_degree_ms": sig[len(sig) // 2], "reps": reps,
            "what": "wg_laplacian_create (a1-a2: column degrees w, dinv, isolated flags, the operator's rows "
                    "ordered by length and columns sorted; a CSR already in HBM) and the a3 signal, host wall "
                    "time around a device sync, median; not in the chain's time (SURVEY 8(d))"}


def single_gpu_line(args, g, config, K, F, world, rank, device, full=True):
    """One graph per rank (no collective): graph_wavelet_features passes timed
    as the driver's contract says.  full=False: value / step / roofline only
    (companion lines)."""
    import wats_hip
    st = g.stats()
    unit = g.values is None or bool(np.all(g.values == 1))   # the value-free Clenshaw chain applies
    L = wats_hip.NormalizedLaplacian.from_graph(g, device=device)
    if getattr(args, "tune", None):
        L.tune(**args.tune)
    pro = prologue_timing(g, L, device) if (full and world == 1) else None
    rng = np.random.default_rng(1 + rank)
    if F == 1:
        X_host = None  # the reference signal log1p(rowsum)
        X = L.log1p_degree()
    else:
        X_host = rng.standard_normal((g.n, F)).astype(np.float32)
        X = torch.from_numpy(X_host).to(device)
    n, nnz = L.n, L.nnz
    S = torch.empty(n, F, dtype=torch.float32, device=device)
    H = torch.empty(n, F, dtype=torch.float32, device=device)
    lib = wats_hip._lib.load()
    stream = torch.cuda.current_stream(device).cuda_stream

    def step():
        wats_hip._lib.check(lib.wg_wavelet_features(L.handle, X.data_ptr(), F, K, args.s, S.data_ptr(),
                                                    H.data_ptr(), stream), "wavelet_features")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    # Clock settle (untimed, reported as settle_s): W passes are ~2 ms of load at the
    # defaults, short of the clock ramp (profiles/r01/s51_iter_sweep.log: the first
    # measurement of a fresh process reads 2-3 us/step slow on arxiv F=40).
    t_settle = time.perf_counter() + args.settle_s
    while time.perf_counter() < t_settle:
        for _ in range(8):
            step()
        torch.cuda.synchronize(device)

    def timed(profile: bool):
        """K passes bracketed by barrier + synchronize; with `profile`, HIP
        events on the launch stream around every step-kernel launch."""
        L.profile_enable(profile)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if profile else None
        if evs:
            evs[0].record()
        for i in range(args.steps):
            step()
            if evs:
                evs[i + 1].record()
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        prof = None
        if profile:
            d = L.profile_durations()
            prof = dict(sum_ms=sum(d), launches=len(d), max_ms=max(d) if d else 0.0, durations=d)
        L.profile_enable(False)
        ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)) if evs else []
        return t1 - t0, prof, ms[len(ms) // 2] if ms else None

    # value: the passes alone, no events at all (per-launch events add ~4.5 us of
    # gap each, 10 % of an arxiv F=40 pass); roofline and the per-pass median:
    # the same K passes again, with events around every step launch and pass
    elapsed, _, _ = timed(False)
    S_host = S.cpu().numpy() if (full and world == 1) else None   # the benchmarked pass's S (parity check)
    elapsed_prof, prof, median_ms = timed(True)
    _log(f"{config}: timed {args.steps} passes in {elapsed:.3f} s")
    cold = cold_chains(step, L, args.cold_reps, device) if (full and args.cold_reps > 0) else None
    f1 = f1_companion(lib, L, K, args.s, args.steps, device, unit) if (full and args.f1_companion and F > 1) else None
    edges_k = float(nnz) * K * args.steps
    if world > 1:
        elapsed = _allreduce(elapsed, dist.ReduceOp.MAX, device)
        edges_k = _allreduce(edges_k, dist.ReduceOp.SUM, device)
    avg_ms = prof["sum_ms"] / max(1, prof["launches"])
    # the folded chain (tuning key fold): each pass's first launch is
    # cheb_team4_first_kernel, which also does the former permute-in pass's work; the roofline is
    # the dominant kernel's (cheb_team4_kernel, the other K - 1 launches, as rocprof averages it)
    team_path = F > 1 and "team:" in L.describe(F)
    folded = team_path and unit and F % 4 == 0 and K >= 2 and prof["launches"] == args.steps * K and \
        int((getattr(args, "tune", None) or {}).get("fold", 1)) == 1
    first_us = None
    if folded:
        d = prof["durations"]
        first = [d[i] for i in range(len(d)) if i % K == 0]
        plain = [d[i] for i in range(len(d)) if i % K != 0]
        first_us = sum(first) / len(first) * 1e3
        avg_ms = sum(plain) / len(plain)
    one_launch_chain = F == 1 and "chain1:" in L.describe(1)
    if one_launch_chain:   # csrc/chain.hip: one launch runs all K steps: per step = / K
        avg_ms /= K
    # the step kernel processes the rows that enter the chain; purely
    # isolated rows (closed form T_k = (-1)^k X0) are handled by finalize
    n_active = n - int(L.info["n_closed_form"])
    b_8d = algorithmic_bytes(n_active, nnz, F)
    lds_info = L.lds_plan_info(active_only=True) if F == 1 else None
    b_step = lds_algorithmic_bytes(lds_info) if lds_info else clenshaw_bytes(n_active, nnz, F, unit)
    # roofline.achieved: SURVEY 8(d)'s per-row / per-nonzero figure x the rows and nonzeros one launch
    # processes (the contract); the bytes this kernel's own algorithm needs are reported beside it.
    # (F == 1 LDS formats: their own model -- SURVEY's 8 B/nnz would read above 1.0)
    if one_launch_chain:   # chain.hip reads neither the LDS plan's format nor values: SURVEY 8(d) / Clenshaw-u bytes
        lds_info = None
        b_step = clenshaw_bytes(n_active, nnz, F, unit)
    b_roof = b_step if lds_info else b_8d
    achieved = b_roof / (avg_ms * 1e-3) / 1e9
    traffic, traffic_src = None, None
    tj = args.traffic_json
    if tj == "auto":
        tj = os.path.join(REPO, "profiles", "r06", "s13_traffic.json") \
            if (config == "ogbn-arxiv" and F == 40 and K == 16) else None
    if tj and tj != "none" and os.path.exists(tj):
        traffic = json.load(open(tj)).get("bytes_per_launch")
        traffic_src = os.path.relpath(tj, REPO) if os.path.isabs(tj) else tj
    line = {
        "metric": f"Chebyshev SpMM-chain edges*K/s ({config}-size, K={K}) + %HBM roofline",
        "value": edges_k / elapsed,
        "unit": "edges*K/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_s": args.settle_s,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{config}-size R-MAT graph (a=.57,b=c=.19), symmetrised, no self loops; "
                        f"graph_wavelet_features K={K}, F={F} "
                        f"{'log1p-degree signal' if F == 1 else 'randn signal columns'}, s={args.s}",
            "N": n, "nnz": nnz, "isolated": st["isolated"], "max_degree": st["max_degree"],
            "K": K, "F": F, "per_rank": "one graph per rank, no collective",
            "parallelism": f"graphs x{world}",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": (f"{traffic_src}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950's 128-B requests counted "
                               f"as 64 B; TCC_EA0_RDREQ_128B x 128 B agrees within 0.4 %) + WRITE_SIZE per launch "
                               f"of this kernel on this workload"
                               if traffic is not None else None),
            "kernel": lds_kernel_name(lds_info, one_launch_chain, "team:" in L.describe(F)),
            "byte_model": _byte_model(lds_info) if lds_info else
                          "SURVEY 8(d): 8 B/nnz + 4(N+1) + 20 N F over the launched rows",
            "algorithmic_bytes_per_launch": b_roof,
            "kernel_byte_model": _byte_model(lds_info) if lds_info else
                                 ("Clenshaw heat sum on u = b dinv (DESIGN.md 4.1): 4 B/nnz + 4(N+1) + 16 N F + 8 N"
                                  if unit else "Clenshaw heat sum (DESIGN.md 4.1): 8 B/nnz + 4(N+1) + 16 N F"),
            "kernel_bytes_per_launch": b_step,
            "kernel_bytes_frac": b_step / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "rows_per_launch": n_active,
            "closed_form_rows": n - n_active,
            "algorithmic_bytes_all_rows": algorithmic_bytes(n, nnz, F),
            "all_rows_frac": algorithmic_bytes(n, nnz, F) / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "frac_note": "frac: SURVEY 8(d)'s B_step over the rows each launch processes (purely isolated "
                         "rows are closed-form and never launched); kernel_bytes_frac: the bytes this "
                         "kernel's algorithm needs (Clenshaw: no S stream; unweighted: no CSR values); "
                         "all_rows_frac: SURVEY 8(d)'s B_step with N = all nodes",
            "avg_launch_us": avg_ms * 1e3,
            "max_launch_us": prof["max_ms"] * 1e3,
            "launches": prof["launches"],
            "first_launch_us": first_us,
            "all_launches_avg_us": prof["sum_ms"] / max(1, prof["launches"]) * 1e3,
            # the same byte model over every launch of the chain, the folded first launch included
            "frac_all_launches": b_roof / (prof["sum_ms"] / max(1, prof["launches"]) * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "launch_note": ("avg_launch_us / achieved / frac: the K - 1 plain step launches of each pass "
                            "(cheb_team4_kernel, the dominant kernel as rocprof averages it); first_launch_us: "
                            "each pass's first launch (cheb_team4_first_kernel: also reads the caller's X0 "
                            "through perm, writes the internal X0 and the closed-form rows' S / H -- the former "
                            "permute-in pass); frac_all_launches: frac's byte model over the mean of all K "
                            "launches, the first included") if folded else None,
        },
        "chain_ms": prof["sum_ms"] / args.steps,
        "median_step_ms_profiled": median_ms,
        "value_median": float(nnz) * K / (median_ms * 1e-3) * world if median_ms else None,
        "ms_per_step_profiled": elapsed_prof / args.steps * 1e3,
        "timing": "value / ms_per_step: K passes without per-launch events; roofline and median: the same K "
                  "passes timed right after with HIP events around every step-kernel launch and every pass "
                  "(ms_per_step_profiled, median_step_ms_profiled; value_median = nnz*K / that median)",
        "edges_K_F_per_s": edges_k * F / elapsed,
    }
    if pro is not None:
        line["prologue"] = pro
    if cold is not None:
        cold["edges_K_per_s"] = float(nnz) * K / (cold["step_ms"] * 1e-3)
        cold["achieved_GBs"] = b_roof / (cold["avg_launch_us"] * 1e-6) / 1e9
        cold["frac"] = cold["achieved_GBs"] / HBM_PEAK_GBS
        line["cold"] = cold
    if f1 is not None:
        line["f1_companion"] = f1
    if full and world == 1 and not args.no_cpu_baseline:
        if X_host is None:
            X_host = L.log1p_degree().cpu().numpy()
        line["cpu_baseline"] = cpu_baseline(g, K, F, args.s, X_host, args.cpu_seconds, S_host)
        line["cpu_baseline"]["host_cpu"] = _cpu_model()
    L.close()
    del S, H, X
    torch.cuda.empty_cache()
    return line


def _companion_summary(d: dict) -> dict:
    """The fields of a companion line worth keeping in the main line."""
    keep = ("metric", "value", "ms_per_step", "value_median", "median_step_ms_profiled", "config")
    out = {k: d[k] for k in keep if k in d}
    r = d.get("roofline", {})
    out["roofline"] = {k: r.get(k) for k in ("achieved", "frac", "kernel_bytes_frac", "all_rows_frac",
                                             "avg_launch_us", "rows_per_launch", "closed_form_rows",
                                             "algorithmic_bytes_per_launch", "kernel")}
    return out


# ----------------------------------------------------------------------------- main
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # WATS_BENCH_DEVICE pins every rank to one device (multi-rank tests on a 1-GPU box)
    dev_idx = int(os.environ.get("WATS_BENCH_DEVICE", local_rank if world > 1 else 0))
    device = torch.device("cuda", dev_idx)
    torch.cuda.set_device(device)
    if world > 1:
        # WATS_BENCH_PG=gloo: rehearse several ranks on one GPU (RCCL refuses two
        # ranks per device); with the IPC exchange the sharded path needs no RCCL
        backend = os.environ.get("WATS_BENCH_PG", "nccl")
        with _stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group(backend)
            dist.barrier()
            # a CPU group created up front: per-rank failure flags are agreed over it before any
            # rank changes course, so no rank starts another collective alone
            global _CPU_GROUP
            _CPU_GROUP = dist.new_group(backend="gloo")
    mode = args.mode if args.mode != "auto" else ("graphs" if world == 1 else "sharded")
    exchanges = [x for x in args.exchange.split(",") if x]
    from wats_hip.graphgen import NAMED_CONFIGS, connect_isolated, named_graph

    line = None
    picked_other = None
    if mode == "sharded":
        # the N > 1 headline: one graph row-sharded over every rank (strong scaling).  A
        # collective that never completes must not cost the whole line: a watchdog prints
        # an error line and ends the process after --headline-timeout seconds.
        import threading
        cfg = args.scale_config if args.mode == "auto" else args.config

        def _expire_headline():
            if rank == 0:
                _emit({"metric": f"Chebyshev SpMM-chain edges*K/s ({cfg}-size, row-sharded over {world} GPUs)",
                       "value": None, "unit": "edges*K/s", "n_gpus": world, "steps": args.steps,
                       "warmup": args.warmup, "higher_is_better": True, "scaling": "strong",
                       "error": f"the row-sharded headline did not finish within {args.headline_timeout:.0f} s"},
                      args.out)
            os._exit(3)
        hw = threading.Timer(args.headline_timeout, _expire_headline)
        hw.daemon = True
        hw.start()
        exc = None
        try:
            line = run_sharded(cfg, args.K, args.F, args.steps, args.warmup, args.seed, args.s, world, rank, device,
                               exchanges[0], median_reps=max(20, args.steps))
        except Exception as e:  # noqa: BLE001 -- keep a headline: the next exchange, noted in the line
            exc = e
        if _any_rank(exc is not None, world):   # every rank switches together, or none does
            if exc is None:
                exc = RuntimeError(f"the {exchanges[0]} headline failed on another rank")
            if len(exchanges) < 2:
                raise exc
            _log(f"headline with exchange {exchanges[0]} failed ({type(exc).__name__}: {exc}); using {exchanges[1]}")
            torch.cuda.empty_cache()
            line = run_sharded(cfg, args.K, args.F, args.steps, args.warmup, args.seed, args.s, world, rank, device,
                               exchanges[1], median_reps=max(20, args.steps))
            line["headline_fallback"] = f"exchange {exchanges[0]} failed: {type(exc).__name__}: {exc}"
            exchanges = exchanges[1:] + exchanges[:1]
        hw.cancel()
        if len(exchanges) > 1 and args.pick_exchange and "headline_fallback" not in line:
            # the same headline with the second exchange, same steps: the line is the faster of the
            # two whose column-sensitive check passed (both are reported).  If the second hangs,
            # a watchdog prints the first line as it is.
            first = line

            def _expire_pick():
                if rank == 0:
                    first["exchange_compare"] = {"error": f"exchange {exchanges[1]} did not finish in "
                                                          f"{args.sharded_timeout:.0f} s"}
                    _emit(first, args.out)
                os._exit(0)
            pw = threading.Timer(args.sharded_timeout, _expire_pick)
            pw.daemon = True
            pw.start()
            try:
                torch.cuda.empty_cache()
                alt = run_sharded(cfg, args.K, args.F, args.steps, args.warmup, args.seed, args.s, world, rank,
                                  device, exchanges[1], median_reps=max(20, args.steps))
            except Exception as exc:  # noqa: BLE001
                alt = {"error": f"{type(exc).__name__}: {exc}", "exchange": exchanges[1]}
            pw.cancel()
            if _any_rank("error" in alt, world) and "error" not in alt:   # failed elsewhere: same choice everywhere
                alt = {"error": f"exchange {exchanges[1]} failed on another rank", "exchange": exchanges[1]}

            def _ok(r):
                return r.get("value") is not None and bool((r.get("check") or {}).get("ok"))
            cmp = {x: ({"value": r.get("value"), "ms_per_step": r.get("ms_per_step"),
                        "check_ok": bool((r.get("check") or {}).get("ok"))} if "error" not in r else r)
                   for x, r in ((exchanges[0], first), (exchanges[1], alt))}
            if _ok(alt) and (not _ok(first) or alt["value"] > first["value"]):
                line, other, other_x = alt, first, exchanges[0]
            else:
                line, other, other_x = first, alt, exchanges[1]
            line["exchange_compare"] = cmp
            line["exchange_choice"] = ("the headline is the faster of the exchanges timed with the same steps "
                                       "whose column-sensitive check passed; the other is attached as "
                                       f"sharded_{cfg.replace('-', '')}_{other_x}")
            picked_other = (other_x, other)
        else:
            picked_other = None
        line["metric"] = (f"Chebyshev SpMM-chain edges*K/s ({cfg}-size, K={line['config']['K']}, F="
                          f"{line['config']['F']}, row-sharded over {world} GPUs)")
        line["headline_note"] = ("N > 1 headline: BASELINE.json configs[3] (Reddit-size, 1-D row-sharded, halo "
                                 f"exchange '{line['config'].get('exchange')}': the faster of the IPC pull and RCCL "
                                 "grouped send/recv whose check passed, exchange_compare); the N = 1 line carries "
                                 "the same run at one rank as `sharded`; same_config_1gpu: the same config "
                                 "unsharded on one GPU")
        try:
            torch.cuda.empty_cache()
            line["same_config_1gpu"] = one_gpu_chain(cfg, args.K, args.F, args.steps, args.seed, args.s, device,
                                                     world, rank)
            line["same_config_1gpu"]["speedup"] = line["value"] / line["same_config_1gpu"]["value"]
        except Exception as exc:  # noqa: BLE001
            line["same_config_1gpu"] = {"error": f"{type(exc).__name__}: {exc}"}
    else:
        n_target, nnz_target, K_def, F_def = NAMED_CONFIGS[args.config]
        K = args.K if args.K is not None else K_def
        F = args.F if args.F is not None else F_def
        g = named_graph(args.config, seed=args.seed + rank)   # independent graph per rank
        line = single_gpu_line(args, g, args.config, K, F, world, rank, device, full=True)
        if world == 1 and args.connected_companion and args.config == "ogbn-arxiv":
            a = argparse.Namespace(**vars(args))
            a.cold_reps = 0
            line["connected_companion"] = _companion_summary(
                single_gpu_line(a, connect_isolated(g, seed=7), "ogbn-arxiv-connected", K, F, world, rank, device,
                                full=False))
            line["connected_companion"]["what"] = ("the same R-MAT graph with every isolated node attached to one "
                                                   "random node (graphgen.connect_isolated): no closed-form rows, "
                                                   "as the real ogbn-arxiv")
        if world == 1 and args.pubmed_companion and args.config == "ogbn-arxiv":
            # BASELINE.json configs[1]: the small, launch-bound chain (replayed as a hipGraph)
            a = argparse.Namespace(**vars(args))
            a.cold_reps = 0
            a.settle_s = 0.1
            pk, pf = NAMED_CONFIGS["pubmed"][2], NAMED_CONFIGS["pubmed"][3]
            pm = _companion_summary(single_gpu_line(a, named_graph("pubmed", seed=args.seed), "pubmed", pk, pf,
                                                    world, rank, device, full=False))
            chain_s = pm["ms_per_step"] * 1e-3
            b = pm["roofline"]["algorithmic_bytes_per_launch"]
            pm["chain_us"] = chain_s * 1e6
            pm["chain_frac"] = pk * b / chain_s / (HBM_PEAK_GBS * 1e9)
            pm["roofline_chain_us"] = pk * b / (HBM_PEAK_GBS * 1e9) * 1e6
            pm["what"] = ("PubMed-size R-MAT, K=16, the reference's F=1 signal: one whole chain per step, the auto "
                          "path (csrc/chain.hip: the chain in one launch of cooperating workgroups, DESIGN.md 4.7); "
                          "chain_frac = K x B_step / chain time / 8 TB/s; multi_launch: the same chain as K + 3 "
                          "launches (tuning key chain = 0)")
            a.tune = {"chain": 0}
            ml = _companion_summary(single_gpu_line(a, named_graph("pubmed", seed=args.seed), "pubmed", pk, pf,
                                                    world, rank, device, full=False))
            pm["multi_launch"] = {"chain_us": ml["ms_per_step"] * 1e3,
                                  "chain_frac": pk * b / (ml["ms_per_step"] * 1e-3) / (HBM_PEAK_GBS * 1e9),
                                  "avg_launch_us": ml["roofline"]["avg_launch_us"], "kernel": ml["roofline"]["kernel"]}
            line["pubmed_companion"] = pm
        del g

    extras = [c for c in (args.sharded_extra or "none").split(",") if c and c != "none"]
    if mode == "sharded":
        extras = [c for c in extras if c != (args.scale_config if args.mode == "auto" else args.config)]
    results = {}
    watchdog = None
    if extras or (mode == "sharded" and args.replicas):
        # Measured after the headline is complete; a Python-level failure is reported in
        # the line instead of losing it, and a watchdog prints the line and ends the
        # process if a run (a collective on several GPUs) does not finish in time.
        import threading

        def _expire():
            if rank == 0:
                results["timeout"] = {"error": f"timeout after {args.sharded_timeout:.0f} s; the runs not "
                                                f"listed did not finish"}
                _attach(line, results, mode)
                _emit(line, args.out)
            os._exit(0)
        watchdog = threading.Timer(args.sharded_timeout, _expire)
        watchdog.daemon = True
        watchdog.start()
    if mode == "sharded" and args.replicas:
        try:
            n_target, nnz_target, K_def, F_def = NAMED_CONFIGS[args.config]
            g = named_graph(args.config, seed=args.seed + rank)
            a = argparse.Namespace(**vars(args))
            a.cold_reps = 0
            results["replicas"] = _companion_summary(single_gpu_line(a, g, args.config, K_def, F_def, world, rank,
                                                                     device, full=False))
            results["replicas"]["what"] = ("one independent ogbn-arxiv-size graph per rank (weak scaling, no "
                                           "collective): the round-1 N > 1 headline")
            del g
        except Exception as exc:  # noqa: BLE001
            results["replicas"] = {"error": f"{type(exc).__name__}: {exc}"}
    for i, c in enumerate(extras):
        # N = 1: the first extra (the Reddit-size F=41 run the N > 1 headline scales) with every exchange
        xs = exchanges if (mode != "sharded" and i == 0) else exchanges[:1]
        for j, x in enumerate(xs):
            key = c if j == 0 else f"{c}_{x}"
            try:
                torch.cuda.empty_cache()
                results[key] = run_sharded(c, None, None, args.sharded_steps, 1, args.seed, args.s, world, rank,
                                           device, x, min_time=0.2)
            except Exception as exc:  # noqa: BLE001
                results[key] = {"error": f"{type(exc).__name__}: {exc}", "exchange": x}
    if mode == "sharded" and len(exchanges) > 1:
        # the headline config with the other exchanges (same line, for the exchange comparison)
        cfg = args.scale_config if args.mode == "auto" else args.config
        if picked_other is not None:   # the exchange the headline did not pick, timed in full
            results[f"{cfg}_{picked_other[0]}"] = picked_other[1]
        for x in exchanges[1:]:
            if picked_other is not None and x in exchanges[:2]:
                continue
            try:
                torch.cuda.empty_cache()
                results[f"{cfg}_{x}"] = run_sharded(cfg, args.K, args.F, args.sharded_steps, 1, args.seed, args.s,
                                                    world, rank, device, x, min_time=0.2)
            except Exception as exc:  # noqa: BLE001
                results[f"{cfg}_{x}"] = {"error": f"{type(exc).__name__}: {exc}", "exchange": x}
    if watchdog is not None:
        watchdog.cancel()
    if rank == 0:
        _attach(line, results, mode)
        _emit(line, args.out)
    if world > 1:
        dist.destroy_process_group()


class _stdout_to_stderr:
    """Point file descriptor 1 at stderr for the duration (native libraries'
    prints included)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


os.environ.setdefault("WATS_DIST_LOG", "1")


def _log(msg: str) -> None:
    """Progress on stderr (rank-prefixed), so long multi-rank runs show where they are."""
    print(f"[bench rank {os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr,
          flush=True)


_CPU_GROUP = None


def _any_rank(flag: bool, world: int) -> bool:
    """True on every rank if `flag` is true on any rank (over the CPU group)."""
    if world <= 1:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=_CPU_GROUP)
    return bool(t.item())


def _allreduce(x: float, op, device) -> float:
    on = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=on)
    dist.all_reduce(t, op=op)
    return float(t.item())


def _attach(line: dict, results: dict, mode: str) -> None:
    """graphs mode: the first sharded run -> line["sharded"], the others ->
    line["sharded_<config>[_<exchange>]"]; sharded mode: every extra under
    its own key ("replicas", "sharded_<config>[_<exchange>]")."""
    first = mode != "sharded"
    for c, r in results.items():
        if c in ("replicas", "timeout"):
            line[c] = r
        elif first:
            line["sharded"] = r
            first = False
        else:
            line["sharded_" + c.replace("-", "")] = r


def _emit(line: dict, out: str | None) -> None:
    js = json.dumps(line)
    print(js, flush=True)
    if out:
        with open(out, "w") as f:
            f.write(js + "\n")


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
