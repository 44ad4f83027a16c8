"""Row-sharded multi-GPU graph-wavelet path.

One process per GPU.  A graph too large (or too slow) for one GPU is split
into contiguous 1-D row blocks balanced by nonzeros.  Each rank owns the rows
``[r0, r1)`` of ``L_hat`` and keeps its column space as ``[owned rows | halo
rows]``, with the halo rows grouped by owner rank.  Row i of ``T_k`` needs
``T_{k-1}`` at i's neighbours, plus ``T_{k-2}`` and ``S`` at row i only.  So the
only exchange per Chebyshev step (reference ``calibration/WATS.py:35-36``) is
the halo rows of ``T_{k-1}``.  That is one all-to-all-v: grouped
ncclSend/ncclRecv in native code (``csrc/dist.hip``, the default, the whole
chain replayed as a hipGraph), or ``torch.distributed.all_to_all_single``
(RCCL over xGMI with the "nccl" backend, or gloo on host copies in tests).
The heat sum and the row-L1 normalisation are row-local.

Setup also needs the Laplacian's column degree ``w = colsum(A) - diag(A)``
(scipy ``_laplacian.py:467``).  It spans all shards, so it costs one
all-reduce of float64 partial column sums.

The planning functions (:func:`partition_rows`, :func:`build_halo_plan`,
:func:`global_column_degree`) are plain numpy / torch.distributed and run on
any backend (CPU-tested with gloo).  :class:`ShardedWavelet` runs the HIP
kernels.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, ptr


def _trace(msg: str) -> None:
    """Setup progress on stderr when WATS_DIST_LOG=1 (long multi-rank setups)."""
    import os
    import sys
    import time
    if os.environ.get("WATS_DIST_LOG") == "1":
        print(f"[dist rank {os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr,
              flush=True)


def partition_rows(indptr: np.ndarray, world: int) -> np.ndarray:
    """Contiguous row blocks balanced by (nnz + rows): returns ``bounds`` of
    length world+1 with rank q owning rows [bounds[q], bounds[q+1])."""
    indptr = np.asarray(indptr, dtype=np.int64)
    n = len(indptr) - 1
    weight = indptr + np.arange(n + 1)           # cumulative nnz + rows
    total = weight[-1]
    targets = (np.arange(1, world) * total) // world
    cuts = np.searchsorted(weight, targets, side="left")
    bounds = np.concatenate([[0], np.clip(cuts, 0, n), [n]]).astype(np.int64)
    bounds = np.maximum.accumulate(bounds)
    if n >= world:
        # hub rows can swallow several targets: keep every shard non-empty
        # (shard q keeps >= 1 row and leaves >= world - q - 1 rows to the rest)
        for q in range(1, world):
            bounds[q] = min(max(bounds[q], bounds[q - 1] + 1), n - (world - q))
    return bounds


@dataclass
class HaloPlan:
    rank: int
    world: int
    bounds: np.ndarray
    r0: int
    r1: int
    n_halo: int
    halo_global: np.ndarray                 # global ids of halo rows, grouped by owner
    recv_counts: list                       # halo rows received per peer
    send_counts: list                       # rows sent per peer
    send_rows: np.ndarray                   # local (caller-order) row ids to send, grouped by peer
    local_indices: np.ndarray               # CSR columns renumbered to [own | halo]
    stats: dict = field(default_factory=dict)

    @property
    def n_own(self) -> int:
        return self.r1 - self.r0

    @property
    def n_cols(self) -> int:
        return self.n_own + self.n_halo


def _rank_world(group=None):
    """(rank, world) of the group; an uninitialised default group is a single rank."""
    if group is None and not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _device_for(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def exchange_int_lists(lists: list, group=None) -> list:
    """All-to-all of variable-length int64 arrays: lists[q] goes to rank q;
    returns what every rank sent to us (index = source rank)."""
    world = dist.get_world_size(group)
    dev = _device_for(group)
    send_counts = torch.tensor([len(x) for x in lists], dtype=torch.int64, device=dev)
    recv_counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rc = recv_counts.cpu().tolist()
    sc = send_counts.cpu().tolist()
    send = torch.from_numpy(np.concatenate([np.asarray(x, np.int64) for x in lists]) if sum(sc) else
                            np.zeros(0, np.int64)).to(dev)
    recv = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc, group=group)
    out = recv.cpu().numpy()
    offs = np.concatenate([[0], np.cumsum(rc)])
    return [out[offs[q]:offs[q + 1]] for q in range(world)]


def build_halo_plan(indptr_local: np.ndarray, indices_global, bounds: np.ndarray, group=None,
                    compute_device=None, col_degree=None) -> HaloPlan:
    """Renumber this rank's CSR columns to [own | halo] and agree with every
    peer on who sends which rows (collective).  The halo is grouped by owner
    rank; with ``col_degree`` (the global column degree, indexed by global
    id) each group is in descending degree (ties by id), so the highest-degree
    halo columns of every peer are a prefix of its group -- the F = 1 hub
    kernel stages those prefixes in LDS (csrc/lds1.hip, build_shard_hub).

    The column work (unique, searchsorted over nnz entries) runs with torch on
    ``compute_device`` (the GPU for large shards; default CPU)."""
    rank, world = _rank_world(group)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    dev = torch.device(compute_device) if compute_device is not None else torch.device("cpu")
    cols = torch.as_tensor(np.asarray(indices_global) if not isinstance(indices_global, torch.Tensor)
                           else indices_global).to(dev, torch.int64)
    own = (cols >= r0) & (cols < r1)
    remote = cols[~own]
    halo_t = torch.unique(remote, sorted=True)
    n_own = r1 - r0
    local = cols - r0
    halo_sorted = halo_t.cpu().numpy()
    owner_sorted = np.searchsorted(bounds, halo_sorted, side="right") - 1
    if col_degree is not None and halo_sorted.size:
        deg = np.asarray(col_degree.cpu().numpy() if isinstance(col_degree, torch.Tensor) else col_degree)
        order = np.lexsort((halo_sorted, -deg[halo_sorted].astype(np.float64), owner_sorted))
    else:
        order = np.lexsort((halo_sorted, owner_sorted))
    rank_of = np.empty(halo_sorted.size, np.int64)   # position in the halo of the id at sorted position i
    rank_of[order] = np.arange(halo_sorted.size)
    local[~own] = n_own + torch.from_numpy(rank_of).to(dev)[torch.searchsorted(halo_t, remote)]
    halo_global = halo_sorted[order]
    owner = owner_sorted[order]
    recv_lists = [halo_global[owner == q] for q in range(world)]
    requested = exchange_int_lists(recv_lists, group) if world > 1 else recv_lists  # what each peer needs from us
    send_rows = np.concatenate(requested).astype(np.int64) - r0 if world else np.zeros(0, np.int64)
    assert np.all((send_rows >= 0) & (send_rows < max(n_own, 1))) or send_rows.size == 0
    plan = HaloPlan(rank=rank, world=world, bounds=np.asarray(bounds), r0=r0, r1=r1, n_halo=int(halo_global.size),
                    halo_global=halo_global, recv_counts=[int(len(x)) for x in recv_lists],
                    send_counts=[int(len(x)) for x in requested], send_rows=send_rows.astype(np.int32),
                    local_indices=local.to(torch.int32).cpu().numpy())
    plan.stats = dict(n_own=n_own, n_halo=plan.n_halo, nnz_local=int(cols.numel()),
                      nnz_remote=int(remote.numel()), send_rows=int(send_rows.size))
    return plan


def gather_rows(X_local: torch.Tensor, bounds: np.ndarray, group=None) -> torch.Tensor:
    """The full (N, F) matrix on every rank from each rank's row block
    ``[bounds[q], bounds[q+1])`` (the optional final H gather
    for a caller -- the WATS head -- that needs every row on one device).
    One all_gather of row blocks padded to the largest block; collective."""
    rank, world = _rank_world(group)
    if world == 1:
        return X_local
    b = np.asarray(bounds, dtype=np.int64)
    sizes = np.diff(b)
    mx = int(sizes.max())
    F = X_local.shape[1] if X_local.dim() == 2 else 1
    dev = _device_for(group)
    pad = torch.zeros(mx, F, dtype=X_local.dtype, device=dev)
    pad[: X_local.shape[0]] = X_local.reshape(-1, F).to(dev)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    out = torch.cat([parts[q][: int(sizes[q])] for q in range(world)])
    return out.to(X_local.device)


def allreduce_column_degree(partial_colsum: torch.Tensor, partial_diag: torch.Tensor, group=None) -> torch.Tensor:
    """``w = colsum(A) - diag(A)`` for every global column: all-reduce the
    float64 partial sums of the shards, then scipy's float32 subtraction
    (``_laplacian.py:467``)."""
    world = _rank_world(group)[1]
    dev = _device_for(group) if world > 1 else partial_colsum.device
    cs = partial_colsum.to(dev, torch.float64)
    dg = partial_diag.to(dev, torch.float64)
    if world > 1:
        dist.all_reduce(cs, group=group)
        dist.all_reduce(dg, group=group)
    return cs.to(torch.float32) - dg.to(torch.float32)


def plan_column_degree(w_global: torch.Tensor, plan: HaloPlan) -> torch.Tensor:
    """The global column degree at this rank's columns [own | halo]."""
    ids = torch.from_numpy(np.concatenate([np.arange(plan.r0, plan.r1), plan.halo_global]).astype(np.int64))
    return w_global[ids.to(w_global.device)]


def global_column_degree(partial_colsum: torch.Tensor, partial_diag: torch.Tensor, plan: HaloPlan,
                         group=None) -> torch.Tensor:
    """``w = colsum(A) - diag(A)`` for the columns [own | halo] of this rank:
    all-reduce the float64 partial sums, then scipy's float32 subtraction."""
    return plan_column_degree(allreduce_column_degree(partial_colsum, partial_diag, group), plan)


def halo_exchange(ext: torch.Tensor, plan: HaloPlan, pack, sendbuf: torch.Tensor, group=None,
                  host_staged: bool = False) -> None:
    """Fill the halo rows ``ext[n_own:]`` of the extended vector with the
    owners' current values: pack the rows each peer asked for (``pack(ext,
    sendbuf)``), then one all-to-all-v.  Collective: every rank calls it every
    step, also with nothing to send."""
    if plan.world == 1:
        return
    pack(ext, sendbuf)
    rc, sc = list(plan.recv_counts), list(plan.send_counts)
    recv = ext[plan.n_own:plan.n_own + sum(rc)]
    snd = sendbuf[:sum(sc)]
    if not host_staged:
        dist.all_to_all_single(recv, snd, output_split_sizes=rc, input_split_sizes=sc, group=group)
    else:
        r = torch.empty(sum(rc), ext.shape[1], dtype=ext.dtype)
        dist.all_to_all_single(r, snd.cpu(), output_split_sizes=rc, input_split_sizes=sc, group=group)
        recv.copy_(r.to(ext.device))


class ShardedWavelet:
    """One rank's shard of ``L_hat`` on its GPU, plus the halo exchange.

    ``exchange="rccl"`` (default): the whole chain in native code
    (``wg_dist_*``, ``csrc/dist.hip``): its own RCCL communicator, grouped
    ncclSend/ncclRecv per step, captured into a hipGraph and replayed.
    ``exchange="ipc"``: the same native chain with a one-sided exchange: the
    ranks' vectors mapped into each other by IPC, halo rows pulled straight
    from the owners' memory, phases ordered by flags (``wg_dist_ipc_*``).
    ``exchange="sdma"``: the same mapping, but each owner packs the rows its
    peers asked for and the receivers copy the packed blocks with peer DMA
    (``hipMemcpyAsync`` on a copy stream, ``wg_dist_ipc_sdma``): no CU time
    for the transfer itself.
    ``exchange="nccl"``: the same exchange from Python, one
    ``torch.distributed.all_to_all_single`` per step (RCCL/xGMI).
    ``exchange="host"``: that collective on host copies (gloo) -- lets several
    ranks share one GPU in tests (RCCL refuses two ranks on one device).
    Each step exchanges the halo, then computes (the overlap variants of round
    2 measured slower and were removed).
    """

    def __init__(self, indptr_local, indices_global, values_local, n_global: int, bounds, group=None,
                 exchange: str = "rccl", device=None, max_features: int = 1):
        from .laplacian import NormalizedLaplacian, require_gpu
        self.device = require_gpu(device)
        self.group = group
        self.exchange = exchange
        indptr_local = np.asarray(indptr_local, np.int64)
        rank, world = _rank_world(group)
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        _trace("column degrees")
        # partial column degrees of this shard, on the GPU (float64 atomics), all-reduced:
        # the halo plan orders each peer's group by this degree (the F = 1 hub kernel)
        lib = _lib.load()
        ip = torch.from_numpy(indptr_local).to(self.device)
        ix = torch.from_numpy(np.asarray(indices_global, np.int32)).to(self.device)
        vals = None if values_local is None else torch.as_tensor(np.asarray(values_local, np.float32)).to(self.device)
        colsum = torch.zeros(n_global, dtype=torch.float64, device=self.device)
        diag = torch.zeros(n_global, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            st = torch.cuda.current_stream(self.device).cuda_stream
            check(lib.wg_column_degree(r1 - r0, r0, ptr(ip), ptr(ix) if ix.numel() else None, ptr(vals),
                                       ptr(colsum), ptr(diag), st), "column_degree")
        w_global = allreduce_column_degree(colsum, diag, group)
        del colsum, diag
        _trace("column degrees done; halo plan")
        self.plan = build_halo_plan(indptr_local, indices_global, bounds, group, compute_device=self.device,
                                    col_degree=w_global)
        p = self.plan
        w_cols = plan_column_degree(w_global, p).to(self.device)
        del w_global
        _trace(f"halo plan done ({p.n_halo} halo rows); operator")
        self.L = NormalizedLaplacian(p.n_own, ip, torch.from_numpy(p.local_indices), vals, n_cols=p.n_cols,
                                     w_cols=w_cols, device=self.device)
        _trace("operator done")
        rows = torch.from_numpy(p.send_rows).to(self.device)
        self.send_rows = torch.empty_like(rows)
        if rows.numel():
            with torch.cuda.device(self.device):
                check(lib.wg_laplacian_map_rows(self.L.handle, 0, ptr(rows), rows.numel(), ptr(self.send_rows),
                                                torch.cuda.current_stream(self.device).cuda_stream), "map_rows")
        self._bufs = {}
        self.profile = False          # record (exchange, step) event pairs per Chebyshev step
        self.events = []
        self._dist = None
        if exchange == "rccl":
            self._dist = self._create_native()
        elif exchange in ("ipc", "sdma"):
            # the shared region is sized for max_features columns (large IPC
            # mappings are slow to set up: keep it to what the chain uses); a
            # call with more columns rebuilds it (collective, like the call)
            self._ipc_F = int(max_features)
            self._dist = self._create_ipc(self._ipc_F)
        elif exchange not in ("nccl", "host"):
            raise ValueError(f"exchange must be 'rccl', 'ipc', 'sdma', 'nccl' or 'host', not {exchange!r}")
        _trace("exchange ready")

    def _create_native(self):
        """The native chain's handle: RCCL unique id from rank 0, broadcast over
        the group, then ncclCommInitRank on every rank (collective)."""
        lib, p = _lib.load(), self.plan
        uid = (ctypes.c_uint8 * 128)()
        if p.rank == 0:
            check(lib.wg_dist_unique_id(uid), "dist_unique_id")
        if p.world > 1:
            obj = [bytes(uid)]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(self.group, 0) if self.group else 0,
                                       group=self.group)
            ctypes.memmove(uid, obj[0], 128)
        sc = np.ascontiguousarray(p.send_counts, dtype=np.int64)
        rc = np.ascontiguousarray(p.recv_counts, dtype=np.int64)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.wg_dist_create(self.L.handle, uid, p.rank, p.world,
                                     ptr(self.send_rows) if self.send_rows.numel() else None,
                                     sc.ctypes.data, rc.ctypes.data, ctypes.byref(h)), "dist_create")
        return h

    def _create_ipc(self, max_features: int):
        """The native chain with the one-sided exchange: every rank exposes its
        ping-pong vectors by IPC and pulls its halo rows straight from the
        owners' memory (no RCCL communicator).  Setup is collective over the
        group (any backend, gloo included)."""
        lib, p = _lib.load(), self.plan
        sc = np.ascontiguousarray(p.send_counts, dtype=np.int64)
        rc = np.ascontiguousarray(p.recv_counts, dtype=np.int64)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib.wg_dist_create(self.L.handle, None, p.rank, p.world,
                                     ptr(self.send_rows) if self.send_rows.numel() else None,
                                     sc.ctypes.data, rc.ctypes.data, ctypes.byref(h)), "dist_create")
            blob = (ctypes.c_uint8 * 128)()
            check(lib.wg_dist_ipc_local(h, int(max_features), blob), "dist_ipc_local")
        _trace("ipc region ready; exchanging handles")
        # what each owner sends me = its internal ids of my halo rows, in my halo order
        send_int = self.send_rows.cpu().numpy().astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(p.send_counts)]).astype(np.int64)
        if p.world > 1:
            blobs = [None] * p.world
            dist.all_gather_object(blobs, bytes(blob), group=self.group)
            src = exchange_int_lists([send_int[offs[q]:offs[q + 1]] for q in range(p.world)], self.group)
        else:
            blobs = [bytes(blob)]
            src = [send_int]
        halo_src = torch.from_numpy(np.concatenate(src).astype(np.int32) if p.n_halo else
                                    np.zeros(1, np.int32)).to(self.device)
        assert sum(len(x) for x in src) == p.n_halo
        allb = (ctypes.c_uint8 * (128 * p.world)).from_buffer_copy(b"".join(blobs))
        _trace("handles exchanged; mapping the peers' regions")
        err = None
        with torch.cuda.device(self.device):
            try:
                check(lib.wg_dist_ipc_connect(h, allb, ptr(halo_src)), "dist_ipc_connect")
            except Exception as exc:  # noqa: BLE001 -- made collective below
                err = exc
        if p.world > 1:
            # every rank must be connected before any enters a chain (a rank waiting on
            # peers that gave up would spin until its 60 s timeout)
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=_device_for(self.group))
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=self.group)
            if not int(ok.item()) and err is None:
                err = RuntimeError("wats_hip: IPC exchange setup failed on another rank")
        if err is None and self.exchange == "sdma":
            # where each owner packed my block in its send buffer: its send offset for me
            offs_q = (exchange_int_lists([[int(offs[q])] for q in range(p.world)], self.group) if p.world > 1
                      else [np.array([0])])
            pso = np.ascontiguousarray([int(x[0]) for x in offs_q], dtype=np.int64)
            with torch.cuda.device(self.device):
                try:
                    check(lib.wg_dist_ipc_sdma(h, pso.ctypes.data), "dist_ipc_sdma")
                except Exception as exc:  # noqa: BLE001 -- made collective below
                    err = exc
            if p.world > 1:
                ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=_device_for(self.group))
                dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=self.group)
                if not int(ok.item()) and err is None:
                    err = RuntimeError("wats_hip: SDMA exchange setup failed on another rank")
        if err is not None:
            lib.wg_dist_destroy(h)
            raise err
        return h

    def check_exchange(self) -> None:
        """Raise if an IPC phase wait timed out (synchronises the device)."""
        if self._dist is not None:
            t = ctypes.c_int32(0)
            check(_lib.load().wg_dist_status(self._dist, ctypes.byref(t)), "dist_status")
            if t.value & 1:
                raise RuntimeError("wats_hip: a peer did not complete its phase within 60 s (IPC exchange)")
            if t.value & 2:
                raise RuntimeError("wats_hip: an IPC phase signal did not release every XCD's L2 (DESIGN.md 7)")

    def set_graph(self, enable: bool) -> None:
        """Replay the native chain as a hipGraph (default) or run it eagerly."""
        if self._dist is not None:
            check(_lib.load().wg_dist_set_graph(self._dist, 1 if enable else 0), "dist_set_graph")

    def close(self) -> None:
        if getattr(self, "_dist", None) is not None:
            _lib.load().wg_dist_destroy(self._dist)
            self._dist = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    # -------------------------------------------------------------- exchange
    def _pack(self, ext: torch.Tensor, out: torch.Tensor) -> None:
        n = int(self.send_rows.numel())
        if n:
            with torch.cuda.device(self.device):
                check(_lib.load().wg_gather_rows(ptr(ext), ptr(self.send_rows), n, ext.shape[1], ptr(out),
                                                 torch.cuda.current_stream(self.device).cuda_stream), "gather_rows")

    def _halo_exchange(self, ext: torch.Tensor) -> None:
        sendbuf = self._buf("send", int(self.send_rows.numel()), ext.shape[1])
        halo_exchange(ext, self.plan, self._pack, sendbuf, self.group, host_staged=(self.exchange != "nccl"))

    def _buf(self, name, rows, F):
        key = (name, F)
        b = self._bufs.get(key)
        if b is None or b.shape[0] < rows:
            b = torch.empty(max(rows, 1), F, dtype=torch.float32, device=self.device)
            self._bufs[key] = b
        return b[:rows]

    def profile_start(self) -> None:
        self.profile = True
        self.L.profile_enable(True)

    def profile_collect(self) -> dict:
        """Mean halo-exchange and step-kernel time (ms) per Chebyshev step; resets."""
        torch.cuda.synchronize(self.device)
        ex = [e[0].elapsed_time(e[1]) for e in self.events]
        self.events = []
        if self._dist is not None:
            tot, cnt = ctypes.c_double(0), ctypes.c_int64(0)
            check(_lib.load().wg_dist_profile_collect(self._dist, ctypes.byref(tot), ctypes.byref(cnt)),
                  "dist_profile_collect")
            ex = [tot.value / cnt.value] * cnt.value if cnt.value else []
        st = self.L.profile_collect()
        self.L.profile_enable(False)
        self.profile = False
        n = max(1, st["launches"])  # one step launch per Chebyshev step
        return dict(exchange_ms=sum(ex) / max(1, len(ex)), step_ms=st["sum_ms"] / n, max_step_ms=st["max_ms"],
                    launches=st["launches"])

    def info(self) -> dict:
        """State of the native chain (wg_dist_info): own / halo / sent rows,
        world, exchange kind, captured graph present."""
        if self._dist is None:
            return {}
        out = (ctypes.c_int64 * 8)()
        check(_lib.load().wg_dist_info(self._dist, out), "dist_info")
        keys = ("overlap", "n_own", "n_halo", "n_send", "world", "exchange", "captured", "tiers")
        d = dict(zip(keys, [int(v) for v in out]))
        del d["overlap"], d["tiers"]
        d["exchange"] = {1: "ipc", 2: "rccl", 3: "sdma"}.get(d["exchange"], "none")
        return d

    # -------------------------------------------------------------- chain
    def u_len(self) -> int:
        """Length of the F == 1 LDS kernel's gather vector u (0: kernel not applicable)."""
        if not hasattr(self, "_u_len"):
            n = ctypes.c_int64(0)
            with torch.cuda.device(self.device):
                check(_lib.load().wg_cheb_u_len(self.L.handle, ctypes.byref(n)), "cheb_u_len")
            self._u_len = int(n.value)
        return self._u_len

    def _wavelet_features_u(self, X: torch.Tensor, k: int, s: float):
        """F == 1, unweighted: the column-blocked LDS kernel; the per-step halo
        exchange carries u = T_{k-1} * dinv (what the kernel gathers)."""
        import math
        p, L, lib = self.plan, self.L, _lib.load()
        ulen = self.u_len()
        U = (self._buf("U0", ulen, 1), self._buf("U1", ulen, 1))
        T = (self._buf("A", p.n_own, 1), self._buf("B", p.n_own, 1))
        S = self._buf("S", p.n_own, 1)
        with torch.cuda.device(self.device):
            st = torch.cuda.current_stream(self.device).cuda_stream
            check(lib.wg_permute_rows(L.handle, 0, 1, ptr(X), ptr(T[0]), st), "permute_rows")
            check(lib.wg_scale_dinv(L.handle, ptr(T[0]), ptr(U[0]), st), "scale_dinv")
        for i in range(1, k + 1):
            cur_u, nxt_u = U[(i - 1) % 2], U[i % 2]
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if (self.profile and p.world > 1) else None
            if ev:
                ev[0].record()
            self._halo_exchange(cur_u[: p.n_cols])
            if ev:
                ev[1].record()
                self.events.append(ev)
            with torch.cuda.device(self.device):
                st = torch.cuda.current_stream(self.device).cuda_stream
                check(lib.wg_cheb_step_u(L.handle, i, ptr(cur_u), ptr(T[(i - 1) % 2]),
                                         None if i == 1 else ptr(T[i % 2]), None if i == k else ptr(T[i % 2]),
                                         None if i == k else ptr(nxt_u), ptr(S), 1.0, math.exp(-s * i), st),
                      "cheb_step_u")
        return S

    def _wavelet_features_native(self, X: torch.Tensor, k: int, s: float, out):
        """The native chain: inputs copied into a persistent buffer and outputs
        written to persistent ones (stable pointers, so the captured hipGraph is
        replayed), then cloned -- unless the caller passes ``out=(H, S)``."""
        p, F = self.plan, X.shape[1]
        xb = self._buf("X", p.n_own, F)
        if xb.data_ptr() != X.data_ptr():
            xb.copy_(X)
        if out is not None:
            H, S = out
            if H.shape != (p.n_own, F) or S.shape != (p.n_own, F) or not (H.is_contiguous() and S.is_contiguous()):
                raise ValueError("out=(H, S) must be contiguous (n_own, F) float32 tensors")
        else:
            H, S = self._buf("Hout", p.n_own, F), self._buf("Sout", p.n_own, F)
        with torch.cuda.device(self.device):
            check(_lib.load().wg_dist_wavelet_features(self._dist, ptr(xb), F, int(k), float(s), ptr(S), ptr(H),
                                                       torch.cuda.current_stream(self.device).cuda_stream),
                  "dist_wavelet_features")
        return (H, S) if out is not None else (H.clone(), S.clone())

    def wavelet_features(self, X0_local: torch.Tensor, k: int = 3, s: float = 0.8, out=None):
        """Owned rows of (H, S) for signal rows X0_local (caller order).
        ``out=(H, S)``: write into these (native exchange only)."""
        import math
        p = self.plan
        L = self.L
        F_in = X0_local.shape[-1] if X0_local.dim() == 2 else 1
        X = X0_local.to(self.device, torch.float32).reshape(p.n_own, F_in).contiguous()   # (0, F) on an empty shard
        F = X.shape[1]
        if self.exchange in ("ipc", "sdma") and F > self._ipc_F:
            self.close()
            self._ipc_F = F
            self._dist = self._create_ipc(F)
        if self._dist is not None:
            # native chain on every rank, empty shards included: a rank with no rows must
            # still take part in every phase of the exchange (RCCL groups / IPC flags)
            return self._wavelet_features_native(X, k, s, out)
        if F == 1 and k >= 1 and p.n_own and self.u_len() > 0:
            S = self._wavelet_features_u(X, k, s)
            from .wavelet import row_l1_normalize
            H_int = row_l1_normalize(S)
            return L.permute(H_int, to_internal=False), L.permute(S, to_internal=False)
        A = self._buf("A", p.n_cols, F)
        B = self._buf("B", p.n_cols, F)
        S = self._buf("S", p.n_own, F)
        with torch.cuda.device(self.device):
            st = torch.cuda.current_stream(self.device).cuda_stream
            if p.n_own:
                check(_lib.load().wg_permute_rows(L.handle, 0, F, ptr(X), ptr(A), st), "permute_rows")
        if k == 0:
            S.copy_(A[: p.n_own])
        bufs = (A, B)
        for i in range(1, k + 1):
            cur = bufs[(i - 1) % 2]
            nxt = bufs[i % 2]
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if (self.profile and p.world > 1) else None
            if ev:
                ev[0].record()
            self._halo_exchange(cur)
            if ev:
                ev[1].record()
                self.events.append(ev)
            L.step(i, cur, None if i == 1 else nxt[: p.n_own], None if i == k else nxt[: p.n_own], S=S,
                   alpha0=1.0, alpha_k=math.exp(-s * i))
        from .wavelet import row_l1_normalize
        H_int = row_l1_normalize(S) if p.n_own else S.clone()
        S_out = L.permute(S, to_internal=False) if p.n_own else S.clone()
        H_out = L.permute(H_int, to_internal=False) if p.n_own else H_int
        return H_out, S_out
