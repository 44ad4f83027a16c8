// dist.hip -- SURVEY section 8(e): the row-sharded Chebyshev chain with the
// per-step halo exchange in native code (RCCL point-to-point over xGMI).
//
// Each rank owns an nnz-balanced row block of L_hat whose columns are
// [own rows | halo rows grouped by owner] (wats_hip/dist.py builds the plan).
// Row i of T_k needs T_{k-1} at i's neighbours (reference calibration/
// WATS.py:35-36), so every step first refreshes the halo: pack the own rows
// each peer asked for, then one grouped ncclSend/ncclRecv per peer (an
// all-to-all-v, received straight into the halo rows of the extended vector),
// then the step kernel.  On the F = 1 LDS path the exchanged vector is
// u = T * dinv, which is what that kernel gathers.
//
// The K-step loop (pack, exchange, step, ..., finalize) is captured once per
// (pointers, F, K, s) into a hipGraph and replayed, so a chain costs one graph
// launch of host time instead of 3K launches and K Python-level collectives.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "internal.h"

namespace wg {
namespace {

__global__ void pack_rows_kernel(int64_t n, int64_t F, const int32_t* __restrict__ rows, const float* __restrict__ src,
                                 float* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * F) return;
  const int64_t i = idx / F;
  dst[idx] = src[(int64_t)rows[i] * F + (idx - i * F)];
}

// the same with 16-B lanes (F % 4 == 0, 16-B aligned rows: every padded chain vector)
__global__ void pack_rows4_kernel(int64_t n, int64_t F4, const int32_t* __restrict__ rows, const float4* __restrict__ src,
                                  float4* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * F4) return;
  const int64_t i = idx / F4;
  dst[idx] = src[(int64_t)rows[i] * F4 + (idx - i * F4)];
}

// pack rows[0, n) of src (F floats per row) into dst, 16-B lanes when the width allows
void launch_pack(int64_t n, int64_t F, const int32_t* rows, const float* src, float* dst, hipStream_t st) {
  if (n <= 0) return;
  if (F % 4 == 0 && (reinterpret_cast<uintptr_t>(src) % 16) == 0 && (reinterpret_cast<uintptr_t>(dst) % 16) == 0)
    hipLaunchKernelGGL(pack_rows4_kernel, dim3((unsigned)ceil_div(n * (F / 4), 256)), dim3(256), 0, st, n, F / 4, rows,
                       reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst));
  else
    hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)ceil_div(n * F, 256)), dim3(256), 0, st, n, F, rows, src, dst);
}

// received rows i (row-block streaming: received contiguously per (block, peer)) -> halo row pos[i]

// ---- one-sided exchange over IPC-mapped peer memory (exchange mode "ipc") ----
// Each rank exposes one allocation: two slots of its extended vector ([own |
// halo] rows, ping-pong) and `world` int64 flags.  A rank's flag q holds how
// many chain phases peer q has completed (phase 0: the chain's first vector,
// phase k: step k).  Before phase p a rank waits until every peer has
// completed p phases: then each peer's step-(p-1) vector is final, and no peer
// still reads the slot phase p overwrites (its last read of that slot was in
// its phase p-1).  The wait and the pull of the halo rows (system-scope loads
// straight from the owners' slots over xGMI) are one kernel; the signal is a
// one-lane kernel after the phase's last kernel.
constexpr int kMaxPeers = 16;

struct IpcPull {
  const float* slot_base[kMaxPeers];  // peer q's slot 0 (mapped); slot 1 at + slot_floats[q]
  int64_t slot_floats[kMaxPeers];
  const int64_t* flags;               // mine: flags[q] = phases peer q completed
  int64_t* count;                     // phases this rank completed
  int64_t* const* peer_flags;         // peer q's flags (mapped), device array [world]
  int32_t* err;
  int32_t world, rank;
};

// wait until every peer has completed as many phases as this rank (ipc_signal_kernel counts them)
__device__ __forceinline__ void ipc_wait(const IpcPull& p) {
  __shared__ int64_t s_target;
  if (threadIdx.x == 0) s_target = *p.count;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int q = threadIdx.x;
    const int64_t target = s_target;
    bool ok = true;
    // once a wait has timed out (a lost peer) later phases do not wait again: the chain
    // finishes in one 60 s timeout, not one per phase, and wg_dist_status reports it
    const bool failed = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (q < p.world && q != p.rank && !failed) {
      const uint64_t t0 = wall_clock64();
      while (__hip_atomic_load(p.flags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (wall_clock64() - t0 > 100ull * 1000 * 1000 * 60) {  // 60 s at the 100 MHz constant clock
          ok = false;
          break;
        }
      }
    }
    if (!ok) __hip_atomic_fetch_or(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
  }
  __syncthreads();
}

// halo row h (owner owner[h], row src[h] of the owner's extended vector) ->
// ext[n_own + h].  Launched after ipc_wait_kernel on the same stream, so it
// needs no wait of its own and can use a full grid (one remote load per lane:
// the pull is latency-bound, 0.8 MB per Reddit-size step over 7 links).
__global__ __launch_bounds__(256) void ipc_pull_kernel(IpcPull p, int slot, int64_t n_own, int64_t h0, int64_t n_halo,
                                                       int64_t F, const int32_t* __restrict__ owner,
                                                       const int32_t* __restrict__ src, float* __restrict__ ext) {
  const int64_t total = n_halo * F;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t idx = h0 * F + i;  // halo rows [h0, h0 + n_halo)
    const int64_t h = idx / F;
    const int q = owner[h];
    WG_DCHECK(q >= 0 && q < p.world && q != p.rank && src[h] >= 0 && ((int64_t)src[h] + 1) * F <= p.slot_floats[q],
              "halo row %lld: owner %d row %d outside its %lld-float slot", (long long)h, q, src[h],
              (long long)(q >= 0 && q < kMaxPeers ? p.slot_floats[q] : -1));
    const float* from = p.slot_base[q] + slot * p.slot_floats[q] + (int64_t)src[h] * F + (idx - h * F);
    ext[n_own * F + idx] = __hip_atomic_load(from, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The same pull with 16-B loads (F % 4 == 0: every row and slot is 16-B aligned): one
// system-scope (sc0 sc1: no stale cached copy of the owner's slot) dwordx4 buffer load
// per lane, 4x fewer remote transactions than ipc_pull_kernel for the F = 44 rows.  Only the
// first Fr columns of each row move (the signal's own columns rounded up to 4: F = 41 at width 48
// pulls 176 of its 192 bytes); the halo rows' pad columns stay zero (transfer() zeroes them once).
__global__ __launch_bounds__(256) void ipc_pull4_kernel(IpcPull p, int slot, int64_t n_own, int64_t h0, int64_t n_halo,
                                                        int64_t F, int64_t Fr, const int32_t* __restrict__ owner,
                                                        const int32_t* __restrict__ src, float* __restrict__ ext) {
  constexpr int kSysCoherent = 1 | 16;  // cache policy sc0 | sc1 (gfx940+ CPol bits)
  const int64_t F4 = F >> 2, R4 = Fr >> 2;
  const int64_t total = n_halo * R4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t hr = i / R4;
    const int64_t c4 = i - hr * R4;
    const int64_t h = h0 + hr;  // halo rows [h0, h0 + n_halo)
    const int64_t idx = h * F4 + c4;
    const int q = owner[h];
    WG_DCHECK(q >= 0 && q < p.world && q != p.rank && src[h] >= 0 && ((int64_t)src[h] + 1) * F <= p.slot_floats[q],
              "halo row %lld: owner %d row %d outside its %lld-float slot", (long long)h, q, src[h],
              (long long)(q >= 0 && q < kMaxPeers ? p.slot_floats[q] : -1));
    const float* base = p.slot_base[q] + slot * p.slot_floats[q];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff,
                                                                        0x00020000);
    const uint32_t off = (uint32_t)(((int64_t)src[h] * F + c4 * 4) * 4);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, kSysCoherent);
    *reinterpret_cast<u32x4*>(ext + n_own * F + idx * 4) = v;
  }
}

#ifdef WG_TIMING_PROBES
// timing probe (knob "xdelay"): hold the stream for `ticks` of the 100 MHz constant clock,
// standing in for link time the one-GPU runs do not have
__global__ void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
#endif

// wait for the peers; one workgroup
__global__ void ipc_wait_kernel(IpcPull p, int) { ipc_wait(p); }

// this rank completed one more phase: every XCD's L2 written back, count += 1, then every peer told.
// Cross-device ordering: a peer pulls this rank's slot rows with system-scope loads
// over xGMI, which read memory (HBM / Infinity Cache), never this device's L2s; the slot rows were
// written by the phase's kernels on up to all 8 XCDs, with write-through (sc1) stores (the step
// kernels' u_k) or plain stores (permute-in, scale_rows: the first vector).  So that this does not
// rest on the scope of the runtime's end-of-kernel release (which this code cannot read, eager or
// replayed from a hipGraph), kIpcSignalBlocks workgroups (one or more on every XCD: workgroups are
// dealt round-robin) each write back their XCD's L2 (__threadfence_system = buffer_wbl2 sc0 sc1 +
// its wait), count their XCD in a mask and arrive on a counter; the last to arrive resets it,
// checks that n_xcc distinct XCDs released (else err |= 2: the ordering is not guaranteed) and
// stores the flags with system-scope release stores.
constexpr int kIpcSignalBlocks = 64;
__global__ void ipc_signal_kernel(int64_t* count, int32_t world, int32_t rank, int64_t* const* peer_flags,
                                  uint32_t* arrive, int32_t n_xcc, int32_t* err) {
  if (threadIdx.x != 0) return;
  __threadfence_system();
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  __hip_atomic_fetch_or(arrive + 1, 1u << (xcc & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t old = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1u != (uint32_t)kIpcSignalBlocks) return;
  __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next phase starts from 0
  const uint32_t mask = __hip_atomic_exchange(arrive + 1, 0u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (__popc(mask) < n_xcc) __hip_atomic_fetch_or(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __threadfence_system();
  const int64_t c = *count + 1;
  *count = c;
  for (int q = 0; q < world; ++q)
    if (q != rank) __hip_atomic_store(peer_flags[q] + rank, c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int nccl_try(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return WG_OK;
  return fail(WG_ERR_HIP, "%s: %s", what, ncclGetErrorString(r));
}

struct GraphKey {
  const float* X0;
  float* S;
  float* H;
  int64_t F;
  int32_t K;
  double s;
  int64_t gen;  // the handle's tune_gen: wg_laplacian_tune frees plans and changes launch knobs
  bool operator==(const GraphKey& o) const {
    return X0 == o.X0 && S == o.S && H == o.H && F == o.F && K == o.K && s == o.s && gen == o.gen;
  }
};

}  // namespace
}  // namespace wg

using namespace wg;

struct wg_dist_s {
  wg_laplacian_t L = nullptr;  // not owned
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  int64_t n_own = 0, n_cols = 0, n_send = 0, n_halo = 0;
  int32_t* send_rows = nullptr;  // internal ids of own rows, grouped by peer
  std::vector<int64_t> send_cnt, recv_cnt, send_off, recv_off;  // [world], [world + 1]
  float* ws = nullptr;
  size_t ws_floats = 0;
  bool use_graph = true;
  hipStream_t cap = nullptr;  // capture / replay stream (the caller's may be the null stream)
  hipEvent_t fork = nullptr, join = nullptr;
  // the stream the handle's last chain was enqueued on (a replay goes into the caller's stream, an
  // eager chain onto cap): a chain enqueued on another stream first waits for it (handoff), since
  // both share the workspace, the exchange slots and the phase counts.  The caller keeps that
  // stream alive while the handle is in use.
  hipStream_t last_on = nullptr;
  hipEvent_t handoff = nullptr;
  hipGraphExec_t exec = nullptr;
  GraphKey key{};
  int warm = 0;  // eager calls made with the current key (the first builds plans / workspace)
  // exchange timing (profile mode, eager only)
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  // exchange mode "ipc" (wg_dist_ipc_local / wg_dist_ipc_connect)
  bool ipc = false;
  int64_t F_max = 0, slot_floats = 0;
  float* region = nullptr;            // [slot 0][slot 1][flags: world int64]
  int64_t* count = nullptr;           // phases completed (device)
  int32_t* err = nullptr;             // 1: a wait timed out; 2: a signal's release missed an XCD (device)
  uint32_t* arrive = nullptr;         // ipc_signal_kernel: [0] arrivals (0 between phases), [1] XCD mask
  int32_t n_xcc = 1;                  // XCDs of this device
  int32_t* halo_owner = nullptr;
  int32_t* halo_src = nullptr;
  std::vector<void*> peer_region;     // IPC-mapped, nullptr for self
  int64_t** peer_flags = nullptr;     // device array [world]
  IpcPull pull{};
  int64_t F_sig = 0;        // the signal columns of the running chain (<= the exchanged width)
  int64_t pads_zeroed = 0;  // the width whose halo pad columns the region holds as zeros
  // exchange mode "sdma" (wg_dist_ipc_sdma, after wg_dist_ipc_connect): each rank packs the rows
  // its peers asked for into one of two send buffers of its region; the receiver copies each
  // owner's packed block into its halo rows with hipMemcpyAsync on a copy stream (DMA engines
  // on a multi-GPU node: no CU time for the transfer), behind the same phase flags
  bool sdma = false;
  hipStream_t copy = nullptr;
  hipEvent_t cev[2] = {nullptr, nullptr};
  int64_t send_base = 0, send_floats = 0;  // mine: [send 0][send 1] at region + send_base
  std::vector<const float*> peer_send;     // peer q's send buffer 0 (mapped); buffer 1 at + peer_send_floats[q]
  std::vector<int64_t> peer_send_floats, peer_send_off;  // and the row where q packed my block

  ~wg_dist_s() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (comm) (void)ncclCommDestroy(comm);
    for (void* q : peer_region)
      if (q) (void)hipIpcCloseMemHandle(q);
    for (void* q : {(void*)region, (void*)count, (void*)err, (void*)arrive, (void*)halo_owner, (void*)halo_src,
                    (void*)peer_flags})
      (void)hipFree(q);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : cev)
      if (e) (void)hipEventDestroy(e);
    if (copy) (void)hipStreamDestroy(copy);
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    if (handoff) (void)hipEventDestroy(handoff);
    if (cap) (void)hipStreamDestroy(cap);
    (void)hipFree(send_rows);
    (void)hipFree(ws);
  }

  int mark(hipStream_t st, bool start) {
    if (!L->prof) return WG_OK;
    if (start) {
      while (ev.size() < ev_used + 2) {
        hipEvent_t e;
        WG_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        ev.push_back(e);
      }
      WG_HIP_TRY(hipEventRecord(ev[ev_used], st));
    } else {
      WG_HIP_TRY(hipEventRecord(ev[ev_used + 1], st));
      ev_used += 2;
    }
    return WG_OK;
  }

  int ipc_signal(hipStream_t st) {
    hipLaunchKernelGGL(ipc_signal_kernel, dim3(kIpcSignalBlocks), dim3(64), 0, st, count, world, rank, peer_flags,
                       arrive, n_xcc, err);
    WG_LAUNCH_CHECK();
    return WG_OK;
  }

  // (signal the previous phase, then) wait for the peers
  int ipc_wait_only(hipStream_t st, bool signal_first = false) {
    if (signal_first)
      if (int rc = ipc_signal(st)) return rc;
    hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, st, pull, 0);
    WG_LAUNCH_CHECK();
    return WG_OK;
  }

  // refresh the halo ext[n_own ...] (F floats per row) from the owners, then the step kernels
  // that gather it run on the same stream.  ipc: `slot` is the region slot ext lives in (the
  // owners' rows are read from the same slot of their regions); the previous phase's completion
  // is signalled by the one-workgroup kernel that then waits for the peers.  rccl: pack the rows
  // the peers asked for, one grouped send / receive straight into the halo rows.
  int exchange(float* ext, float* sendbuf, int64_t F, hipStream_t st, int slot = 0) {
    if (int rc = transfer(ext, sendbuf, F, st, slot)) return rc;
#ifdef WG_TIMING_PROBES
    if (L->tune.xdelay > 0 && n_halo > 0) {  // timing probe: simulated link time, one spinning wave
      hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, (uint64_t)(100.0 * L->tune.xdelay));
      WG_LAUNCH_CHECK();
    }
#endif
    return WG_OK;
  }

  int transfer(float* ext, float* sendbuf, int64_t F, hipStream_t st, int slot) {
    if (ipc && world == 1) return WG_OK;  // no peers: nothing to wait for or pull
    if (ipc && sdma) {
      if (int rc = mark(st, true)) return rc;
      // owner: this phase's rows for every peer, packed in the peers' halo order, then the
      // phase signalled (ipc_signal_kernel writes back every XCD's L2 before the flags)
      float* sb = region + send_base + slot * send_floats;
      if (n_send > 0) {
        launch_pack(n_send, F, send_rows, ext, sb, st);
        WG_LAUNCH_CHECK();
      }
      if (int rc = ipc_signal(st)) return rc;
      // receiver, on the copy stream: wait for every peer's signal of this phase, then one copy
      // per owner of its packed block into this rank's halo rows; the step waits for the copies
      WG_HIP_TRY(hipEventRecord(cev[0], st));
      WG_HIP_TRY(hipStreamWaitEvent(copy, cev[0], 0));
      hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, copy, pull, 0);
      WG_LAUNCH_CHECK();
      for (int q = 0; q < world; ++q) {
        if (q == rank || recv_cnt[q] == 0) continue;
        const float* from = peer_send[q] + slot * peer_send_floats[q] + peer_send_off[q] * F;
        WG_HIP_TRY(hipMemcpyAsync(ext + (n_own + recv_off[q]) * F, from, sizeof(float) * recv_cnt[q] * F,
                                  hipMemcpyDeviceToDevice, copy));
      }
      WG_HIP_TRY(hipEventRecord(cev[1], copy));
      WG_HIP_TRY(hipStreamWaitEvent(st, cev[1], 0));
      return mark(st, false);
    }
    if (ipc) {
      if (int rc = mark(st, true)) return rc;
      // one spinning workgroup signals and waits (ranks sharing a GPU in tests must not
      // starve each other's kernels), then full grids pull the halo rows
      if (int rc = ipc_wait_only(st, /*signal_first=*/true)) return rc;
      const int64_t total = n_halo * F;
      const bool v4 = (F % 4 == 0) && slot_floats * 4 < ((int64_t)1 << 31);
      // the columns that carry the signal (pad columns beyond them are zero on every owner)
      const int64_t Fr = std::min<int64_t>(F, (F_sig + 3) / 4 * 4);
      if (v4 && Fr < F && pads_zeroed != F) {  // pad columns of the halo rows (both slots) are never pulled
        for (int sl = 0; sl < 2; ++sl)
          WG_HIP_TRY(hipMemsetAsync(region + sl * slot_floats + n_own * F, 0, sizeof(float) * n_halo * F, st));
        pads_zeroed = F;
      }
      if (Fr >= F) pads_zeroed = 0;  // a full-width pull writes the columns a narrower signal leaves zero
      if (total > 0) {
        const int64_t work = v4 ? n_halo * (Fr / 4) : total;
        const int blocks = (int)std::min<int64_t>(65535, ceil_div(work, 256));
        if (v4)
          hipLaunchKernelGGL(ipc_pull4_kernel, dim3(blocks), dim3(256), 0, st, pull, slot, n_own, (int64_t)0, n_halo, F,
                             Fr, halo_owner, halo_src, ext);
        else
          hipLaunchKernelGGL(ipc_pull_kernel, dim3(blocks), dim3(256), 0, st, pull, slot, n_own, (int64_t)0, n_halo, F,
                             halo_owner, halo_src, ext);
        WG_LAUNCH_CHECK();
      }
      return mark(st, false);
    }
    if (world == 1 && n_send == 0) return WG_OK;
    if (int rc = mark(st, true)) return rc;
    if (n_send > 0) {
      launch_pack(n_send, F, send_rows, ext, sendbuf, st);
      WG_LAUNCH_CHECK();
    }
    if (int rc = nccl_try(ncclGroupStart(), "ncclGroupStart")) return rc;
    for (int q = 0; q < world; ++q) {
      if (send_cnt[q] > 0)
        if (int rc = nccl_try(ncclSend(sendbuf + send_off[q] * F, (size_t)(send_cnt[q] * F), ncclFloat32, q, comm, st),
                              "ncclSend")) {
          (void)ncclGroupEnd();
          return rc;
        }
      if (recv_cnt[q] > 0)
        if (int rc = nccl_try(ncclRecv(ext + (n_own + recv_off[q]) * F, (size_t)(recv_cnt[q] * F), ncclFloat32, q, comm,
                                       st),
                              "ncclRecv")) {
          (void)ncclGroupEnd();
          return rc;
        }
    }
    if (int rc = nccl_try(ncclGroupEnd(), "ncclGroupEnd")) return rc;
    return mark(st, false);
  }

  // the whole chain on stream st (eager, or being captured)
  int chain(const float* X0, int64_t F, int32_t K, double s, float* S, float* H, hipStream_t st) {
    Lds1Plan* lp = nullptr;
    if (F == 1 && K >= 1)
      if (int rc = get_lds1_plan(L, /*active_only=*/false, &lp)) return rc;
    const int64_t Fp = lp ? F : padded_features(L, F);  // internal width (zero pad columns, float4 lanes)
    F_sig = F;
    const size_t ext = ((size_t)n_cols * Fp + 63) / 64 * 64;
    const size_t own = ((size_t)n_own * Fp + 63) / 64 * 64;
    const size_t snd = ((size_t)std::max<int64_t>(n_send, 1) * Fp + 63) / 64 * 64;
    const size_t ulen = lp ? ((size_t)lp->u_floats() + 63) / 64 * 64 : 0;
    // lds: T ping-pong (own rows) + u ping-pong (padded column space); else T ping-pong over [own | halo]
    // F > 1 / weighted: heat sum by Clenshaw's recurrence (as wg_wavelet_features), X0 kept in its own buffer
    const bool clen = !lp && L->tune.clenshaw && K >= 1;
    const size_t need = (lp ? 2 * own + (ipc ? 0 : 2 * ulen) : (ipc ? 0 : 2 * ext)) + own + snd + (clen ? own : 0);
    if (ws_floats < need) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      WG_HIP_TRY(hipStreamIsCapturing(st, &cs));
      if (cs != hipStreamCaptureStatusNone) return fail(WG_ERR_UNSUPPORTED, "wg_dist: workspace growth during capture");
      WG_HIP_TRY(hipStreamSynchronize(st));
      (void)hipFree(ws);
      ws = nullptr;
      ws_floats = 0;
      WG_HIP_TRY(hipMalloc(&ws, need * sizeof(float)));
      ws_floats = need;
    }
    float* p = ws;
    auto take = [&](size_t n) {
      float* q = p;
      p += n;
      return q;
    };
    // ipc: the exchanged vectors live in the shared region's two slots, and
    // every phase (first vector, each step) is bracketed by wait and signal
    if (ipc && (lp ? (int64_t)ulen : (int64_t)ext) > slot_floats)
      return fail(WG_ERR_UNSUPPORTED, "wg_dist: F=%lld exceeds the IPC region (F_max=%lld)", (long long)F,
                  (long long)F_max);
    const bool sig = ipc && K >= 1 && world > 1;
    if (lp) {
      float* T[2] = {take(own), take(own)};
      float* U[2] = {ipc ? region : take(ulen), ipc ? region + slot_floats : take(ulen)};
      float* sint = take(own);
      float* sendbuf = take(snd);
      int rc = launch_permute(L, 0, 1, X0, T[0], st);
      if (!rc && sig) rc = ipc_wait_only(st);
      if (!rc) rc = launch_scale_dinv(L, n_own, T[0], U[0], st);
      for (int32_t k = 1; k <= K && !rc; ++k) {  // the exchange signals phase k-1, then waits
        rc = exchange(U[(k - 1) & 1], sendbuf, 1, st, (k - 1) & 1);
        if (!rc)
          rc = launch_lds1_step(L, lp, k, U[(k - 1) & 1], T[(k - 1) & 1], k >= 2 ? T[k & 1] : nullptr,
                                k == K ? nullptr : T[k & 1], k == K ? nullptr : U[k & 1], sint, 1.0,
                                std::exp(-s * (double)k), st);
      }
      if (!rc && sig) rc = ipc_signal(st);  // phase K
      if (!rc) rc = launch_finalize(L, 1, sint, nullptr, 0.0, S, H, st);
      return rc;
    }
    float* A[2] = {ipc ? region : take(ext), ipc ? region + slot_floats : take(ext)};
    float* sint = take(own);
    float* sendbuf = take(snd);
    int rc = WG_OK;
    if (sig) rc = ipc_wait_only(st);
    // unweighted (u = b * dinv exchanged) Clenshaw chains at an unpadded width: one pass writes X0
    // (internal order), u_0 = X0 * dinv into slot 0, the closed-form rows' S / H straight to the
    // caller's rows and zeros to their u rows in both slots; the last step writes S / H of the
    // active rows to the caller's rows (no finalize pass) -- as wg_wavelet_features
    const int useu_f = (L->unit && L->values_null && L->tune.uscale && L->tune.hot == 0) ? 1 : 0;
    const bool fused = !lp && L->tune.clenshaw && K >= 1 && useu_f && Fp == F && L->tune.fuse_finalize && S && H &&
                       step_single_tile(L, F, {A[0], A[1], S, H});
    float* x0f = fused ? take(own) : nullptr;
    double coef_f = 0.0;  // closed-form rows: S = X0 * sum_k (-1)^k c_k (as wg_wavelet_features)
    for (int32_t k = 0; k <= K; ++k) coef_f += ((k & 1) ? -1.0 : 1.0) * std::exp(-s * (double)k);
    if (!rc)
      rc = fused ? launch_permute_in_closed(L, F, X0, x0f, coef_f, S, H, A[0], st, A[1])
                 : launch_permute_pad(L, F, Fp, X0, A[0], st);
    if (!rc && K == 0)
      rc = hipMemcpyAsync(sint, A[0], sizeof(float) * n_own * Fp, hipMemcpyDeviceToDevice, st) == hipSuccess
               ? WG_OK
               : fail(WG_ERR_HIP, "wg_dist: copy");
    if (clen) {
      // b_K = c_K X0 implicit; b_k = c_k X0 + 2 L_hat b_{k+1} - b_{k+2} written over b_{k+2} (own rows)
      // in the slot the forward chain would write; S = c_0 X0 + L_hat b_1 - b_2 (capi.hip).
      // Phase j = 1..K exchanges slot (j-1)&1, exactly as the forward chain's step j.
      float* x0 = fused ? x0f : take(own);
      if (!rc && !fused &&
          hipMemcpyAsync(x0, A[0], sizeof(float) * n_own * Fp, hipMemcpyDeviceToDevice, st) != hipSuccess)
        rc = fail(WG_ERR_HIP, "wg_dist: copy X0");
      std::vector<double> c(K + 1);
      for (int32_t k = 0; k <= K; ++k) c[k] = std::exp(-s * (double)k);
      // unweighted graph (every rank created its shard with values == NULL): the stored b_k
      // are u_k = b_k * dinv, so the gathers read no CSR values (as wg_wavelet_features,
      // DESIGN.md 4.1) and the halo rows exchanged are u rows; X0 (phase 1) stays unscaled
      const int useu = (L->unit && L->values_null && L->tune.uscale &&
                        L->tune.hot == 0) ? 1 : 0;
      // phase 1 exchanges and gathers u_0 = X0 * dinv (own rows scaled in place; x0 keeps X0)
      // value-free like every later phase.  The choice depends only on useu, which every rank
      // shares (values == NULL on every shard), never on this rank's own hybrid-step plan: the
      // halo rows a rank receives in phase 1 must be in the format it gathers (a
      // shard that declined its plan must not send unscaled rows to one that took it).
      const bool u0 = useu && K >= 1;
      if (!rc && u0 && !fused) rc = launch_scale_rows(L, n_own, Fp, x0, A[0], st);
      // the closed-form own rows [n_active, n_own) are never written by the steps (active rows only)
      // nor gathered, but a hybrid step's dense tile stages whole 32-row column tiles: keep them
      // zero in the other slot (finite u_0 in A[0]) so that 0 x stale never enters an MFMA sum
      if (!rc && !fused && L->n_active < n_own &&
          hipMemsetAsync(A[1] + L->n_active * Fp, 0, sizeof(float) * (n_own - L->n_active) * Fp, st) != hipSuccess)
        rc = fail(WG_ERR_HIP, "wg_dist: zero the closed-form rows");
      for (int32_t j = 1; j <= K && !rc; ++j) {
        const int32_t k = K - j;  // this phase computes b_k (k = 0: the final S)
        float* cur = A[(j - 1) & 1];
        const bool prev_stored = j >= 3;  // b_{k+2} in slot j&1 (j == 2: the implicit b_K; j == 1: zero)
        const double ck = c[k] - (j == 2 ? c[K] : 0.0);
        const double cacc = (j == 1) ? (k == 0 ? c[K] : 2.0 * c[K]) : (k == 0 ? 1.0 : 2.0);
        ClenArgs cl{x0, ck, cacc, k == 0 ? 1 : 0};
        cl.uin = useu && (j >= 2 || u0);  // j == 1 gathers X0 itself, or u_0
        cl.uprev = useu && prev_stored;
        cl.uout = useu;                   // ignored on the final step (k == 0 writes S)
        rc = exchange(cur, sendbuf, Fp, st, (j - 1) & 1);
        // only the active rows: purely isolated own rows (no entries, w = 0; relabelled to the end
        // of the shard by the prologue) are never gathered by any rank and have T_k = (-1)^k X0, so
        // their S is written in closed form by the fused permute-in or the finalize below (WATS.py:55,
        // -1 diagonal)
        if (!rc)
          rc = launch_step(L, 2, Fp, cur, prev_stored ? A[j & 1] : nullptr, k == 0 ? nullptr : A[j & 1],
                           k == 0 ? sint : nullptr, (k == 0 && fused) ? H : nullptr, 1.0, 0.0, st,
                           /*active_only=*/true, (k == 0 && fused) ? S : nullptr, &cl);
      }
      if (!rc && sig) rc = ipc_signal(st);  // phase K
      if (!rc && !fused) {
        double coef = 0.0;  // closed-form rows: S = X0 * sum_k (-1)^k c_k (as wg_wavelet_features)
        for (int32_t k = 0; k <= K; ++k) coef += ((k & 1) ? -1.0 : 1.0) * c[k];
        rc = launch_finalize(L, F, sint, x0, coef, S, H, st, Fp);
      }
      return rc;
    } else {
      for (int32_t k = 1; k <= K && !rc; ++k) {
        float* cur = A[(k - 1) & 1];
        rc = exchange(cur, sendbuf, Fp, st, (k - 1) & 1);
        if (!rc)
          rc = launch_step(L, k, Fp, cur, k >= 2 ? A[k & 1] : nullptr, k == K ? nullptr : A[k & 1], sint, nullptr,
                           1.0, std::exp(-s * (double)k), st);
      }
    }
    if (!rc && sig) rc = ipc_signal(st);  // phase K
    if (!rc) rc = launch_finalize(L, F, sint, nullptr, 0.0, S, H, st, Fp);
    return rc;
  }
};

extern "C" {

int wg_dist_unique_id(void* out) {
  if (!out) return fail(WG_ERR_INVALID, "wg_dist_unique_id: NULL");
  ncclUniqueId id;
  if (int rc = nccl_try(ncclGetUniqueId(&id), "ncclGetUniqueId")) return rc;
  std::memcpy(out, &id, sizeof(id));
  return WG_OK;
}

int wg_dist_create(wg_laplacian_t L, const void* unique_id, int32_t rank, int32_t world, const int32_t* send_rows,
                   const int64_t* send_counts, const int64_t* recv_counts, wg_dist_t* out) {
  if (!out) return fail(WG_ERR_INVALID, "wg_dist_create: out is NULL");
  *out = nullptr;
  if (!L || world < 1 || rank < 0 || rank >= world || !send_counts || !recv_counts)
    return fail(WG_ERR_INVALID, "wg_dist_create: bad arguments (rank=%d world=%d)", rank, world);
  auto* D = new wg_dist_s();
  D->L = L;
  D->rank = rank;
  D->world = world;
  D->n_own = L->n_rows;
  D->n_cols = L->n_cols;
  const int64_t nc = world;
  D->send_cnt.assign(send_counts, send_counts + nc);
  D->recv_cnt.assign(recv_counts, recv_counts + nc);
  D->send_off.assign(nc + 1, 0);
  D->recv_off.assign(nc + 1, 0);
  for (int64_t i = 0; i < nc; ++i) {
    if (D->send_cnt[i] < 0 || D->recv_cnt[i] < 0) {
      delete D;
      return fail(WG_ERR_INVALID, "wg_dist_create: negative count for peer %d", (int)i);
    }
    D->send_off[i + 1] = D->send_off[i] + D->send_cnt[i];
    D->recv_off[i + 1] = D->recv_off[i] + D->recv_cnt[i];
  }
  D->n_send = D->send_off[nc];
  D->n_halo = D->recv_off[nc];
  if (D->n_halo > 0 && D->n_own + D->n_halo == L->n_cols) {
    // the halo groups (one per peer, each in descending degree: wats_hip/dist.py) for
    // the F = 1 hub plan of a shard; plans built before this point are dropped
    L->halo_off.assign(D->recv_off.begin(), D->recv_off.end());
    release_lds1(L);
  }
  if (D->n_own + D->n_halo != D->n_cols || (D->n_send > 0 && !send_rows)) {
    const long long nh = (long long)D->n_halo, nc = (long long)D->n_cols, no = (long long)D->n_own;
    delete D;
    return fail(WG_ERR_INVALID, "wg_dist_create: halo rows %lld + own rows %lld != handle columns %lld", nh, no, nc);
  }
  int rc = WG_OK;
  if (D->n_send > 0) {
    rc = dmalloc(&D->send_rows, (size_t)D->n_send);
    if (!rc && hipMemcpy(D->send_rows, send_rows, sizeof(int32_t) * D->n_send, hipMemcpyDefault) != hipSuccess)
      rc = fail(WG_ERR_HIP, "wg_dist_create: send_rows copy");
  }
  if (!rc && (hipStreamCreateWithFlags(&D->cap, hipStreamNonBlocking) != hipSuccess ||
              hipEventCreateWithFlags(&D->fork, hipEventDisableTiming) != hipSuccess ||
              hipEventCreateWithFlags(&D->join, hipEventDisableTiming) != hipSuccess ||
              hipEventCreateWithFlags(&D->handoff, hipEventDisableTiming) != hipSuccess))
    rc = fail(WG_ERR_HIP, "wg_dist_create: stream/event");
  if (!rc && unique_id) {  // NULL: no RCCL communicator (one-sided IPC exchange, wg_dist_ipc_*)
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    rc = nccl_try(ncclCommInitRank(&D->comm, world, id, rank), "ncclCommInitRank");
  }
  if (rc) {
    delete D;
    return rc;
  }
  *out = D;
  return WG_OK;
}

int wg_dist_destroy(wg_dist_t D) {
  if (!D) return WG_OK;
  (void)hipDeviceSynchronize();
  if (D->ipc && D->world > 1 && D->cap) {
    // peers may still pull from this rank's region in their last phase: wait until
    // every peer has completed as many phases as this rank (its last write here is
    // its final signal), then unmap and free.  A lost peer times out (60 s).
    hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, D->cap, D->pull, 0);
    (void)hipStreamSynchronize(D->cap);
  }
  delete D;
  return WG_OK;
}

int wg_dist_set_graph(wg_dist_t D, int32_t enable) {
  if (!D) return fail(WG_ERR_INVALID, "wg_dist_set_graph: NULL handle");
  D->use_graph = enable != 0;
  return WG_OK;
}

int wg_dist_wavelet_features(wg_dist_t D, const float* X0, int64_t F, int32_t K, double s, float* S, float* H,
                             void* stream_) {
  if (!D || F < 1 || K < 0 || (D->n_own && (!X0 || !S || !H)))  // an empty shard passes no rows
    return fail(WG_ERR_INVALID, "wg_dist_wavelet_features: bad arguments (F=%lld K=%d)", (long long)F, K);
  if (!D->comm && !D->ipc && (D->n_send > 0 || D->n_halo > 0 || D->world > 1))
    return fail(WG_ERR_INVALID, "wg_dist_wavelet_features: no exchange (no RCCL id given and IPC not connected)");
  hipStream_t st = as_stream(stream_);
  const GraphKey key{X0, S, H, F, K, s, D->L->tune_gen};
  if (!(key == D->key)) {
    if (D->exec) {
      WG_HIP_TRY(hipDeviceSynchronize());  // its last replay ran on some caller stream
      (void)hipGraphExecDestroy(D->exec);
      D->exec = nullptr;
      D->last_on = nullptr;
    }
    D->key = key;
    D->warm = 0;
  }
  // order this chain after the handle's previous one when that ran on another stream (no event
  // per call on the usual path: the marker is recorded only when the stream changes)
  auto after_last = [&](hipStream_t target) -> int {
    if (D->last_on && D->last_on != target) {
      WG_HIP_TRY(hipEventRecord(D->handoff, D->last_on));
      WG_HIP_TRY(hipStreamWaitEvent(target, D->handoff, 0));
    }
    D->last_on = target;
    return WG_OK;
  };
  // eager: profiling (per-step events), graphs disabled, or the first call with
  // these arguments (it builds the kernel plans and the workspace).  Either way the chain
  // runs on the handle's own non-blocking stream (cap), joined to the caller's: on the legacy
  // null stream the step kernels would wait for every blocking stream's work.
  if (!D->use_graph || D->L->prof || D->warm == 0 || hybrid_conc_in_use(D->L, F)) {
    if (int rc = after_last(D->cap)) return rc;
    WG_HIP_TRY(hipEventRecord(D->fork, st));
    WG_HIP_TRY(hipStreamWaitEvent(D->cap, D->fork, 0));
    const int rc = D->chain(X0, F, K, s, S, H, D->cap);
    if (!rc) ++D->warm;
    WG_HIP_TRY(hipEventRecord(D->join, D->cap));
    WG_HIP_TRY(hipStreamWaitEvent(st, D->join, 0));
    return rc;
  }
  if (!D->exec) {
    hipGraph_t g = nullptr;
    WG_HIP_TRY(hipEventRecord(D->fork, st));  // capture on the handle's stream (the caller's may be the null one)
    WG_HIP_TRY(hipStreamWaitEvent(D->cap, D->fork, 0));
    WG_HIP_TRY(hipStreamBeginCapture(D->cap, hipStreamCaptureModeRelaxed));
    const int rc = D->chain(X0, F, K, s, S, H, D->cap);
    const hipError_t ec = hipStreamEndCapture(D->cap, &g);
    if (rc) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    if (ec != hipSuccess) return fail(WG_ERR_HIP, "wg_dist: capture failed: %s", hipGetErrorString(ec));
    const hipError_t ei = hipGraphInstantiate(&D->exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) {
      D->exec = nullptr;
      return fail(WG_ERR_HIP, "wg_dist: graph instantiate: %s", hipGetErrorString(ei));
    }
  }
  // the replay goes straight into the caller's stream: a fork / join through the handle's stream
  // per call left ~25-30 us of idle GPU between back-to-back chains (r04 s35 kernel trace)
  if (int rc = after_last(st)) return rc;
  WG_HIP_TRY(hipGraphLaunch(D->exec, st));
  return WG_OK;
}

int wg_dist_ipc_local(wg_dist_t D, int64_t F_max, void* blob) {
  if (!D || F_max < 1 || !blob) return fail(WG_ERR_INVALID, "wg_dist_ipc_local: bad arguments");
  if (D->world > kMaxPeers) return fail(WG_ERR_UNSUPPORTED, "wg_dist_ipc_local: world > %d", kMaxPeers);
  if (D->region) return fail(WG_ERR_INVALID, "wg_dist_ipc_local: already set up");
  // a slot holds the extended vector at F_max, or the F = 1 LDS kernel's u (padded column space)
  int64_t ulen = 0;
  Lds1Plan* lp = nullptr;
  if (int rc = get_lds1_plan(D->L, /*active_only=*/false, &lp)) return rc;
  if (lp) ulen = lp->u_floats();
  D->F_max = F_max;
  D->slot_floats = (std::max<int64_t>(D->n_cols * padded_features(D->L, F_max), ulen) + 63) / 64 * 64;
  // [slot 0][slot 1][flags: world int64][send 0][send 1] (the send buffers: exchange mode "sdma")
  D->send_base = (2 * D->slot_floats + 2 * (int64_t)D->world + 63) / 64 * 64;
  D->send_floats = (std::max<int64_t>(D->n_send, 1) * padded_features(D->L, F_max) + 63) / 64 * 64;
  const size_t bytes = sizeof(float) * (D->send_base + 2 * D->send_floats);
  if (int rc = dmalloc(reinterpret_cast<char**>(&D->region), bytes)) return rc;
  if (int rc = dmalloc(&D->count, 1)) return rc;
  if (int rc = dmalloc(&D->err, 1)) return rc;
  if (int rc = dmalloc(&D->arrive, 2)) return rc;
  WG_HIP_TRY(hipMemset(D->arrive, 0, 2 * sizeof(uint32_t)));
  {
    int dev = 0, nx = 1;
    WG_HIP_TRY(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || nx < 1) nx = 1;
    D->n_xcc = std::min(nx, 16);
  }
  WG_HIP_TRY(hipMemset(D->region, 0, bytes));
  WG_HIP_TRY(hipMemset(D->count, 0, sizeof(int64_t)));
  WG_HIP_TRY(hipMemset(D->err, 0, sizeof(int32_t)));
  hipIpcMemHandle_t h;
  WG_HIP_TRY(hipIpcGetMemHandle(&h, D->region));
  char* out = static_cast<char*>(blob);
  std::memset(out, 0, 128);
  std::memcpy(out, &h, sizeof(h));
  std::memcpy(out + 64, &D->slot_floats, sizeof(int64_t));
  std::memcpy(out + 72, &D->send_base, sizeof(int64_t));
  std::memcpy(out + 80, &D->send_floats, sizeof(int64_t));
  WG_HIP_TRY(hipDeviceSynchronize());
  return WG_OK;
}

int wg_dist_ipc_connect(wg_dist_t D, const void* blobs, const int32_t* halo_src) {
  if (!D || !blobs || (D->n_halo > 0 && !halo_src)) return fail(WG_ERR_INVALID, "wg_dist_ipc_connect: bad arguments");
  if (!D->region) return fail(WG_ERR_INVALID, "wg_dist_ipc_connect: call wg_dist_ipc_local first");
  if (D->ipc || !D->peer_region.empty()) return fail(WG_ERR_INVALID, "wg_dist_ipc_connect: already connected");
  const char* b = static_cast<const char*>(blobs);
  D->peer_region.assign(D->world, nullptr);
  D->peer_send.assign(D->world, nullptr);
  D->peer_send_floats.assign(D->world, 0);
  std::vector<int64_t*> pf(D->world, nullptr);
  IpcPull p{};
  for (int q = 0; q < D->world; ++q) {
    hipIpcMemHandle_t h;
    int64_t sf = 0;
    std::memcpy(&h, b + 128 * q, sizeof(h));
    std::memcpy(&sf, b + 128 * q + 64, sizeof(int64_t));
    int64_t sbase = 0, sfl = 0;
    std::memcpy(&sbase, b + 128 * q + 72, sizeof(int64_t));
    std::memcpy(&sfl, b + 128 * q + 80, sizeof(int64_t));
    float* base = D->region;
    if (q != D->rank) {
      void* mp = nullptr;
      WG_HIP_TRY(hipIpcOpenMemHandle(&mp, h, hipIpcMemLazyEnablePeerAccess));
      D->peer_region[q] = mp;
      base = static_cast<float*>(mp);
    }
    p.slot_base[q] = base;
    p.slot_floats[q] = sf;
    D->peer_send[q] = base + sbase;
    D->peer_send_floats[q] = sfl;
    pf[q] = reinterpret_cast<int64_t*>(base + 2 * sf);
  }
  if (int rc = dmalloc(&D->peer_flags, (size_t)D->world)) return rc;
  WG_HIP_TRY(hipMemcpy(D->peer_flags, pf.data(), sizeof(int64_t*) * D->world, hipMemcpyHostToDevice));
  std::vector<int32_t> owner(D->n_halo);
  for (int q = 0; q < D->world; ++q)
    for (int64_t i = D->recv_off[q]; i < D->recv_off[q + 1]; ++i) owner[i] = (int32_t)q;
  if (D->n_halo > 0) {
    if (int rc = dmalloc(&D->halo_owner, (size_t)D->n_halo)) return rc;
    if (int rc = dmalloc(&D->halo_src, (size_t)D->n_halo)) return rc;
    WG_HIP_TRY(hipMemcpy(D->halo_owner, owner.data(), sizeof(int32_t) * D->n_halo, hipMemcpyHostToDevice));
    WG_HIP_TRY(hipMemcpy(D->halo_src, halo_src, sizeof(int32_t) * D->n_halo, hipMemcpyDefault));
  }
  p.flags = reinterpret_cast<const int64_t*>(D->region + 2 * D->slot_floats);
  p.count = D->count;
  p.peer_flags = D->peer_flags;
  p.err = D->err;
  p.world = D->world;
  p.rank = D->rank;
  D->pull = p;
  D->ipc = true;
  return WG_OK;
}

int wg_dist_ipc_sdma(wg_dist_t D, const int64_t* peer_send_off) {
  if (!D || !peer_send_off) return fail(WG_ERR_INVALID, "wg_dist_ipc_sdma: NULL argument");
  if (!D->ipc) return fail(WG_ERR_INVALID, "wg_dist_ipc_sdma: call wg_dist_ipc_connect first");
  for (int q = 0; q < D->world; ++q)
    if (q != D->rank && D->recv_cnt[q] > 0 &&
        (peer_send_off[q] < 0 ||
         (peer_send_off[q] + D->recv_cnt[q]) * padded_features(D->L, D->F_max) > D->peer_send_floats[q]))
      return fail(WG_ERR_INVALID, "wg_dist_ipc_sdma: rank %d's block for this rank lies outside its send buffer", q);
  WG_HIP_TRY(hipDeviceSynchronize());
  if (!D->copy) WG_HIP_TRY(hipStreamCreateWithFlags(&D->copy, hipStreamNonBlocking));
  for (hipEvent_t& e : D->cev)
    if (!e) WG_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  D->peer_send_off.assign(peer_send_off, peer_send_off + D->world);
  D->sdma = true;
  if (D->exec) {  // a chain captured with the pull exchange is not replayed
    (void)hipGraphExecDestroy(D->exec);
    D->exec = nullptr;
  }
  D->warm = 0;
  return WG_OK;
}

int wg_dist_status(wg_dist_t D, int32_t* timed_out) {
  if (!D || !timed_out) return fail(WG_ERR_INVALID, "wg_dist_status: NULL argument");
  *timed_out = 0;
  if (!D->err) return WG_OK;
  WG_HIP_TRY(hipDeviceSynchronize());
  WG_HIP_TRY(hipMemcpy(timed_out, D->err, sizeof(int32_t), hipMemcpyDeviceToHost));
  return WG_OK;
}

int wg_dist_info(wg_dist_t D, int64_t* out) {
  if (!D || !out) return fail(WG_ERR_INVALID, "wg_dist_info: NULL argument");
  out[0] = 0;  // exchange, then the step (the overlap variants of round 2 are removed)
  out[1] = D->n_own;
  out[2] = D->n_halo;
  out[3] = D->n_send;
  out[4] = D->world;
  out[5] = D->ipc ? (D->sdma ? 3 : 1) : (D->comm ? 2 : 0);
  out[6] = D->exec ? 1 : 0;
  out[7] = 1;  // halo tiers
  return WG_OK;
}

int wg_dist_profile_collect(wg_dist_t D, double* exchange_ms, int64_t* count) {
  if (!D || !exchange_ms || !count) return fail(WG_ERR_INVALID, "wg_dist_profile_collect: NULL argument");
  double tot = 0.0;
  for (size_t i = 0; i + 1 < D->ev_used; i += 2) {
    WG_HIP_TRY(hipEventSynchronize(D->ev[i + 1]));
    float ms = 0.0f;
    WG_HIP_TRY(hipEventElapsedTime(&ms, D->ev[i], D->ev[i + 1]));
    tot += ms;
  }
  *exchange_ms = tot;
  *count = (int64_t)(D->ev_used / 2);
  D->ev_used = 0;
  return WG_OK;
}

}  // extern "C"
