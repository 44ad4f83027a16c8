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
  bool operator==(const GraphKey& o) const {
    return X0 == o.X0 && S == o.S && H == o.H && F == o.F && K == o.K && s == o.s;
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
  std::vector<int64_t> send_cnt, recv_cnt, send_off, recv_off;
  float* ws = nullptr;
  size_t ws_floats = 0;
  bool use_graph = true;
  hipStream_t cap = nullptr;  // capture / replay stream (the caller's may be the null stream)
  hipEvent_t fork = nullptr, join = nullptr;
  hipGraphExec_t exec = nullptr;
  GraphKey key{};
  int warm = 0;  // eager calls made with the current key (the first builds plans / workspace)
  // exchange timing (profile mode, eager only)
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;

  ~wg_dist_s() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (comm) (void)ncclCommDestroy(comm);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
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

  // refresh the halo rows ext[n_own ...] (F floats per row) from their owners
  int exchange(float* ext, float* sendbuf, int64_t F, hipStream_t st) {
    if (world == 1 && n_send == 0) return WG_OK;
    if (int rc = mark(st, true)) return rc;
    if (n_send > 0) {
      hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)ceil_div(n_send * F, 256)), dim3(256), 0, st, n_send, F,
                         send_rows, ext, sendbuf);
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
        if (int rc = nccl_try(ncclRecv(ext + (n_own + recv_off[q]) * F, (size_t)(recv_cnt[q] * F), ncclFloat32, q,
                                       comm, st),
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
    const size_t ext = ((size_t)n_cols * F + 63) / 64 * 64;
    const size_t own = ((size_t)n_own * F + 63) / 64 * 64;
    const size_t snd = ((size_t)std::max<int64_t>(n_send, 1) * F + 63) / 64 * 64;
    const size_t ulen = lp ? ((size_t)lp->lchunks * lp->nb * 32 + 63) / 64 * 64 : 0;
    // lds: T ping-pong (own rows) + u ping-pong (padded column space); else T ping-pong over [own | halo]
    const size_t need = (lp ? 2 * own + 2 * ulen : 2 * ext) + own + snd;
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
    if (lp) {
      float* T[2] = {take(own), take(own)};
      float* U[2] = {take(ulen), take(ulen)};
      float* sint = take(own);
      float* sendbuf = take(snd);
      int rc = launch_permute(L, 0, 1, X0, T[0], st);
      if (!rc) rc = launch_scale_dinv(L, n_own, T[0], U[0], st);
      for (int32_t k = 1; k <= K && !rc; ++k) {
        rc = exchange(U[(k - 1) & 1], sendbuf, 1, st);
        if (!rc)
          rc = launch_lds1_step(L, lp, k, U[(k - 1) & 1], T[(k - 1) & 1], k >= 2 ? T[k & 1] : nullptr,
                                k == K ? nullptr : T[k & 1], k == K ? nullptr : U[k & 1], sint, 1.0,
                                std::exp(-s * (double)k), st);
      }
      if (!rc) rc = launch_finalize(L, 1, sint, nullptr, 0.0, S, H, st);
      return rc;
    }
    float* A[2] = {take(ext), take(ext)};
    float* sint = take(own);
    float* sendbuf = take(snd);
    int rc = launch_permute(L, 0, F, X0, A[0], st);
    if (!rc && K == 0)
      rc = hipMemcpyAsync(sint, A[0], sizeof(float) * n_own * F, hipMemcpyDeviceToDevice, st) == hipSuccess
               ? WG_OK
               : fail(WG_ERR_HIP, "wg_dist: copy");
    for (int32_t k = 1; k <= K && !rc; ++k) {
      float* cur = A[(k - 1) & 1];
      rc = exchange(cur, sendbuf, F, st);
      if (!rc)
        rc = launch_step(L, k, F, cur, k >= 2 ? A[k & 1] : nullptr, k == K ? nullptr : A[k & 1], sint, nullptr, 1.0,
                         std::exp(-s * (double)k), st);
    }
    if (!rc) rc = launch_finalize(L, F, sint, nullptr, 0.0, S, H, st);
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
  if (!L || !unique_id || world < 1 || rank < 0 || rank >= world || !send_counts || !recv_counts)
    return fail(WG_ERR_INVALID, "wg_dist_create: bad arguments (rank=%d world=%d)", rank, world);
  auto* D = new wg_dist_s();
  D->L = L;
  D->rank = rank;
  D->world = world;
  D->n_own = L->n_rows;
  D->n_cols = L->n_cols;
  D->send_cnt.assign(send_counts, send_counts + world);
  D->recv_cnt.assign(recv_counts, recv_counts + world);
  D->send_off.assign(world + 1, 0);
  D->recv_off.assign(world + 1, 0);
  for (int q = 0; q < world; ++q) {
    if (D->send_cnt[q] < 0 || D->recv_cnt[q] < 0) {
      delete D;
      return fail(WG_ERR_INVALID, "wg_dist_create: negative count for peer %d", q);
    }
    D->send_off[q + 1] = D->send_off[q] + D->send_cnt[q];
    D->recv_off[q + 1] = D->recv_off[q] + D->recv_cnt[q];
  }
  D->n_send = D->send_off[world];
  D->n_halo = D->recv_off[world];
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
              hipEventCreateWithFlags(&D->join, hipEventDisableTiming) != hipSuccess))
    rc = fail(WG_ERR_HIP, "wg_dist_create: stream/event");
  if (!rc) {
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
  if (!D || F < 1 || K < 0 || !S || !H || (D->n_own && !X0))
    return fail(WG_ERR_INVALID, "wg_dist_wavelet_features: bad arguments (F=%lld K=%d)", (long long)F, K);
  hipStream_t st = as_stream(stream_);
  const GraphKey key{X0, S, H, F, K, s};
  if (!(key == D->key)) {
    if (D->exec) {
      WG_HIP_TRY(hipStreamSynchronize(D->cap));
      (void)hipGraphExecDestroy(D->exec);
      D->exec = nullptr;
    }
    D->key = key;
    D->warm = 0;
  }
  // eager: profiling (per-step events), graphs disabled, or the first call with
  // these arguments (it builds the kernel plans and the workspace)
  if (!D->use_graph || D->L->prof || D->warm == 0) {
    const int rc = D->chain(X0, F, K, s, S, H, st);
    if (!rc) ++D->warm;
    return rc;
  }
  WG_HIP_TRY(hipEventRecord(D->fork, st));
  WG_HIP_TRY(hipStreamWaitEvent(D->cap, D->fork, 0));
  if (!D->exec) {
    hipGraph_t g = nullptr;
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
  WG_HIP_TRY(hipGraphLaunch(D->exec, D->cap));
  WG_HIP_TRY(hipEventRecord(D->join, D->cap));
  WG_HIP_TRY(hipStreamWaitEvent(st, D->join, 0));
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
