// NOT BUILT -- a measured dead end kept for the record: the persistent
// LDS-hub wave kernel for F = 40 was slower than cheb_step_kernel at every hub size
// (profiles/r03/s15-s18_hubw_*.log).  It referenced internal.h declarations since removed.

// hub.hip -- the LDS-hub wave kernel: the Chebyshev / Clenshaw step for wide
// signals (F > 1, float4 lanes) with the hub rows of the gathered vector in
// LDS (reference calibration/WATS.py:32-36 recurrence; heat sum :65-68 and
// normalisation :71-72 in the shared epilogue, step_dev.h).
//
// Why.  The gather kernel (cheb_step_kernel) is bound by L1->L2 line requests:
// every nonzero of an F = 40 step fetches a 160-B row of T_{k-1} / u as two
// 128-B lines, ~56 requests in flight per CU at ~330 cycles.
// After the descending-degree relabelling the lowest column ids take most of
// the gathers (ogbn-arxiv-size R-MAT: the top 1 000 of 94 k columns 35 %);
// from LDS they cost no L1 request at all.  Round 1's LDS hub (a persistent
// workgroup walking the plan's 4-wave units with a barrier per unit) lost to
// the non-persistent kernel: every unit waited for its slowest wave.  Here:
//
//  * one 1024-thread workgroup per CU stages rows [0, H) of the gathered
//    vector (H x W floats, up to ~157 KB) once per launch;
//  * every WAVE pulls its own work from per-XCD queues (a returning atomic per
//    batch of units, stealing from the other queues when its own is empty), so
//    no wave waits for another;
//  * a unit is one wave pass over up to G / LN team rows (LN sub-groups per
//    row), or one chunk of a long row (the chunk's float64 partial stored
//    write-through, an arrival counter per row, the last chunk combining in
//    chunk order and running the epilogue -- step.hip's split-row hand-off at
//    wave granularity);
//  * rows are column-sorted, so a row's hub entries are a prefix: the prefix
//    is summed from LDS (ds_read_b128), the rest gathered from global memory,
//    with the cooperative index loads of accumulate_bcast;
//  * the last workgroup out resets the queue heads for the next launch.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "step_dev.h"

namespace wg {
namespace {

constexpr int kHubThreads = 1024;
constexpr int kQueues = 32;  // workgroup b pulls from queue b % 32 (four per XCD: b % 8 is its XCD)
constexpr int kCtrStride = 64;  // queue heads 256 B apart (one returning atomic per word saturates at
                                // ~88 per us, MI355X_MICROARCH.md dequeue row)

extern __shared__ __align__(16) float g_hubw_lds[];

struct HubArgs {
  const int4* units;     // {row, e0, e1, chunk} split chunks / {first row, rows, LN, -1} team passes
  int32_t n_units;
  int32_t batch;         // units per dequeue
  int32_t* ctr;          // [kQueues + 1] * kCtrStride: queue heads, then the workgroups-done count
  const int32_t* hsplit; // [rows] first entry with column >= H (rows column-sorted)
  int32_t H;             // hub rows in LDS
  const int2* rowchunks; // split rows: {first chunk, chunks} by internal row
  int32_t* arrivals;     // split rows: monotonic arrival counters by internal row
  double* partial;       // [chunks][W]
};

// accumulate_bcast with the gathered rows read from the LDS hub (hub = this lane's column slice)
template <int VEC, int U>
__device__ __forceinline__ void accumulate_bcast_lds(const StepArgs& a, int32_t e, int32_t e1, int32_t stride,
                                                     const float* hub, int W, double (&acc)[VEC], int fs, int base) {
  const int LF = a.LF;
  if (e >= e1) return;
  const int32_t n = (e1 - e + stride - 1) / stride;
  for (int32_t t0 = 0; t0 < n; t0 += LF) {
    const int32_t tt = t0 + fs;
    int32_t myc = 0;
    float myv = 0.0f;
    if (tt < n) {
      const int32_t idx = e + tt * stride;
      myc = a.col[idx];
      myv = a.val ? a.val[idx] : 1.0f;
    }
    const int cnt = min(LF, n - t0);
    for (int j = 0; j < cnt; j += U) {
      int32_t c[U];
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int src = base + min(j + u, LF - 1);
        c[u] = __shfl(myc, src, 64);
        v[u] = __shfl(myv, src, 64);
      }
      float x[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j + u < cnt) load_vec<VEC>(hub + c[u] * W, x[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j + u < cnt) {
#pragma unroll
          for (int q = 0; q < VEC; ++q) acc[q] = fma((double)v[u], (double)x[u][q], acc[q]);
        }
      }
    }
  }
}

// entries e, e + stride, ... < e1, one loop for hub and tail alike (one round trip of index loads
// per LF entries, software-pipelined): every entry reads LDS row min(c, H) (row H is zeros) and
// issues a raw buffer load of T_{k-1} row c whose offset is dropped -- zero, no memory request --
// when c < H; one of the two terms is 0, so the sum is exact (step_dev.h accumulate_bcast_buf
// with nullable values)
template <int VEC, int U>
__device__ __forceinline__ void hub_range(const StepArgs& a, int32_t e, int32_t e1, int32_t stride, int32_t H,
                                          __amdgpu_buffer_rsrc_t rs, uint32_t xoff_b, const float* hub, int W,
                                          double (&acc)[VEC], int fs, int base) {
#ifdef WG_HUB_TWO_LOOPS  // timing variant: the hub prefix from LDS, then the tail with plain global loads
  int32_t hs = e;  // first entry with column >= H (rows column-sorted), by bisection
  {
    int32_t lo = e - (e - (e1 - 1)) % 1, hi = e1;
    lo = e;
    while (lo < hi) {
      const int32_t mid = lo + (hi - lo) / 2;
      if (a.col[mid] < H) lo = mid + 1; else hi = mid;
    }
    hs = lo;
  }
  const int32_t pe = hs;
  accumulate_bcast_lds<VEC, U>(a, e, pe, stride, hub, W, acc, fs, base);
  int32_t t = e;
  if (pe > t) t += (pe - t + stride - 1) / stride * stride;
  accumulate_bcast<VEC, U>(a, t, e1, stride, a.xm1 + fs * VEC, acc, fs, base);
  return;
#endif
  constexpr uint32_t kDrop = 0x80000000u;
  const int LF = a.LF;
  const uint32_t ldb = (uint32_t)a.ld * 4u;
  if (e >= e1) return;
  const int32_t n = (e1 - e + stride - 1) / stride;
  int32_t idx = e + min(fs, n - 1) * stride;
  int32_t myc = a.col[idx];
  float myv = a.val ? a.val[idx] : 1.0f;
  for (int32_t t0 = 0; t0 < n; t0 += LF) {
    const int32_t cc = myc;
    const float cv = myv;
    idx = e + min(t0 + LF + fs, n - 1) * stride;  // next LF pairs (clamped: always a valid entry)
    myc = a.col[idx];
    myv = a.val ? a.val[idx] : 1.0f;
    const int cnt = min(LF, n - t0);
    for (int j = 0; j < cnt; j += U) {
      int32_t c[U];
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int src = base + min(j + u, LF - 1);
        c[u] = __shfl(cc, src, 64);
        v[u] = __shfl(cv, src, 64);
      }
      float x[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool ok = j + u < cnt;
        const bool in_hub = c[u] < H;
        const uint32_t off = (ok && !in_hub) ? (uint32_t)c[u] * ldb + xoff_b : kDrop;
        const f32x4 g = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        const float* hp = hub + ((ok && in_hub) ? c[u] : H) * W;
        float y[VEC];
        load_vec<VEC>(hp, y);
#pragma unroll
        for (int q = 0; q < VEC; ++q) x[u][q] = g[q] + y[q];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double vv = (j + u < cnt) ? (double)v[u] : 0.0;
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = fma(vv, (double)x[u][q], acc[q]);
      }
    }
  }
}

template <int VEC>
__device__ __forceinline__ void hub_unit(const StepArgs& a, const HubArgs& h, const int4 un, int lane,
                                         __amdgpu_buffer_rsrc_t rs) {
  const int LF = a.LF;
  const int W = LF * VEC;
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;
  if (un.w < 0) {
    // ---- team pass: rows [un.x, un.x + un.y), LN = un.z sub-groups per row
    const int LN = un.z;
    const int TS = LF * LN;
    const int team = lane / TS;
    const int tl = lane - team * TS;
    const int ns = tl / LF;
    const int fs = tl - ns * LF;
    const int64_t row = (int64_t)un.x + team;
    const bool active = team < un.y && (team + 1) * TS <= 64;
    EpiIn<VEC> in;
    if (active) {
      const uint32_t xoff = (uint32_t)(fs * VEC * 4);
      if (ns == 0) epi_prefetch<VEC>(a, row, fs, in);
      const int32_t e0 = a.rowptr[row], e1 = a.rowptr[row + 1];
      if (LF % 5 == 0) hub_range<VEC, 5>(a, e0 + ns, e1, LN, h.H, rs, xoff, g_hubw_lds + fs * VEC, W, acc, fs, lane - fs);
      else hub_range<VEC, 4>(a, e0 + ns, e1, LN, h.H, rs, xoff, g_hubw_lds + fs * VEC, W, acc, fs, lane - fs);
    }
    reduce_subgroups<VEC>(acc, LN, LF, team * TS, fs);
    if (active && ns == 0) step_epilogue<VEC>(a, row, fs, acc, in, team * TS);
    return;
  }
  // ---- one chunk [un.y, un.z) of split row un.x: G sub-groups stride G, a float64 partial, the last
  // arriving chunk combines the row (write-through partials drained before the arrival; MI355X_MICROARCH.md
  // hand-off table row 1, as step.hip's split rows)
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int64_t row = un.x;
  if (sg < G) {
    const uint32_t xoff = (uint32_t)(fs * VEC * 4);
    if (LF % 5 == 0) hub_range<VEC, 5>(a, un.y + sg, un.z, G, h.H, rs, xoff, g_hubw_lds + fs * VEC, W, acc, fs, lane - fs);
    else hub_range<VEC, 4>(a, un.y + sg, un.z, G, h.H, rs, xoff, g_hubw_lds + fs * VEC, W, acc, fs, lane - fs);
  }
  reduce_subgroups<VEC>(acc, G, LF, 0, fs);
  if (lane < LF) {
    double* p = h.partial + (int64_t)un.w * W + fs * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) __hip_atomic_store(p + j, acc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int2 rc = h.rowchunks[row];
  int last = 0;
  if (lane == 0) {
    const int old = __hip_atomic_fetch_add(h.arrivals + row, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = ((old + 1) % rc.y) == 0;  // monotonic counter: every rc.y-th arrival completes a step
  }
  last = __shfl(last, 0, 64);
  if (last && lane < LF) {
    EpiIn<VEC> in;
    epi_prefetch<VEC>(a, row, fs, in);
    double sum[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) sum[j] = 0.0;
    for (int q = 0; q < rc.y; ++q) {
      const double* pp = h.partial + (int64_t)(rc.x + q) * W + fs * VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) sum[j] += __hip_atomic_load(pp + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    step_epilogue<VEC>(a, row, fs, sum, in, 0);
  }
}

template <int VEC>
__global__ __launch_bounds__(kHubThreads) void cheb_hubw_kernel(StepArgs a, HubArgs h) {
  const int W = a.LF * VEC;
  // ---- stage the hub: rows [0, H) of the gathered vector
  {
    const int per_row = W / VEC;
    for (int i = threadIdx.x; i < (h.H + 1) * per_row; i += kHubThreads) {  // row H: zeros
      const int r = i / per_row, c = i - r * per_row;
      float x[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) x[j] = 0.0f;
      if (r < h.H) load_vec<VEC>(a.xm1 + (int64_t)r * a.ld + c * VEC, x);
      float* d = g_hubw_lds + r * W + c * VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) d[j] = x[j];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // ---- per-wave work from this workgroup's queue (units q, q + 32, ...): the wave's first batch
  // is static (its index among the queue's waves), later ones come from the queue head, which
  // counts past the static batches -- no start-up burst of atomics, ~1-2 dequeues per wave
  const int q = blockIdx.x % kQueues;
  const int nwg_q = ((int)gridDim.x - q + kQueues - 1) / kQueues;  // workgroups on this queue
  const int nw_q = nwg_q * (kHubThreads / 64);                      // waves on this queue
  const int wq = (blockIdx.x / kQueues) * (kHubThreads / 64) + (threadIdx.x >> 6);
  const int cnt = (h.n_units - q + kQueues - 1) / kQueues;
  const int nb = (cnt + h.batch - 1) / h.batch;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.xm1), 0, (int)a.xm1_bytes, 0x00020000);
  for (int b = wq; b < nb;) {
    int nx = 0;  // the next batch's dequeue, issued before this batch (its latency overlaps the work)
    if (lane == 0) nx = __hip_atomic_fetch_add(h.ctr + q * kCtrStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int i1 = min(cnt, (b + 1) * h.batch);
    for (int i = b * h.batch; i < i1; ++i) hub_unit<VEC>(a, h, h.units[q + (int64_t)i * kQueues], lane, rs);
    b = nw_q + __shfl(nx, 0, 64);
  }
  // ---- the last workgroup out resets the queue heads for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t* done = h.ctr + kQueues * kCtrStride;
    const int old = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (int)gridDim.x - 1) {
      for (int k = 0; k < kQueues; ++k) __hip_atomic_store(h.ctr + k * kCtrStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <typename T>
int upload(T** d, const std::vector<T>& v) {
  if (int rc = dmalloc(d, v.size())) return rc;
  if (!v.empty()) WG_HIP_TRY(hipMemcpy(*d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return WG_OK;
}

int divisor_at_least_g(int G, int64_t want) {
  for (int d = 1; d <= G; ++d)
    if (G % d == 0 && d >= want) return d;
  return G;
}

int build_hub_plan(wg_laplacian_s* L, bool active_only, int LF, int W, HubPlan* p) {
  const int64_t n = active_only ? L->n_active : L->n_rows;
  const int G = 64 / LF;
  const int64_t lds_rows = (160 * 1024 - 256) / (W * 4) - 1;  // + one zero row
  const int64_t H = std::min<int64_t>(L->tune.hubw_rows > 0 ? L->tune.hubw_rows : lds_rows, std::min(lds_rows, L->n_cols));
  std::vector<int32_t> rp(n + 1);
  WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  const int64_t nnz = rp[n];
  std::vector<int32_t> col(std::max<int64_t>(nnz, 1));
  if (nnz) WG_HIP_TRY(hipMemcpy(col.data(), L->col, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
  std::vector<int32_t> hs(std::max<int64_t>(n, 1));
  int64_t hub_nnz = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int32_t* b = col.data() + rp[r];
    const int32_t* e = col.data() + rp[r + 1];
    hs[r] = (int32_t)(std::lower_bound(b, e, (int32_t)H) - col.data());
    hub_nnz += hs[r] - rp[r];
  }
  // team rows up to G * iter entries (LN = smallest divisor of G with LN * iter >= len), longer
  // rows in chunks of G * chunk_iter entries; units: chunks first, then team passes, by length
  const int iter = L->tune.hubw_iter > 0 ? L->tune.hubw_iter : 192;
  const int chunk_iter = L->tune.hubw_chunk > 0 ? L->tune.hubw_chunk : 64;
  const int64_t team_max = (int64_t)G * iter, CH = (int64_t)G * chunk_iter;
  std::vector<int4> units;
  std::vector<int2> rc;
  int32_t n_chunks = 0;
  int64_t r = 0;
  for (; r < n && rp[r + 1] - rp[r] > team_max; ++r) {
    const int64_t len = rp[r + 1] - rp[r];
    const int c = (int)((len + CH - 1) / CH);
    rc.push_back(int2{n_chunks, c});
    for (int q = 0; q < c; ++q)
      units.push_back(int4{(int)r, (int)(rp[r] + q * CH), (int)std::min<int64_t>(rp[r + 1], rp[r] + (q + 1) * CH),
                           n_chunks + q});
    n_chunks += c;
  }
  const int64_t n_split = r;
  while (r < n) {
    const int64_t len = std::max<int64_t>(1, rp[r + 1] - rp[r]);
    const int LN = divisor_at_least_g(G, (len + iter - 1) / iter);
    const int tpw = G / LN;
    int64_t k = 1;  // rows of this pass: same LN (lengths only decrease)
    while (k < tpw && r + k < n &&
           divisor_at_least_g(G, (std::max<int64_t>(1, rp[r + k + 1] - rp[r + k]) + iter - 1) / iter) == LN)
      ++k;
    units.push_back(int4{(int)r, (int)k, LN, -1});
    r += k;
  }
  p->H = (int32_t)H;
  p->n_units = (int32_t)units.size();
  p->n_chunks = n_chunks;
  p->width = W;
  p->lf = LF;
  {
    int n_cu = 256;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t waves = (int64_t)(L->tune.hubw_wg > 0 ? L->tune.hubw_wg : n_cu) * (kHubThreads / 64);
    p->batch = L->tune.hubw_batch > 0 ? L->tune.hubw_batch
                                      : (int)std::max<int64_t>(1, (int64_t)units.size() / (3 * waves));
  }
  std::vector<int2> rcf(std::max<int64_t>(n_split, 1));
  for (int64_t i = 0; i < n_split; ++i) rcf[i] = rc[i];
  int rc_ = upload(&p->units, units);
  if (!rc_) rc_ = upload(&p->hsplit, hs);
  if (!rc_) rc_ = upload(&p->rowchunks, rcf);
  if (!rc_) rc_ = dmalloc(&p->arrivals, std::max<int64_t>(n_split, 1));
  if (!rc_) rc_ = dmalloc(&p->partial, (size_t)std::max(n_chunks, 1) * W);
  if (!rc_) rc_ = dmalloc(&p->ctr, (size_t)(kQueues + 1) * kCtrStride);
  if (rc_) return rc_;
  WG_HIP_TRY(hipMemset(p->arrivals, 0, sizeof(int32_t) * std::max<int64_t>(n_split, 1)));
  WG_HIP_TRY(hipMemset(p->ctr, 0, sizeof(int32_t) * (kQueues + 1) * kCtrStride));
  char buf[256];
  snprintf(buf, sizeof(buf), "hubw: %lld hub rows in LDS (%.1f %% of the entries), %d units (%lld split rows in %d "
           "chunks of %lld, team passes up to %lld entries), batch %d\n", (long long)H,
           nnz ? 100.0 * hub_nnz / nnz : 0.0, p->n_units, (long long)n_split, n_chunks, (long long)CH,
           (long long)team_max, p->batch);
  p->text = buf;
  return WG_OK;
}

}  // namespace

void HubPlan::release() {
  for (void* q : {(void*)units, (void*)hsplit, (void*)rowchunks, (void*)arrivals, (void*)partial, (void*)ctr})
    (void)hipFree(q);
  *this = HubPlan{};
}

void release_hubw(wg_laplacian_s* L) {
  for (auto*& p : L->hubw) {
    if (p) {
      p->release();
      delete p;
      p = nullptr;
    }
  }
}

bool hubw_wanted(const wg_laplacian_s* L, int64_t F, int vec, int LF) {
  if (L->tune.hubw == 0 || vec != 4 || LF < 2 || LF * vec != F || !L->reordered || !L->cols_sorted) return false;
  if (L->tune.hubw == 1) return true;
  // auto: wide rows of a graph whose gathers dominate
  return F >= 16 && L->nnz >= ((int64_t)1 << 20);
}

int launch_hubw(wg_laplacian_s* L, const StepArgs& a, bool active_only, hipStream_t stream) {
  const int ai = active_only ? 1 : 0;
  const int W = a.LF * 4;
  if (L->hubw[ai] && (L->hubw[ai]->width != W || L->hubw[ai]->lf != a.LF)) {
    WG_HIP_TRY(hipStreamSynchronize(stream));
    L->hubw[ai]->release();
    delete L->hubw[ai];
    L->hubw[ai] = nullptr;
  }
  if (!L->hubw[ai]) {
    auto* p = new HubPlan();
    if (int rc = build_hub_plan(L, active_only, a.LF, W, p)) {
      p->release();
      delete p;
      return rc;
    }
    L->hubw[ai] = p;
  }
  HubPlan* p = L->hubw[ai];
  static int n_cu = 0;
  static bool attr_set = false;
  if (!n_cu) {
    int dev = 0;
    WG_HIP_TRY(hipGetDevice(&dev));
    WG_HIP_TRY(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (!attr_set) {
    WG_HIP_TRY(hipFuncSetAttribute((const void*)cheb_hubw_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024));
    attr_set = true;
  }
  HubArgs h{};
  h.units = p->units;
  h.n_units = p->n_units;
  h.batch = p->batch;
  h.ctr = p->ctr;
  h.hsplit = p->hsplit;
  h.H = p->H;
  h.rowchunks = p->rowchunks;
  h.arrivals = p->arrivals;
  h.partial = p->partial;
  // rowchunks / arrivals are indexed by internal row: the split rows are rows [0, n_split)
  const size_t lds = (size_t)(p->H + 1) * W * sizeof(float);
  if (a.xm1_bytes >= ((int64_t)1 << 31)) return fail(WG_ERR_UNSUPPORTED, "hubw: gathered vector over 2 GB");
  const int grid = L->tune.hubw_wg > 0 ? L->tune.hubw_wg : n_cu;  // any size: every queue has >= 1 workgroup
  if (grid < kQueues) return fail(WG_ERR_INVALID, "hubw: %d workgroups < %d queues", grid, kQueues);
  hipLaunchKernelGGL(cheb_hubw_kernel<4>, dim3(grid), dim3(kHubThreads), lds, stream, a, h);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

const char* hubw_text(const wg_laplacian_s* L) {
  for (int i = 1; i >= 0; --i)
    if (L->hubw[i]) return L->hubw[i]->text.c_str();
  return "";
}

}  // namespace wg
