// step.hip -- the Chebyshev step kernel (the hot loop of
// chebyshev_polynomials, reference calibration/WATS.py:32-36, with the heat
// sum of WATS.py:65-68 and optionally the row-L1 normalisation of :71-72 fused
// into the per-row epilogue), its launch plan, and the row-order kernels.
//
// Work decomposition (rows are relabelled by descending length, so rows of a
// bucket are contiguous):
//  * A "sub-group" is LF lanes that together cover the F signal columns of one
//    gathered row with VEC-wide loads (F = LF * VEC); a wave holds G = 64/LF
//    sub-groups.
//  * Team mode (short rows): LN sub-groups (LN a divisor of G) share one row
//    and split its nonzeros; G/LN rows per wave.  The LN partial sums meet in
//    a fixed shuffle order (tree for power-of-two LN).
//  * Chunk mode (long rows): a 256-lane workgroup = 4G sub-groups processes a
//    chunk of at most CH nonzeros of one row and reduces it through an LDS
//    tree.  A row with several chunks publishes each chunk's float64 partial;
//    the last workgroup to arrive (agent-scope atomic counter, release/acquire
//    per cdna_hip_programming.md Guideline 16) sums the partials in chunk
//    order -- deterministic regardless of arrival order -- and runs the
//    epilogue.  No workgroup ever waits on another.
// Row sums accumulate in float64 (products of two float32 are exact).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "internal.h"

namespace wg {
namespace {

struct StepArgs {
  const int32_t* rowptr;
  const int32_t* col;
  const float* val;
  const uint8_t* iso;
  const float* xm1;   // T_{k-1}: n_cols rows (owned + halo)
  const float* xm2;   // T_{k-2}: n_rows rows (k >= 2)
  float* xk;          // T_k (nullable)
  float* S;           // heat-kernel sum (nullable)
  float* H;           // normalised output (nullable; only when the tile covers all F)
  int64_t ld;         // row stride (floats) of every vector
  int32_t LF;         // lanes across the tile's columns (tile width = LF * VEC)
  int32_t k;          // step index (1 or >= 2)
  double alpha0;
  double alpha_k;
  const ChunkDesc* chunks;
  double* partial;
  unsigned int* arrive;
  int64_t seg_mask;
};

template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, float (&x)[VEC]) {
  if constexpr (VEC == 1) {
    x[0] = *p;
  } else if constexpr (VEC == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    x[0] = v.x; x[1] = v.y;
  } else {
    const float4 v = *reinterpret_cast<const float4*>(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* p, const double (&x)[VEC]) {
  if constexpr (VEC == 1) {
    *p = (float)x[0];
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2((float)x[0], (float)x[1]);
  } else {
    *reinterpret_cast<float4*>(p) = make_float4((float)x[0], (float)x[1], (float)x[2], (float)x[3]);
  }
}

// Per-row epilogue, run by the LF lanes holding the row's sums (`lane0` = wave
// lane of the row's first column slice, for the H shuffle).
template <int VEC>
__device__ __forceinline__ void step_epilogue(const StepArgs& a, int64_t row, int fs, double (&acc)[VEC],
                                              int lane0) {
  const int64_t off = row * a.ld + (int64_t)fs * VEC;
  float x[VEC];
  if (a.iso[row]) {  // L_hat_ii = -1 (scipy setdiag(1 - iso), then "- identity")
    load_vec<VEC>(a.xm1 + off, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] -= (double)x[j];
  }
  double t[VEC];
  if (a.k == 1) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = acc[j];
  } else {
    load_vec<VEC>(a.xm2 + off, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = 2.0 * acc[j] - (double)x[j];
  }
  if (a.xk) store_vec<VEC>(a.xk + off, t);
  if (a.S) {
    double s[VEC];
    if (a.k == 1) {  // S = alpha0*T_0 + alpha1*T_1, T_0 = own row of xm1
      load_vec<VEC>(a.xm1 + off, x);
#pragma unroll
      for (int j = 0; j < VEC; ++j) s[j] = a.alpha0 * (double)x[j] + a.alpha_k * t[j];
    } else {
      load_vec<VEC>(a.S + off, x);
#pragma unroll
      for (int j = 0; j < VEC; ++j) s[j] = (double)x[j] + a.alpha_k * t[j];
    }
    store_vec<VEC>(a.S + off, s);
    if (a.H) {
      double part = 0.0;
#pragma unroll
      for (int j = 0; j < VEC; ++j) part += fabs(s[j]);
      double tot = 0.0;
      for (int q = 0; q < a.LF; ++q) tot += __shfl(part, lane0 + q, 64);
      const double den = tot + 1e-8;
      double h[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) h[j] = s[j] / den;
      store_vec<VEC>(a.H + off, h);
    }
  }
}

// acc += sum over e = e, e+stride, ... < e1 of val[e] * x[col[e]] (float64).
template <int VEC>
__device__ __forceinline__ void accumulate(const StepArgs& a, int32_t e, int32_t e1, int32_t stride,
                                           const float* __restrict__ xb, double (&acc)[VEC]) {
  const int32_t* __restrict__ col = a.col;
  const float* __restrict__ val = a.val;
  const int64_t ld = a.ld;
  for (; e + 3 * stride < e1; e += 4 * stride) {
    int32_t c[4];
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = col[e + u * stride];
      v[u] = val[e + u * stride];
    }
    float x[4][VEC];
#pragma unroll
    for (int u = 0; u < 4; ++u) load_vec<VEC>(xb + (int64_t)c[u] * ld, x[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] = fma((double)v[u], (double)x[u][j], acc[j]);
  }
  for (; e < e1; e += stride) {
    const int32_t c = col[e];
    const float v = val[e];
    float x[VEC];
    load_vec<VEC>(xb + (int64_t)c * ld, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = fma((double)v, (double)x[j], acc[j]);
  }
}

template <int VEC>
__global__ __launch_bounds__(kBlock) void cheb_step_kernel(StepArgs a, SegTable tab) {
  __shared__ double red[kBlock * VEC];
  __shared__ int s_last;
  int si = 0;
  for (int i = 1; i < tab.n; ++i)
    if ((int32_t)blockIdx.x >= tab.s[i].blk_begin) si = i;
  const Seg seg = tab.s[si];
  if (!((a.seg_mask >> si) & 1)) return;  // timing attribution only
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int LF = a.LF;
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;

  if (seg.mode == 0) {
    // ---------------- team mode
    const int LN = seg.ln;
    const int TS = LF * LN;
    const int tpw = 64 / TS;
    const int team = lane / TS;
    const int tl = lane - team * TS;
    const int ns = tl / LF;
    const int fs = tl - ns * LF;
    const int64_t row = (int64_t)seg.begin + (int64_t)(blockIdx.x - seg.blk_begin) * (4 * tpw) + wave * tpw + team;
    const bool active = team < tpw && row < seg.end;
    if (active) {
      const int32_t e0 = a.rowptr[row], e1 = a.rowptr[row + 1];
      accumulate<VEC>(a, e0 + ns, e1, LN, a.xm1 + fs * VEC, acc);
    }
    if (LN > 1) {
      if ((LN & (LN - 1)) == 0) {
        for (int off = LN >> 1; off >= 1; off >>= 1) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] += __shfl_down(acc[j], off * LF, 64);
        }
      } else {
        double tot[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) tot[j] = acc[j];
        for (int q = 1; q < LN; ++q) {
          const int src = team * TS + q * LF + fs;
#pragma unroll
          for (int j = 0; j < VEC; ++j) tot[j] += __shfl(acc[j], src, 64);
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] = tot[j];
      }
    }
    if (active && ns == 0) step_epilogue<VEC>(a, row, fs, acc, team * TS);
    return;
  }

  // ---------------- chunk mode: one workgroup per chunk of a long row
  const int G = 64 / LF;
  const int NS = 4 * G;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int sub = wave * G + sg;
  const int cid = seg.begin + (int)(blockIdx.x - seg.blk_begin);
  const ChunkDesc d = a.chunks[cid];
  const int width = LF * VEC;
  if (sg < G) {
    accumulate<VEC>(a, d.e0 + sub, d.e1, NS, a.xm1 + fs * VEC, acc);
    const int base = (sub * LF + fs) * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) red[base + j] = acc[j];
  }
  __syncthreads();
  int p2 = 1;
  while (p2 < NS) p2 <<= 1;
  for (int s = p2 >> 1; s >= 1; s >>= 1) {
    for (int idx = threadIdx.x; idx < s * width; idx += kBlock) {
      if (idx / width + s < NS) red[idx] += red[idx + s * width];
    }
    __syncthreads();
  }
  if (d.count > 1) {
    // publish this chunk's partial, then count arrivals
    if (threadIdx.x < width) a.partial[(int64_t)cid * width + threadIdx.x] = red[threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned prev = __hip_atomic_fetch_add(a.arrive + d.first, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      const int last = (prev == (unsigned)(d.count - 1));
      if (last) {
        __hip_atomic_store(a.arrive + d.first, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x < width) {
      double sum = 0.0;
      for (int q = 0; q < d.count; ++q) sum += a.partial[(int64_t)(d.first + q) * width + threadIdx.x];
      red[threadIdx.x] = sum;
    }
    __syncthreads();
  }
  if (threadIdx.x < LF) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = red[threadIdx.x * VEC + j];
    step_epilogue<VEC>(a, d.row, threadIdx.x, acc, 0);
  }
}

// internal S -> caller-order S and H = S / (||S||_1 + 1e-8); team of LF lanes per row.
template <int VEC>
__global__ __launch_bounds__(kBlock) void finalize_kernel(int64_t n, int64_t F, int LF, const int32_t* __restrict__ perm,
                                                          const float* __restrict__ Sint, float* __restrict__ S,
                                                          float* __restrict__ H) {
  const int lane = threadIdx.x & 63;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + sg;
  const bool active = sg < G && row < n;
  float x[VEC];
  double part = 0.0;
  if (active) {
    load_vec<VEC>(Sint + row * F + fs * VEC, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) part += fabs((double)x[j]);
  }
  double tot = 0.0;
  for (int q = 0; q < LF; ++q) tot += __shfl(part, sg * LF + q, 64);
  if (!active) return;
  const int64_t r = perm ? perm[row] : row;
  double s[VEC], h[VEC];
  const double den = tot + 1e-8;
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    s[j] = (double)x[j];
    h[j] = s[j] / den;
  }
  if (S) store_vec<VEC>(S + r * F + fs * VEC, s);
  if (H) store_vec<VEC>(H + r * F + fs * VEC, h);
}

// wide-F fallback (F > 64*VEC): wave per row.
__global__ __launch_bounds__(kBlock) void finalize_wide_kernel(int64_t n, int64_t F, const int32_t* __restrict__ perm,
                                                               const float* __restrict__ Sint, float* __restrict__ S,
                                                               float* __restrict__ H) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const int64_t r = perm ? perm[row] : row;
  double part = 0.0;
  for (int64_t f = lane; f < F; f += 64) part += fabs((double)Sint[row * F + f]);
  for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off, 64);
  const double den = part + 1e-8;
  for (int64_t f = lane; f < F; f += 64) {
    const float s = Sint[row * F + f];
    if (S) S[r * F + f] = s;
    if (H) H[r * F + f] = (float)((double)s / den);
  }
}

template <int VEC>
__global__ __launch_bounds__(kBlock) void permute_kernel(int64_t n, int64_t F, int LF, const int32_t* __restrict__ perm,
                                                         int direction, const float* __restrict__ src,
                                                         float* __restrict__ dst) {
  const int lane = threadIdx.x & 63;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + sg;
  if (sg >= G || row >= n) return;
  const int64_t r = perm[row];
  const int64_t si = (direction == 0 ? r : row) * F + fs * VEC;
  const int64_t di = (direction == 0 ? row : r) * F + fs * VEC;
  float x[VEC];
  load_vec<VEC>(src + si, x);
  double y[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) y[j] = x[j];
  store_vec<VEC>(dst + di, y);
}

__global__ void permute_wide_kernel(int64_t n, int64_t F, const int32_t* __restrict__ perm, int direction,
                                    const float* __restrict__ src, float* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * F) return;
  const int64_t i = idx / F;
  const int64_t f = idx - i * F;
  const int64_t r = perm[i];
  if (direction == 0) dst[idx] = src[r * F + f];
  else dst[r * F + f] = src[idx];
}

__global__ __launch_bounds__(kBlock) void l1_normalize_kernel(int64_t n, int64_t F, const float* __restrict__ S,
                                                              float* __restrict__ H) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  double part = 0.0;
  for (int64_t f = lane; f < F; f += 64) part += fabs((double)S[row * F + f]);
  for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off, 64);
  const double den = part + 1e-8;
  for (int64_t f = lane; f < F; f += 64) H[row * F + f] = (float)((double)S[row * F + f] / den);
}

// smallest divisor of G that is >= want (G itself if none smaller)
int divisor_at_least(int G, int64_t want) {
  for (int d = 1; d <= G; ++d)
    if (G % d == 0 && d >= want) return d;
  return G;
}

template <int VEC>
int launch_step_vec(wg_laplacian_s* L, const StepArgs& a, const SegTable& tab, hipStream_t stream) {
  hipLaunchKernelGGL(cheb_step_kernel<VEC>, dim3(tab.total_blocks), dim3(kBlock), 0, stream, a, tab);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // namespace

void Plan::release() {
  (void)hipFree(chunks);
  (void)hipFree(partial);
  (void)hipFree(arrive);
  chunks = nullptr;
  partial = nullptr;
  arrive = nullptr;
}

int pick_vec(int64_t F, std::initializer_list<const void*> ptrs) {
  auto aligned = [&](uintptr_t al) {
    for (const void* p : ptrs)
      if (p && (reinterpret_cast<uintptr_t>(p) % al)) return false;
    return true;
  };
  if (F % 4 == 0 && aligned(16)) return 4;
  if (F % 2 == 0 && aligned(8)) return 2;
  return 1;
}

// Build (once per tile shape) the segment table and the chunk table.
int get_plan(wg_laplacian_s* L, int LF, int VEC, Plan** out) {
  const int key = LF * 8 + VEC;
  auto it = L->plans.find(key);
  if (it != L->plans.end()) {
    *out = &it->second;
    return WG_OK;
  }
  Plan p;
  p.width = LF * VEC;
  const int G = 64 / LF;
  const int64_t n = L->n_rows;
  const int iter = std::max(1, L->tune.iter);
  const int64_t team_max = (int64_t)G * iter;
  const int64_t CH = (int64_t)4 * G * std::max(1, L->tune.chunk_iter);
  SegTable& t = p.tab;
  char buf[256];
  if (!L->reordered) {
    // caller order: a single team segment sized by the average row length
    const int ln = divisor_at_least(G, ceil_div(std::max<int64_t>(1, L->avg_len), iter));
    const int tpw = G / ln;
    t.s[0] = Seg{0, (int32_t)n, 0, ln, 0};
    t.n = n > 0 ? 1 : 0;
    t.total_blocks = (int32_t)ceil_div(n, 4 * tpw);
    snprintf(buf, sizeof(buf), "team rows[0,%lld) ln=%d (no reorder)\n", (long long)n, ln);
    p.text = buf;
  } else {
    // rows are sorted by descending length: highest bucket first
    int64_t n_chunk_rows = 0;
    for (int b = kBuckets - 1; b >= 0; --b) {
      const int64_t maxlen = (b == 0) ? 1 : (1ll << b);
      if (maxlen > team_max) n_chunk_rows += L->bucket[b];
    }
    int nseg = 0;
    int32_t blk = 0;
    if (n_chunk_rows > 0) {
      std::vector<int32_t> rp(n_chunk_rows + 1);
      WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr, sizeof(int32_t) * (n_chunk_rows + 1), hipMemcpyDeviceToHost));
      std::vector<ChunkDesc> ch;
      for (int64_t r = 0; r < n_chunk_rows; ++r) {
        const int64_t len = rp[r + 1] - rp[r];
        const int cnt = (int)std::max<int64_t>(1, ceil_div(len, CH));
        const int first = (int)ch.size();
        for (int q = 0; q < cnt; ++q) {
          ChunkDesc d{};
          d.row = (int32_t)r;
          d.e0 = (int32_t)(rp[r] + q * CH);
          d.e1 = (int32_t)std::min<int64_t>(rp[r + 1], rp[r] + (q + 1) * CH);
          d.first = first;
          d.count = cnt;
          ch.push_back(d);
        }
      }
      p.n_chunks = (int32_t)ch.size();
      int rc = dmalloc(&p.chunks, ch.size());
      if (!rc) rc = dmalloc(&p.partial, ch.size() * (size_t)p.width);
      if (!rc) rc = dmalloc(&p.arrive, ch.size());
      if (rc) {
        p.release();
        return rc;
      }
      WG_HIP_TRY(hipMemcpy(p.chunks, ch.data(), sizeof(ChunkDesc) * ch.size(), hipMemcpyHostToDevice));
      WG_HIP_TRY(hipMemset(p.arrive, 0, sizeof(unsigned int) * ch.size()));
      t.s[nseg++] = Seg{0, p.n_chunks, 0, 4 * G, 1};
      blk = p.n_chunks;
      snprintf(buf, sizeof(buf), "chunk rows[0,%lld) chunks=%d CH=%lld\n", (long long)n_chunk_rows, p.n_chunks,
               (long long)CH);
      p.text += buf;
    }
    int32_t row = (int32_t)n_chunk_rows;
    for (int b = kBuckets - 1; b >= 0; --b) {
      const int32_t cnt = (int32_t)L->bucket[b];
      const int64_t maxlen = (b == 0) ? 1 : (1ll << b);
      if (!cnt || maxlen > team_max) continue;
      int ln = divisor_at_least(G, ceil_div(maxlen, iter));
      Seg* last = nseg ? &t.s[nseg - 1] : nullptr;
      if (last && last->mode == 0 && (last->ln == ln || nseg == kMaxSeg)) {
        if (last->ln != ln) ln = last->ln;  // out of slots: extend
        last->end = row + cnt;
        blk = last->blk_begin + (int32_t)ceil_div(last->end - last->begin, 4 * (G / ln));
      } else {
        t.s[nseg++] = Seg{row, row + cnt, blk, ln, 0};
        blk += (int32_t)ceil_div(cnt, 4 * (G / ln));
      }
      row += cnt;
    }
    t.n = nseg;
    t.total_blocks = blk;
    for (int i = 0; i < nseg; ++i) {
      if (t.s[i].mode != 0) continue;
      snprintf(buf, sizeof(buf), "team rows[%d,%d) ln=%d blocks=%d\n", t.s[i].begin, t.s[i].end, t.s[i].ln,
               (i + 1 < nseg ? t.s[i + 1].blk_begin : blk) - t.s[i].blk_begin);
      p.text += buf;
    }
  }
  auto res = L->plans.emplace(key, p);
  *out = &res.first->second;
  return WG_OK;
}

int launch_step(wg_laplacian_s* L, int32_t k, int64_t F, const float* xm1, const float* xm2, float* xk, float* S,
                float* H, double alpha0, double alpha_k, hipStream_t stream) {
  if (L->n_rows == 0) return WG_OK;
  const int vec = pick_vec(F, {xm1, xm2, xk, S, H});
  const int64_t max_tile = 64 * (int64_t)vec;  // LF <= 64
  const bool fuse_h = (H != nullptr) && F <= max_tile;
  for (int64_t f0 = 0; f0 < F; f0 += max_tile) {
    const int64_t fw = std::min<int64_t>(max_tile, F - f0);
    const int LF = (int)(fw / vec);
    Plan* plan = nullptr;
    int rc = get_plan(L, LF, vec, &plan);
    if (rc) return rc;
    if (plan->tab.total_blocks == 0) continue;
    StepArgs a{};
    a.rowptr = L->rowptr;
    a.col = L->col;
    a.val = L->val;
    a.iso = L->iso;
    a.xm1 = xm1 + f0;
    a.xm2 = xm2 ? xm2 + f0 : nullptr;
    a.xk = xk ? xk + f0 : nullptr;
    a.S = S ? S + f0 : nullptr;
    a.H = fuse_h ? H + f0 : nullptr;
    a.ld = F;
    a.LF = LF;
    a.k = k;
    a.alpha0 = alpha0;
    a.alpha_k = alpha_k;
    a.chunks = plan->chunks;
    a.partial = plan->partial;
    a.arrive = plan->arrive;
    a.seg_mask = L->tune.seg_mask;
    if (vec == 4) rc = launch_step_vec<4>(L, a, plan->tab, stream);
    else if (vec == 2) rc = launch_step_vec<2>(L, a, plan->tab, stream);
    else rc = launch_step_vec<1>(L, a, plan->tab, stream);
    if (rc) return rc;
  }
  if (H && !fuse_h) {
    hipLaunchKernelGGL(l1_normalize_kernel, dim3(ceil_div(L->n_rows, 4)), dim3(kBlock), 0, stream, L->n_rows, F, S, H);
    WG_LAUNCH_CHECK();
  }
  return WG_OK;
}

int launch_finalize(wg_laplacian_s* L, int64_t F, const float* Sint, float* S, float* H, hipStream_t stream) {
  const int64_t n = L->n_rows;
  if (n == 0) return WG_OK;
  const int vec = pick_vec(F, {Sint, S, H});
  if (F <= 64 * vec) {
    const int LF = (int)(F / vec);
    const int G = 64 / LF;
    const dim3 grid((unsigned)ceil_div(n, 4 * G));
    if (vec == 4) hipLaunchKernelGGL(finalize_kernel<4>, grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, Sint, S, H);
    else if (vec == 2) hipLaunchKernelGGL(finalize_kernel<2>, grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, Sint, S, H);
    else hipLaunchKernelGGL(finalize_kernel<1>, grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, Sint, S, H);
  } else {
    hipLaunchKernelGGL(finalize_wide_kernel, dim3(ceil_div(n, 4)), dim3(kBlock), 0, stream, n, F, L->perm, Sint, S, H);
  }
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int launch_permute(wg_laplacian_s* L, int direction, int64_t F, const float* src, float* dst, hipStream_t stream) {
  const int64_t n = L->n_rows;
  if (n == 0) return WG_OK;
  const int vec = pick_vec(F, {src, dst});
  if (F <= 64 * vec) {
    const int LF = (int)(F / vec);
    const int G = 64 / LF;
    const dim3 grid((unsigned)ceil_div(n, 4 * G));
    if (vec == 4) hipLaunchKernelGGL(permute_kernel<4>, grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, direction, src, dst);
    else if (vec == 2) hipLaunchKernelGGL(permute_kernel<2>, grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, direction, src, dst);
    else hipLaunchKernelGGL(permute_kernel<1>, grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, direction, src, dst);
  } else {
    hipLaunchKernelGGL(permute_wide_kernel, dim3(ceil_div(n * F, 256)), dim3(256), 0, stream, n, F, L->perm, direction,
                       src, dst);
  }
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int launch_l1_normalize(const float* S, float* H, int64_t n, int64_t F, hipStream_t stream) {
  hipLaunchKernelGGL(l1_normalize_kernel, dim3(ceil_div(n, 4)), dim3(kBlock), 0, stream, n, F, S, H);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // namespace wg
