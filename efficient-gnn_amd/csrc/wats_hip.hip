// wats_hip.hip -- MI355X (gfx950 / CDNA4) kernels + C ABI for the WATS
// graph-wavelet feature extractor (reference: calibration/WATS.py:24-74 of
// CaptainCuong/Efficient-GNN, arithmetic of scipy.sparse csgraph.laplacian +
// CSR @ dense).  C ABI declared in include/wats_hip.h.
//
// Design (DESIGN.md has the full rationale):
//  * The normalised, rescaled Laplacian L_hat is materialised once per graph
//    ("prologue") as an int32 CSR with float32 values computed in scipy's exact
//    op order  -((a_ij / sqrt(w_i)) / sqrt(w_j))  -- bit-identical to scipy.
//    Self loops are dropped (scipy overwrites the diagonal); isolated rows
//    (w_i == 0) carry L_hat_ii = -1 as a per-row flag instead of a stored entry.
//  * Rows are relabelled by descending degree (a symmetric permutation
//    P L_hat P^T).  Hubs get the lowest ids, so the gathered rows that most
//    edges reference sit in a compact, L2-resident prefix of the vector, and
//    rows of similar length are contiguous, which lets the step kernel bin
//    them into segments with a per-segment lane-team width (no divergence
//    waste, hub rows first in dispatch order).  Each row keeps its original
//    column order, so per-row accumulation order does not depend on the
//    relabelling.
//  * One launch per Chebyshev step.  Each row is processed by a "team" of
//    LF x LN lanes: LF lanes cover the F signal columns with VEC-wide vector
//    loads, LN lanes split the row's nonzeros.  Row sums accumulate in
//    float64 (exact products of two float32s) and the LN partial sums meet in
//    a fixed __shfl_down tree -> deterministic, and accurate on hub rows
//    (sequential fp32 sums fail 1e-5 there).
//    Rows longer than the team limit get a whole 256-lane workgroup with an
//    LDS tree.  The recurrence, the heat-kernel accumulation S += alpha_k T_k
//    and (on the last step) the row-L1 normalisation are fused into the
//    per-row epilogue, so each step streams T_{k-1} (gathered), T_{k-2}, T_k
//    and S exactly once.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "wats_hip.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(e_ == hipErrorOutOfMemory ? WG_ERR_OOM : WG_ERR_HIP, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(e_), __FILE__, __LINE__);                    \
  } while (0)

#define LAUNCH_CHECK() HIP_TRY(hipGetLastError())

constexpr int kBlock = 256;     // 4 waves of 64
constexpr int kMaxSeg = 24;
constexpr int kBuckets = 33;    // row-length buckets: b=0: len<=1, b: 2^(b-1) < len <= 2^b

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// Segment table for the step kernel (by value in the kernel arguments).
// ---------------------------------------------------------------------------
struct Seg {
  int32_t row_begin;   // internal row range [row_begin, row_end)
  int32_t row_end;
  int32_t blk_begin;   // first workgroup of this segment
  int32_t ln;          // lanes splitting a row's nonzeros (team mode)
  int32_t block_mode;  // 1: one 256-lane workgroup per row
};
struct SegTable {
  Seg s[kMaxSeg];
  int32_t n;
  int32_t total_blocks;
};

struct StepArgs {
  const int32_t* rowptr;
  const int32_t* col;
  const float* val;
  const uint8_t* iso;
  const float* xm1;   // T_{k-1}: n_cols rows
  const float* xm2;   // T_{k-2}: n_rows rows (k >= 2)
  float* xk;          // T_k (nullable)
  float* S;           // heat-kernel sum (nullable)
  float* H;           // normalised output (nullable; needs S and all F in one tile)
  int64_t ld;         // row stride (floats) of every vector
  int32_t LF;         // lanes across the F columns of this tile (F = LF * VEC)
  int32_t k;          // step index (1 or >= 2)
  double alpha0;
  double alpha_k;
};

template <int VEC> struct VecT;
template <> struct VecT<1> { using T = float; };
template <> struct VecT<2> { using T = float2; };
template <> struct VecT<4> { using T = float4; };

template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, float (&x)[VEC]) {
  if constexpr (VEC == 1) {
    x[0] = *p;
  } else if constexpr (VEC == 2) {
    float2 v = *reinterpret_cast<const float2*>(p);
    x[0] = v.x; x[1] = v.y;
  } else {
    float4 v = *reinterpret_cast<const float4*>(p);
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

// Per-row epilogue: diagonal (isolated rows), recurrence, heat-kernel sum,
// optional row-L1 normalisation.  Called by the LF lanes holding the row's sums;
// `lane0` is the wave lane of the row's first F-slice (for the H shuffle).
template <int VEC>
__device__ __forceinline__ void step_epilogue(const StepArgs& a, int64_t row, int fs,
                                              double (&acc)[VEC], int lane0) {
  const int64_t off = row * a.ld + (int64_t)fs * VEC;
  float x[VEC];
  if (a.iso[row]) {  // L_hat_ii = -1  (scipy setdiag(1 - iso) then "- identity")
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
    if (a.k == 1) {  // S = alpha0*T_0 + alpha1*T_1 ; T_0 = own row of xm1
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

// One Chebyshev step over every row of L_hat.  Grid = segment blocks.
template <int VEC>
__global__ __launch_bounds__(kBlock) void cheb_step_kernel(StepArgs a, SegTable tab) {
  __shared__ double red[kBlock * VEC];
  int si = 0;
  for (int i = 1; i < tab.n; ++i)
    if ((int32_t)blockIdx.x >= tab.s[i].blk_begin) si = i;
  const Seg seg = tab.s[si];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int LF = a.LF;
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;

  if (!seg.block_mode) {
    const int LN = seg.ln;
    const int TS = LF * LN;
    const int tpw = 64 / TS;
    const int team = lane / TS;
    const int tl = lane - team * TS;
    const int fs = tl % LF;
    const int ns = tl / LF;
    const int64_t row = (int64_t)seg.row_begin +
                        (int64_t)(blockIdx.x - seg.blk_begin) * (4 * tpw) + wave * tpw + team;
    const bool active = team < tpw && row < seg.row_end;
    if (active) {
      const int32_t e0 = a.rowptr[row], e1 = a.rowptr[row + 1];
      accumulate<VEC>(a, e0 + ns, e1, LN, a.xm1 + fs * VEC, acc);
    }
    for (int off = LN >> 1; off >= 1; off >>= 1) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += __shfl_down(acc[j], off * LF, 64);
    }
    if (active && ns == 0) step_epilogue<VEC>(a, row, fs, acc, team * TS);
  } else {
    // one workgroup per (long) row: spw sub-teams of LF lanes per wave
    const int spw = 64 / LF;
    const int ns_total = 4 * spw;
    const int sub_in_wave = lane / LF;
    const int fs = lane - sub_in_wave * LF;
    const int sub = wave * spw + sub_in_wave;
    const int64_t row = (int64_t)seg.row_begin + (blockIdx.x - seg.blk_begin);
    const bool live = sub_in_wave < spw;
    if (live) {
      const int32_t e0 = a.rowptr[row], e1 = a.rowptr[row + 1];
      accumulate<VEC>(a, e0 + sub, e1, ns_total, a.xm1 + fs * VEC, acc);
      const int base = (sub * LF + fs) * VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) red[base + j] = acc[j];
    }
    __syncthreads();
    int p2 = 1;
    while (p2 < ns_total) p2 <<= 1;
    const int width = LF * VEC;
    for (int s = p2 >> 1; s >= 1; s >>= 1) {
      for (int idx = threadIdx.x; idx < s * width; idx += kBlock) {
        const int sidx = idx / width;
        if (sidx + s < ns_total) red[idx] += red[idx + s * width];
      }
      __syncthreads();
    }
    if (threadIdx.x < LF) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] = red[threadIdx.x * VEC + j];
      step_epilogue<VEC>(a, row, threadIdx.x, acc, 0);
    }
  }
}

// ---------------------------------------------------------------------------
// Prologue kernels
// ---------------------------------------------------------------------------

// Wave per row: off-diagonal count, row sum incl. diagonal (float64), diagonal
// value, optional column sums (float64 atomics).
__global__ __launch_bounds__(kBlock) void row_info_kernel(
    int64_t n_rows, const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, int32_t* __restrict__ offdiag_len, double* __restrict__ rowsum,
    float* __restrict__ diag, double* __restrict__ colsum) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int64_t e0 = indptr[row], e1 = indptr[row + 1];
  int cnt = 0;
  double rs = 0.0;
  float dg = 0.0f;
  for (int64_t e = e0 + lane; e < e1; e += 64) {
    const int32_t c = indices[e];
    const float v = values ? values[e] : 1.0f;
    rs += (double)v;
    if (c == row) dg += v; else ++cnt;
    if (colsum) atomicAdd(colsum + c, (double)v);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    cnt += __shfl_down(cnt, off, 64);
    rs += __shfl_down(rs, off, 64);
    dg += __shfl_down(dg, off, 64);
  }
  if (lane == 0) {
    offdiag_len[row] = cnt;
    rowsum[row] = rs;
    diag[row] = dg;
  }
}

// w_j = float32(colsum_j) - diag_j  (scipy: float32 sum minus float32 diagonal),
// sw_j = w_j == 0 ? 1 : sqrt(w_j), iso_j = (w_j == 0).
__global__ void degree_kernel(int64_t n_cols, int64_t n_rows, const double* __restrict__ colsum,
                              const float* __restrict__ diag, const float* __restrict__ w_cols,
                              float* __restrict__ sw, uint8_t* __restrict__ iso_col) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_cols) return;
  float w;
  if (w_cols) {
    w = w_cols[j];
  } else {
    w = (float)colsum[j] - (j < n_rows ? diag[j] : 0.0f);
  }
  const bool iso = (w == 0.0f);
  sw[j] = iso ? 1.0f : sqrtf(w);
  iso_col[j] = iso ? 1 : 0;
}

__global__ void f64_to_f32_kernel(int64_t n, const double* __restrict__ in, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (float)in[i];
}

__global__ void iota_kernel(int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)i;
}

__global__ void invert_perm_kernel(int64_t n, const int32_t* __restrict__ perm,
                                   int32_t* __restrict__ iperm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) iperm[perm[i]] = (int32_t)i;
}

__global__ void gather_len_kernel(int64_t n, const int32_t* __restrict__ perm,
                                  const int32_t* __restrict__ len, int32_t* __restrict__ out,
                                  const uint8_t* __restrict__ iso_col, uint8_t* __restrict__ iso_row) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int32_t r = perm[i];
    out[i] = len[r];
    iso_row[i] = iso_col[r];
  }
}

// Wave per internal row: copy the original row's off-diagonal entries (column
// order preserved), relabel columns, compute the scipy-exact L_hat value.
__global__ __launch_bounds__(kBlock) void fill_lhat_kernel(
    int64_t n_rows, const int32_t* __restrict__ perm, const int32_t* __restrict__ iperm,
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, const float* __restrict__ sw,
    const int32_t* __restrict__ rowptr, int32_t* __restrict__ col, float* __restrict__ val) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n_rows) return;
  const int32_t r = perm[i];
  const float swr = sw[r];
  const int64_t e0 = indptr[r], e1 = indptr[r + 1];
  int32_t pos = rowptr[i];
  for (int64_t base = e0; base < e1; base += 64) {
    const int64_t e = base + lane;
    int32_t c = 0;
    bool keep = false;
    if (e < e1) {
      c = indices[e];
      keep = (c != r);
    }
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (keep) {
      const float a = values ? values[e] : 1.0f;
      // scipy _laplacian.py:472-474: data /= w[row]; data /= w[col]; data *= -1
      const float v = -((a / swr) / sw[c]);
      col[pos + before] = (c < n_rows) ? iperm[c] : c;
      val[pos + before] = v;
    }
    pos += __popcll(m);
  }
}

__global__ void bucket_hist_kernel(int64_t n, const int32_t* __restrict__ len,
                                   unsigned int* __restrict__ hist) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t l = len[i];
  int b = 0;
  if (l > 1) b = 32 - __clz(l - 1);  // ceil(log2(l))
  atomicAdd(hist + b, 1u);
}

// X0 = log1p(rowsum) (calibration/WATS.py:58-59); float32 row sum, then a
// correctly rounded log1p.
__global__ void log1p_degree_kernel(int64_t n, const float* __restrict__ rowsum, float* __restrict__ x0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x0[i] = (float)log1p((double)rowsum[i]);
}

__global__ void permute_rows_kernel(int64_t n, int64_t F, const int32_t* __restrict__ perm, int direction,
                                    const float* __restrict__ src, float* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * F) return;
  const int64_t i = idx / F;
  const int64_t f = idx - i * F;
  const int64_t r = perm[i];
  if (direction == 0) dst[idx] = src[r * F + f];
  else dst[r * F + f] = src[idx];
}

// Final pass of graph_wavelet_features: internal S -> caller-order S and H.
// Team of LF lanes per row (VEC=1 scalar columns), fixed-order L1 sum.
__global__ __launch_bounds__(kBlock) void finalize_kernel(int64_t n, int64_t F, const int32_t* __restrict__ perm,
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

__global__ void gather_rows_kernel(int64_t n, int64_t F, const int32_t* __restrict__ rows,
                                   const float* __restrict__ src, float* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * F) return;
  const int64_t i = idx / F;
  const int64_t f = idx - i * F;
  dst[idx] = src[(int64_t)rows[i] * F + f];
}

// Dense ingestion: wave per row.
__global__ __launch_bounds__(kBlock) void dense_count_kernel(int64_t n_rows, int64_t n_cols, int64_t ld,
                                                             const float* __restrict__ adj,
                                                             int64_t* __restrict__ counts) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const float* p = adj + row * ld;
  int64_t cnt = 0;
  for (int64_t c = lane; c < n_cols; c += 64) cnt += (p[c] != 0.0f);
  for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_down(cnt, off, 64);
  if (lane == 0) counts[row] = cnt;
}

__global__ __launch_bounds__(kBlock) void dense_fill_kernel(int64_t n_rows, int64_t n_cols, int64_t ld,
                                                            const float* __restrict__ adj,
                                                            const int64_t* __restrict__ indptr,
                                                            int32_t* __restrict__ indices,
                                                            float* __restrict__ values) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const float* p = adj + row * ld;
  int64_t pos = indptr[row];
  for (int64_t base = 0; base < n_cols; base += 64) {
    const int64_t c = base + lane;
    const float v = (c < n_cols) ? p[c] : 0.0f;
    const bool nz = (v != 0.0f);
    const unsigned long long m = __ballot(nz);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (nz) {
      indices[pos + before] = (int32_t)c;
      values[pos + before] = v;
    }
    pos += __popcll(m);
  }
}

__global__ __launch_bounds__(kBlock) void column_degree_kernel(int64_t n_rows, int64_t row_offset,
                                                               const int64_t* __restrict__ indptr,
                                                               const int32_t* __restrict__ indices,
                                                               const float* __restrict__ values,
                                                               double* __restrict__ colsum,
                                                               double* __restrict__ diag) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int64_t grow = row + row_offset;
  for (int64_t e = indptr[row] + lane; e < indptr[row + 1]; e += 64) {
    const int32_t c = indices[e];
    const double v = values ? (double)values[e] : 1.0;
    atomicAdd(colsum + c, v);
    if (c == grow) atomicAdd(diag + grow, v);
  }
}

// Export L_hat in caller numbering (off-diagonal entries, original column order).
__global__ void export_len_kernel(int64_t n, const int32_t* __restrict__ iperm, const int32_t* __restrict__ rowptr,
                                  int64_t* __restrict__ lens) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t i = iperm[r];
  lens[r] = rowptr[i + 1] - rowptr[i];
}

__global__ void export_fill_kernel(int64_t n_rows, const int32_t* __restrict__ perm, const int32_t* __restrict__ iperm,
                                   const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                   const float* __restrict__ val, const int64_t* __restrict__ out_ptr,
                                   int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int32_t i = iperm[r];
  int64_t o = out_ptr[r];
  for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e, ++o) {
    const int32_t c = col[e];
    out_idx[o] = (c < n_rows) ? perm[c] : c;
    out_val[o] = val[e];
  }
}

__global__ void export_iso_kernel(int64_t n, const int32_t* __restrict__ iperm, const uint8_t* __restrict__ iso,
                                  uint8_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n) out[r] = iso[iperm[r]];
}

template <typename T>
int dmalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return WG_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// Handle
// ---------------------------------------------------------------------------
struct wg_laplacian_s {
  int device = 0;
  int64_t n_rows = 0, n_cols = 0, nnz_input = 0, nnz = 0, n_iso = 0, max_row = 0;
  bool reordered = true;
  int32_t* rowptr = nullptr;  // internal order, int32
  int32_t* col = nullptr;
  float* val = nullptr;
  uint8_t* iso = nullptr;     // internal order
  int32_t* perm = nullptr;    // internal -> caller row
  int32_t* iperm = nullptr;   // caller -> internal row
  float* rowsum = nullptr;    // caller order, float32 (for X0)
  unsigned int bucket[kBuckets] = {0};  // rows per length bucket (internal rows sorted descending)
  int64_t avg_len = 0;
  // workspace for wg_wavelet_features
  float* ws = nullptr;
  size_t ws_floats = 0;
  // live step-kernel timing (wg_profile_*)
  bool prof = false;
  std::vector<hipEvent_t> ev;  // pool, pairs (start, stop)
  size_t ev_used = 0;

  ~wg_laplacian_s() {
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    for (void* p : {(void*)rowptr, (void*)col, (void*)val, (void*)iso, (void*)perm, (void*)iperm,
                    (void*)rowsum, (void*)ws})
      (void)hipFree(p);
  }
};

namespace {

// Build the step kernel's segment table for a tile of F = LF * VEC columns.
SegTable build_segments(const wg_laplacian_s* L, int LF) {
  SegTable t{};
  int ln_max = 1;
  while (ln_max * 2 * LF <= 64) ln_max *= 2;
  const int64_t n = L->n_rows;
  if (!L->reordered) {
    // caller order: one team segment, LN from the average row length
    int ln = 1;
    while (ln < ln_max && ln * 2 <= std::max<int64_t>(1, L->avg_len / 2)) ln *= 2;
    const int tpw = 64 / (LF * ln);
    t.s[0] = Seg{0, (int32_t)n, 0, ln, 0};
    t.n = 1;
    t.total_blocks = (int32_t)ceil_div(n, 4 * tpw);
    return t;
  }
  // rows are sorted by descending length: bucket kBuckets-1 first.
  const int64_t long_len = (int64_t)ln_max * 16;   // > this: workgroup per row
  int32_t row = 0;
  int32_t blk = 0;
  int nseg = 0;
  auto push = [&](int32_t r0, int32_t r1, int ln, int block_mode) {
    if (r1 <= r0) return;
    int64_t nb = block_mode ? (r1 - r0) : ceil_div(r1 - r0, 4 * (64 / (LF * ln)));
    if (nseg > 0 && t.s[nseg - 1].ln == ln && t.s[nseg - 1].block_mode == block_mode &&
        t.s[nseg - 1].row_end == r0) {
      // merge: recompute blocks of the merged segment
      Seg& s = t.s[nseg - 1];
      s.row_end = r1;
      int64_t nb2 = block_mode ? (s.row_end - s.row_begin)
                               : ceil_div(s.row_end - s.row_begin, 4 * (64 / (LF * ln)));
      blk = s.blk_begin + (int32_t)nb2;
      return;
    }
    t.s[nseg] = Seg{r0, r1, blk, ln, block_mode};
    blk += (int32_t)nb;
    ++nseg;
  };
  for (int b = kBuckets - 1; b >= 0; --b) {
    const int32_t cnt = (int32_t)L->bucket[b];
    if (!cnt) continue;
    const int64_t maxlen = (b == 0) ? 1 : (1ll << b);
    int ln;
    int block_mode = 0;
    if (maxlen > long_len) {
      block_mode = 1;
      ln = ln_max;
    } else {
      // ~4 nonzeros per lane for long rows, one team lane per nonzero below that
      int64_t want = std::max<int64_t>(1, maxlen / 4);
      ln = 1;
      while (ln < ln_max && ln < want) ln *= 2;
      if (maxlen <= 4) ln = std::min<int>(ln_max, (int)std::max<int64_t>(1, maxlen));
    }
    if (nseg == kMaxSeg - 1 && !(t.s[nseg - 1].ln == ln && t.s[nseg - 1].block_mode == block_mode)) {
      // out of segment slots: extend the last segment (correct, slightly slower)
      ln = t.s[nseg - 1].ln;
      block_mode = t.s[nseg - 1].block_mode;
    }
    push(row, row + cnt, ln, block_mode);
    row += cnt;
  }
  t.n = nseg;
  t.total_blocks = blk;
  return t;
}

int pick_vec(int64_t F, std::initializer_list<const void*> ptrs) {
  auto aligned = [&](uintptr_t a) {
    for (const void* p : ptrs)
      if (p && (reinterpret_cast<uintptr_t>(p) % a)) return false;
    return true;
  };
  if (F % 4 == 0 && aligned(16)) return 4;
  if (F % 2 == 0 && aligned(8)) return 2;
  return 1;
}

int launch_step(const wg_laplacian_s* L, int32_t k, int64_t F, const float* xm1, const float* xm2, float* xk,
                float* S, float* H, double alpha0, double alpha_k, hipStream_t stream) {
  if (L->n_rows == 0) return WG_OK;
  const int vec = pick_vec(F, {xm1, xm2, xk, S, H});
  const int64_t max_tile = 64 * (int64_t)vec;  // LF <= 64
  const bool fuse_h = (H != nullptr) && F <= max_tile;
  for (int64_t f0 = 0; f0 < F; f0 += max_tile) {
    const int64_t fw = std::min<int64_t>(max_tile, F - f0);
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
    a.LF = (int32_t)(fw / vec);
    a.k = k;
    a.alpha0 = alpha0;
    a.alpha_k = alpha_k;
    const SegTable tab = build_segments(L, a.LF);
    if (tab.total_blocks == 0) continue;
    dim3 grid(tab.total_blocks), block(kBlock);
    if (vec == 4) hipLaunchKernelGGL(cheb_step_kernel<4>, grid, block, 0, stream, a, tab);
    else if (vec == 2) hipLaunchKernelGGL(cheb_step_kernel<2>, grid, block, 0, stream, a, tab);
    else hipLaunchKernelGGL(cheb_step_kernel<1>, grid, block, 0, stream, a, tab);
    LAUNCH_CHECK();
  }
  if (H && !fuse_h) {
    hipLaunchKernelGGL(l1_normalize_kernel, dim3(ceil_div(L->n_rows, 4)), dim3(kBlock), 0, stream, L->n_rows, F,
                       S, H);
    LAUNCH_CHECK();
  }
  return WG_OK;
}

template <typename F_>
int cub_call(hipStream_t stream, F_&& fn) {
  size_t bytes = 0;
  HIP_TRY(fn(nullptr, bytes));
  void* tmp = nullptr;
  HIP_TRY(hipMalloc(&tmp, std::max<size_t>(bytes, 1)));
  hipError_t e = fn(tmp, bytes);
  hipError_t e2 = hipStreamSynchronize(stream);
  (void)hipFree(tmp);
  HIP_TRY(e);
  HIP_TRY(e2);
  return WG_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* wg_last_error(void) { return g_err.c_str(); }

int wg_abi_version(void) { return WG_ABI_VERSION; }

int wg_dense_to_csr_count(const float* adj, int64_t n_rows, int64_t n_cols, int64_t ld, int64_t* indptr,
                          int64_t* nnz_host, void* stream_) {
  if (n_rows < 0 || n_cols < 0 || ld < n_cols || !indptr || !nnz_host || (n_rows > 0 && n_cols > 0 && !adj))
    return fail(WG_ERR_INVALID, "wg_dense_to_csr_count: bad arguments");
  if (n_cols > INT32_MAX) return fail(WG_ERR_INVALID, "wg_dense_to_csr_count: n_cols exceeds int32");
  hipStream_t stream = as_stream(stream_);
  HIP_TRY(hipMemsetAsync(indptr, 0, sizeof(int64_t), stream));
  if (n_rows > 0) {
    hipLaunchKernelGGL(dense_count_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, stream, n_rows, n_cols, ld,
                       adj, indptr + 1);
    LAUNCH_CHECK();
    int rc = cub_call(stream, [&](void* tmp, size_t& bytes) {
      return hipcub::DeviceScan::InclusiveSum(tmp, bytes, indptr + 1, indptr + 1, (int)n_rows, stream);
    });
    if (rc) return rc;
  }
  HIP_TRY(hipMemcpyAsync(nnz_host, indptr + n_rows, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  return WG_OK;
}

int wg_dense_to_csr_fill(const float* adj, int64_t n_rows, int64_t n_cols, int64_t ld, const int64_t* indptr,
                         int32_t* indices, float* values, void* stream_) {
  if (n_rows < 0 || n_cols < 0 || ld < n_cols || !indptr) return fail(WG_ERR_INVALID, "wg_dense_to_csr_fill: bad arguments");
  if (n_rows == 0 || n_cols == 0) return WG_OK;
  hipLaunchKernelGGL(dense_fill_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, as_stream(stream_), n_rows,
                     n_cols, ld, adj, indptr, indices, values);
  LAUNCH_CHECK();
  return WG_OK;
}

int wg_column_degree(int64_t n_rows, int64_t row_offset, const int64_t* indptr, const int32_t* indices,
                     const float* values, double* colsum_f64, double* diag_f64, void* stream_) {
  if (n_rows < 0 || !indptr || !colsum_f64 || !diag_f64) return fail(WG_ERR_INVALID, "wg_column_degree: bad arguments");
  if (n_rows == 0) return WG_OK;
  hipLaunchKernelGGL(column_degree_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, as_stream(stream_), n_rows,
                     row_offset, indptr, indices, values, colsum_f64, diag_f64);
  LAUNCH_CHECK();
  return WG_OK;
}

int wg_laplacian_create(int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t* indptr, const int32_t* indices,
                        const float* values, const float* w_cols, uint32_t flags, void* stream_,
                        wg_laplacian_t* out) {
  if (!out) return fail(WG_ERR_INVALID, "wg_laplacian_create: out is NULL");
  *out = nullptr;
  if (n_rows < 0 || n_cols < n_rows || nnz < 0 || !indptr || (nnz > 0 && !indices))
    return fail(WG_ERR_INVALID, "wg_laplacian_create: bad shape (n_rows=%lld n_cols=%lld nnz=%lld)",
                (long long)n_rows, (long long)n_cols, (long long)nnz);
  if (nnz > INT32_MAX || n_cols > INT32_MAX)
    return fail(WG_ERR_UNSUPPORTED, "wg_laplacian_create: nnz/n_cols exceed int32 (shard the graph)");
  if (n_cols > n_rows && !w_cols)
    return fail(WG_ERR_INVALID, "wg_laplacian_create: halo columns need w_cols");
  hipStream_t stream = as_stream(stream_);
  auto* L = new wg_laplacian_s();
  HIP_TRY(hipGetDevice(&L->device));
  L->n_rows = n_rows;
  L->n_cols = n_cols;
  L->nnz_input = nnz;
  L->reordered = !(flags & WG_FLAG_NO_REORDER);
  int rc = WG_OK;
  int32_t* len = nullptr;
  int32_t* len_sorted = nullptr;
  int32_t* ids = nullptr;
  double* rowsum64 = nullptr;
  float* diag = nullptr;
  double* colsum = nullptr;
  float* sw = nullptr;
  uint8_t* iso_col = nullptr;
  unsigned int* hist = nullptr;
  const int64_t nb_rows = std::max<int64_t>(1, ceil_div(n_rows, 256));
  const int64_t nb_cols = std::max<int64_t>(1, ceil_div(n_cols, 256));
#define TRY(x)               \
  do {                       \
    rc = (x);                \
    if (rc != WG_OK) goto done; \
  } while (0)
#define TRYH(x)                                                                               \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      rc = fail(e_ == hipErrorOutOfMemory ? WG_ERR_OOM : WG_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
      goto done;                                                                              \
    }                                                                                         \
  } while (0)
  {
    TRY(dmalloc(&len, n_rows));
    TRY(dmalloc(&len_sorted, n_rows));
    TRY(dmalloc(&ids, n_rows));
    TRY(dmalloc(&rowsum64, n_rows));
    TRY(dmalloc(&diag, n_rows));
    TRY(dmalloc(&sw, n_cols));
    TRY(dmalloc(&iso_col, n_cols));
    TRY(dmalloc(&hist, kBuckets));
    TRY(dmalloc(&L->rowptr, n_rows + 1));
    TRY(dmalloc(&L->iso, n_rows));
    TRY(dmalloc(&L->perm, n_rows));
    TRY(dmalloc(&L->iperm, n_rows));
    TRY(dmalloc(&L->rowsum, n_rows));
    if (!w_cols) {
      TRY(dmalloc(&colsum, n_cols));
      TRYH(hipMemsetAsync(colsum, 0, sizeof(double) * std::max<int64_t>(1, n_cols), stream));
    }
    if (n_rows > 0) {
      hipLaunchKernelGGL(row_info_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, stream, n_rows, indptr,
                         indices, values, len, rowsum64, diag, colsum);
      TRYH(hipGetLastError());
    }
    if (n_cols > 0) {
      hipLaunchKernelGGL(degree_kernel, dim3(nb_cols), dim3(256), 0, stream, n_cols, n_rows, colsum, diag, w_cols,
                         sw, iso_col);
      TRYH(hipGetLastError());
    }
    // permutation
    if (n_rows > 0) {
      hipLaunchKernelGGL(iota_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, ids);
      TRYH(hipGetLastError());
      if (L->reordered) {
        TRY(cub_call(stream, [&](void* tmp, size_t& bytes) {
          return hipcub::DeviceRadixSort::SortPairsDescending(tmp, bytes, len, len_sorted, ids, L->perm,
                                                              (int)n_rows, 0, 32, stream);
        }));
      } else {
        TRYH(hipMemcpyAsync(L->perm, ids, sizeof(int32_t) * n_rows, hipMemcpyDeviceToDevice, stream));
      }
      hipLaunchKernelGGL(invert_perm_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, L->perm, L->iperm);
      TRYH(hipGetLastError());
      hipLaunchKernelGGL(gather_len_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, L->perm, len, len_sorted,
                         iso_col, L->iso);
      TRYH(hipGetLastError());
      TRYH(hipMemsetAsync(L->rowptr, 0, sizeof(int32_t), stream));
      TRY(cub_call(stream, [&](void* tmp, size_t& bytes) {
        return hipcub::DeviceScan::InclusiveSum(tmp, bytes, len_sorted, L->rowptr + 1, (int)n_rows, stream);
      }));
      int32_t total = 0;
      TRYH(hipMemcpyAsync(&total, L->rowptr + n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
      TRYH(hipStreamSynchronize(stream));
      L->nnz = total;
      TRY(dmalloc(&L->col, L->nnz));
      TRY(dmalloc(&L->val, L->nnz));
      hipLaunchKernelGGL(fill_lhat_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, stream, n_rows, L->perm,
                         L->iperm, indptr, indices, values, sw, L->rowptr, L->col, L->val);
      TRYH(hipGetLastError());
      // row-length buckets (internal order is sorted when reordered)
      TRYH(hipMemsetAsync(hist, 0, sizeof(unsigned int) * kBuckets, stream));
      hipLaunchKernelGGL(bucket_hist_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, len_sorted, hist);
      TRYH(hipGetLastError());
      TRYH(hipMemcpyAsync(L->bucket, hist, sizeof(unsigned int) * kBuckets, hipMemcpyDeviceToHost, stream));
      // float32 row sums (caller order) for X0
      hipLaunchKernelGGL(f64_to_f32_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, rowsum64, L->rowsum);
      TRYH(hipGetLastError());
      TRYH(hipStreamSynchronize(stream));
      // stats
      std::vector<uint8_t> isoh(n_rows);
      TRYH(hipMemcpy(isoh.data(), L->iso, n_rows, hipMemcpyDeviceToHost));
      int64_t niso = 0;
      for (auto v : isoh) niso += v;
      L->n_iso = niso;
      int32_t first_len = 0;
      if (L->reordered) {
        TRYH(hipMemcpy(&first_len, len_sorted, sizeof(int32_t), hipMemcpyDeviceToHost));
        L->max_row = first_len;
      } else {
        std::vector<int32_t> lh(n_rows);
        TRYH(hipMemcpy(lh.data(), len_sorted, sizeof(int32_t) * n_rows, hipMemcpyDeviceToHost));
        L->max_row = n_rows ? *std::max_element(lh.begin(), lh.end()) : 0;
      }
      L->avg_len = n_rows ? L->nnz / n_rows : 0;
    } else {
      TRYH(hipMemsetAsync(L->rowptr, 0, sizeof(int32_t), stream));
      TRYH(hipStreamSynchronize(stream));
    }
  }
done:
#undef TRY
#undef TRYH
  (void)hipFree(len);
  (void)hipFree(len_sorted);
  (void)hipFree(ids);
  (void)hipFree(rowsum64);
  (void)hipFree(diag);
  (void)hipFree(colsum);
  (void)hipFree(sw);
  (void)hipFree(iso_col);
  (void)hipFree(hist);
  if (rc != WG_OK) {
    delete L;
    return rc;
  }
  *out = L;
  return WG_OK;
}

int wg_laplacian_destroy(wg_laplacian_t L) {
  if (!L) return WG_OK;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(L->device);
  (void)hipDeviceSynchronize();
  delete L;
  (void)hipSetDevice(cur);
  return WG_OK;
}

int wg_laplacian_get_info(wg_laplacian_t L, wg_laplacian_info* info) {
  if (!L || !info) return fail(WG_ERR_INVALID, "wg_laplacian_get_info: NULL argument");
  info->n_rows = L->n_rows;
  info->n_cols = L->n_cols;
  info->nnz_input = L->nnz_input;
  info->nnz = L->nnz;
  info->n_isolated = L->n_iso;
  info->max_row_nnz = L->max_row;
  info->n_segments = build_segments(L, 1).n;
  info->reordered = L->reordered ? 1 : 0;
  return WG_OK;
}

int wg_laplacian_export(wg_laplacian_t L, int64_t* indptr, int32_t* indices, float* values, uint8_t* iso,
                        void* stream_) {
  if (!L || !indptr) return fail(WG_ERR_INVALID, "wg_laplacian_export: NULL argument");
  hipStream_t stream = as_stream(stream_);
  const int64_t n = L->n_rows;
  HIP_TRY(hipMemsetAsync(indptr, 0, sizeof(int64_t), stream));
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(export_len_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, n, L->iperm, L->rowptr,
                     indptr + 1);
  LAUNCH_CHECK();
  int rc = cub_call(stream, [&](void* tmp, size_t& bytes) {
    return hipcub::DeviceScan::InclusiveSum(tmp, bytes, indptr + 1, indptr + 1, (int)n, stream);
  });
  if (rc) return rc;
  hipLaunchKernelGGL(export_fill_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, n, L->perm, L->iperm,
                     L->rowptr, L->col, L->val, indptr, indices, values);
  LAUNCH_CHECK();
  if (iso) {
    hipLaunchKernelGGL(export_iso_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, n, L->iperm, L->iso, iso);
    LAUNCH_CHECK();
  }
  return WG_OK;
}

int wg_log1p_degree(wg_laplacian_t L, float* x0, void* stream_) {
  if (!L || (!x0 && L->n_rows)) return fail(WG_ERR_INVALID, "wg_log1p_degree: NULL argument");
  if (L->n_rows == 0) return WG_OK;
  hipLaunchKernelGGL(log1p_degree_kernel, dim3(ceil_div(L->n_rows, 256)), dim3(256), 0, as_stream(stream_),
                     L->n_rows, L->rowsum, x0);
  LAUNCH_CHECK();
  return WG_OK;
}

int wg_cheb_step(wg_laplacian_t L, int32_t k, int64_t F, const float* t_km1, const float* t_km2, float* t_k,
                 float* S, float* H, double alpha0, double alpha_k, void* stream_) {
  if (!L || k < 1 || F < 1 || !t_km1 || (k >= 2 && !t_km2) || (H && !S))
    return fail(WG_ERR_INVALID, "wg_cheb_step: bad arguments (k=%d F=%lld)", k, (long long)F);
  return launch_step(L, k, F, t_km1, t_km2, t_k, S, H, alpha0, alpha_k, as_stream(stream_));
}

int wg_permute_rows(wg_laplacian_t L, int32_t direction, int64_t F, const float* src, float* dst, void* stream_) {
  if (!L || F < 1 || (direction != 0 && direction != 1) || (L->n_rows && (!src || !dst)))
    return fail(WG_ERR_INVALID, "wg_permute_rows: bad arguments");
  const int64_t total = L->n_rows * F;
  if (total == 0) return WG_OK;
  hipLaunchKernelGGL(permute_rows_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, as_stream(stream_), L->n_rows,
                     F, L->perm, direction, src, dst);
  LAUNCH_CHECK();
  return WG_OK;
}

int wg_wavelet_features(wg_laplacian_t L, const float* X0, int64_t F, int32_t K, double s, float* S, float* H,
                        void* stream_) {
  if (!L || F < 1 || K < 0 || (!S && !H) || (L->n_rows && !X0))
    return fail(WG_ERR_INVALID, "wg_wavelet_features: bad arguments (F=%lld K=%d)", (long long)F, K);
  if (L->n_cols != L->n_rows)
    return fail(WG_ERR_INVALID, "wg_wavelet_features: sharded handle (halo columns); use wg_cheb_step");
  hipStream_t stream = as_stream(stream_);
  const int64_t n = L->n_rows;
  if (n == 0) return WG_OK;
  const size_t need = (size_t)3 * n * F + 64;
  if (L->ws_floats < need) {
    HIP_TRY(hipStreamSynchronize(stream));
    (void)hipFree(L->ws);
    L->ws = nullptr;
    L->ws_floats = 0;
    HIP_TRY(hipMalloc(&L->ws, need * sizeof(float)));
    L->ws_floats = need;
  }
  // 256-B aligned sub-buffers
  const size_t stride = ((size_t)n * F + 63) / 64 * 64;
  float* b0 = L->ws;               // T_0 then T_2, T_4, ...
  float* b1 = L->ws + stride;      // T_1, T_3, ...
  float* sint = L->ws + 2 * stride;
  hipLaunchKernelGGL(permute_rows_kernel, dim3(ceil_div(n * F, 256)), dim3(256), 0, stream, n, F, L->perm, 0, X0,
                     b0);
  LAUNCH_CHECK();
  if (K == 0) {
    HIP_TRY(hipMemcpyAsync(sint, b0, sizeof(float) * n * F, hipMemcpyDeviceToDevice, stream));
  }
  for (int32_t k = 1; k <= K; ++k) {
    const float* xm1 = (k & 1) ? b0 : b1;
    const float* xm2 = (k == 1) ? nullptr : ((k & 1) ? b1 : b0);
    float* xk = (k == K) ? nullptr : ((k & 1) ? b1 : b0);  // in place over T_{k-2}
    const double ak = std::exp(-s * (double)k);
    hipEvent_t e_stop = nullptr;
    if (L->prof) {
      while (L->ev.size() < L->ev_used + 2) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        L->ev.push_back(e);
      }
      HIP_TRY(hipEventRecord(L->ev[L->ev_used], stream));
      e_stop = L->ev[L->ev_used + 1];
      L->ev_used += 2;
    }
    int rc = launch_step(L, k, F, xm1, xm2, xk, sint, nullptr, 1.0, ak, stream);
    if (rc) return rc;
    if (e_stop) HIP_TRY(hipEventRecord(e_stop, stream));
  }
  hipLaunchKernelGGL(finalize_kernel, dim3(ceil_div(n, 4)), dim3(kBlock), 0, stream, n, F, L->perm, sint, S, H);
  LAUNCH_CHECK();
  return WG_OK;
}

int wg_profile_enable(wg_laplacian_t L, int32_t enable) {
  if (!L) return fail(WG_ERR_INVALID, "wg_profile_enable: NULL handle");
  L->prof = enable != 0;
  return WG_OK;
}

int wg_profile_collect(wg_laplacian_t L, double* sum_ms, int64_t* launches, double* max_ms) {
  if (!L || !sum_ms || !launches) return fail(WG_ERR_INVALID, "wg_profile_collect: NULL argument");
  double tot = 0.0, mx = 0.0;
  for (size_t i = 0; i + 1 < L->ev_used; i += 2) {
    HIP_TRY(hipEventSynchronize(L->ev[i + 1]));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, L->ev[i], L->ev[i + 1]));
    tot += ms;
    mx = std::max(mx, (double)ms);
  }
  *sum_ms = tot;
  *launches = (int64_t)(L->ev_used / 2);
  if (max_ms) *max_ms = mx;
  L->ev_used = 0;
  return WG_OK;
}

int wg_row_l1_normalize(const float* S, float* H, int64_t n_rows, int64_t F, void* stream_) {
  if (n_rows < 0 || F < 1 || (n_rows && (!S || !H))) return fail(WG_ERR_INVALID, "wg_row_l1_normalize: bad arguments");
  if (n_rows == 0) return WG_OK;
  hipLaunchKernelGGL(l1_normalize_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, as_stream(stream_), n_rows, F,
                     S, H);
  LAUNCH_CHECK();
  return WG_OK;
}

int wg_gather_rows(const float* src, const int32_t* rows, int64_t n, int64_t F, float* dst, void* stream_) {
  if (n < 0 || F < 1 || (n && (!src || !rows || !dst))) return fail(WG_ERR_INVALID, "wg_gather_rows: bad arguments");
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(n * F, 256)), dim3(256), 0, as_stream(stream_), n, F, rows,
                     src, dst);
  LAUNCH_CHECK();
  return WG_OK;
}

}  // extern "C"
