// lds1.hip -- the F == 1 Chebyshev step for unweighted graphs, with the
// gather vector staged in LDS (reference calibration/WATS.py:32-36: the
// recurrence; :65-68: the heat sum, fused into the epilogue).
//
// Why: at F == 1 every nonzero is one random 4-byte gather.  The gather kernel
// (step.hip) issues it as a global load, and the texture-address unit then
// spends about one cycle per distinct cache line: on the Reddit-size graph it
// was 90 % busy and the step ran at 17 % of the HBM roofline (profiles/r01
// s7, s11).  A random ds_read_b32 costs a few LDS cycles instead.
//
// Operator.  For an unweighted graph (every off-diagonal a_ij == 1) scipy's
// value is L_hat_ij = -fl(fl(1 / sw_i) / sw_j) (_laplacian.py:472-474), i.e.
// -dinv_i * dinv_j up to float32 rounding.  So
//     (L_hat x)_i = -dinv_i * sum_j u_j  (- x_i if row i is isolated),
//     u_j = fl32(x_j * dinv_j),
// and the entry stream carries column ids only: no values.  The difference
// from the scipy-rounded values is a few float32 ulps per term, far inside
// the 1e-5 contract (tests/test_gpu_parity.py).
//
// Layout.  Columns are dealt to NB blocks in 32-column chunks (chunk c ->
// block c % NB), which spreads the high-degree columns (relabelled to the
// front) evenly over the blocks.  Block b's entries are stored block-major,
// rows in internal order, with 16-bit local column ids
//     local(c) = (c / 32 / NB) * 32 + c % 32,
// 2 bytes per nonzero instead of 8 (int32 index + float32 value).
//
// Kernel.  One 1024-thread workgroup per CU holds one block of u in LDS
// (<= 160 KiB) and walks a contiguous range of "row groups" of that block:
// 64 / LN consecutive rows, LN lanes per row (LN a power of two sized to the
// rows' lengths).  Waves take groups from an LDS counter.  Sums are float64
// in a fixed order, so results do not depend on the schedule.  With NB == 1
// the epilogue runs in place; otherwise every (block, row) writes a float32
// partial and combine_lds1_kernel adds the NB partials in block order and runs
// the epilogue.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <utility>

#include "internal.h"

namespace wg {
namespace {

constexpr int kLdsThreads = 1024;

struct Lds1Args {
  const int32_t* brp;
  const uint16_t* bcol;
  const int32_t* gcol;  // mode 4: the operator's int32 columns (internal, sorted per row), or a shard's remapped ones
  int32_t hub;          // mode 4: columns [0, hub) staged in LDS, LDS slot hub = 0
  int32_t u_bytes;      // mode 4: extent of u_in (raw-buffer gathers of the tail columns)
  int32_t gshift;       // mode 4: a tail column c (>= hub) is gathered from u[c - gshift] (0, or hub on a shard)
  int32_t n_hranges;    // mode 4 on a shard: LDS slots filled from these ranges of u (0: slots = u[0, hub))
  const int4* hranges;
  const int2* gsell;    // mode 4, SELL-64 ids: per group {first 64-slot line, turns} (nullable)
  const int32_t* csell;
  const int2* groups;
  const int4* wgs;
  const float* u_in;   // u_{k-1}, n_cols (padded to a multiple of 32)
  const float* xm1;    // T_{k-1} own rows (isolated rows' diagonal; T_0 when k == 1)
  const float* xm2;    // T_{k-2} (k >= 2)
  float* xk;           // T_k (nullable)
  float* u_out;        // u_k = T_k * dinv (nullable)
  float* S;            // heat sum (nullable)
  float* part;         // block partials (nb > 1)
  const double* dinv;
  const uint8_t* iso;
  int32_t n;
  int32_t nb;
  int32_t lchunks;
  int32_t k;
  double alpha0;
  double alpha_k;
  int32_t probe_fold;  // -DWG_TIMING_PROBES, hub teams: tail columns folded into [hub, hub + probe_fold)
};

// T_k,i = 2 (L_hat T_{k-1})_i - T_{k-2,i}  (k == 1: T_1 = L_hat T_0), S, u_k.
__device__ __forceinline__ void lds1_epilogue(const Lds1Args& a, int32_t row, double acc) {
  const double di = a.dinv[row];
  double off = -di * acc;
  const float xo = a.xm1[row];
  if (a.iso[row]) off -= (double)xo;  // L_hat_ii = -1
  double t;
  if (a.k == 1) {
    t = off;
  } else {
    t = 2.0 * off - (double)a.xm2[row];
  }
  if (a.xk) __builtin_nontemporal_store((float)t, a.xk + row);
  if (a.u_out) a.u_out[row] = (float)(t * di);
  if (a.S) {
    const double s = (a.k == 1) ? a.alpha0 * (double)xo + a.alpha_k * t : (double)a.S[row] + a.alpha_k * t;
    __builtin_nontemporal_store((float)s, a.S + row);
  }
}

extern __shared__ float g_u_lds[];

// a padding column id for the hub teams' x_of: LDS slot min(c, hub) = the zero slot, and the
// tail gather's byte offset (c - gshift) * 4 wraps past the buffer's extent (< 2^31 bytes), so
// the raw buffer load returns 0 -- a pad adds exactly 0.0
constexpr int32_t kPadCol = 0x7fffffff;

template <bool DIRECT>
__global__ __launch_bounds__(kLdsThreads) void cheb_lds1_kernel(Lds1Args a) {
  __shared__ int s_next;
  const int4 d = a.wgs[blockIdx.x];
  const int b = d.x;
  // stage block b of u: local chunk lc <- global chunk lc * nb + b (128 B each)
  {
    const int n4 = a.lchunks * 8;
    const float4* src = reinterpret_cast<const float4*>(a.u_in);
    float4* dst = reinterpret_cast<float4*>(g_u_lds);
    for (int i = threadIdx.x; i < n4; i += kLdsThreads) {
      const int64_t g4 = ((int64_t)(i >> 3) * a.nb + b) * 8 + (i & 7);
      dst[i] = src[g4];
    }
  }
  if (threadIdx.x == 0) s_next = d.y;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const float* __restrict__ u = g_u_lds;
  const uint16_t* __restrict__ bcol = a.bcol;
  const int32_t* __restrict__ rp = a.brp + (int64_t)b * a.n;
  for (;;) {
    int g = 0;
    if (lane == 0) g = atomicAdd(&s_next, 1);
    g = __builtin_amdgcn_readfirstlane(__shfl(g, 0, 64));
    if (g >= d.z) break;
    const int2 gd = a.groups[g];
    const int nrows = gd.y & 0xffff;
    const int ln = gd.y >> 16;        // power of two, <= 64
    const int sh = __ffs(ln) - 1;
    const int team = lane >> sh;
    const int q = lane & (ln - 1);
    const int32_t row = gd.x + team;
    const bool act = team < nrows;
    double acc = 0.0;
    if (act) {
      const int32_t e1 = rp[row + 1];
      int32_t e = rp[row] + q;
      for (; e + 3 * ln < e1; e += 4 * ln) {
        const uint16_t c0 = bcol[e], c1 = bcol[e + ln], c2 = bcol[e + 2 * ln], c3 = bcol[e + 3 * ln];
        const float x0 = u[c0], x1 = u[c1], x2 = u[c2], x3 = u[c3];
        acc += (double)x0;
        acc += (double)x1;
        acc += (double)x2;
        acc += (double)x3;
      }
      for (; e < e1; e += ln) acc += (double)u[bcol[e]];
#ifdef WG_DEBUG_BOUNDS
      for (int32_t e2 = rp[row] + q; e2 < e1; e2 += ln)
        WG_DCHECK(bcol[e2] < a.lchunks * 32, "block %d row %d: local column %d past %d staged", b, row, (int)bcol[e2],
                  a.lchunks * 32);
#endif
    }
    for (int o = ln >> 1; o >= 1; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (act && q == 0) {
      if constexpr (DIRECT) lds1_epilogue(a, row, acc);
      else a.part[(int64_t)b * a.n + row] = (float)acc;
    }
  }
}

// Mode 4, "hub teams": the column space does not fit LDS, but the rows are
// short (the windows' padding would dominate).  The hub columns [0, hub) --
// the highest-degree ones after relabelling, which receive most gathers
// (ogbn-arxiv-size R-MAT: the top 32 768 columns take 93 %) -- are staged in
// LDS; the tail columns are raw-buffer loads of u.  Branch-free: every entry
// reads LDS slot min(c, hub) (slot hub holds 0) and issues a buffer load
// whose offset is dropped (out of range -> 0, no memory request) for hub
// columns, and the two are added (one of them is 0, so the sum is exact).
// Row teams, row groups and the LDS counter as cheb_lds1_kernel; one column
// block, so the epilogue runs in place.
__global__ __launch_bounds__(kLdsThreads) void cheb_hub1_kernel(Lds1Args a) {
  __shared__ int s_next;
  constexpr uint32_t kDrop = 0x80000000u;
  const int4 d = a.wgs[blockIdx.x];
  const int H = a.hub;
  if (a.n_hranges == 0) {
    const float4* src = reinterpret_cast<const float4*>(a.u_in);
    float4* dst = reinterpret_cast<float4*>(g_u_lds);
    for (int i = threadIdx.x; i < H / 4; i += kLdsThreads) dst[i] = src[i];
    if (threadIdx.x < 32) g_u_lds[H + threadIdx.x] = 0.0f;
  } else {  // a shard's hub: its own top columns and each peer group's top columns
    for (int r = 0; r < a.n_hranges; ++r) {
      const int4 hr = a.hranges[r];
      for (int i = threadIdx.x; i < hr.z; i += kLdsThreads) g_u_lds[hr.y + i] = a.u_in[(int64_t)hr.x + i];
    }
    if (threadIdx.x < 32) g_u_lds[H + threadIdx.x] = 0.0f;
  }
  if (threadIdx.x == 0) s_next = d.y;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.u_in), 0, a.u_bytes, 0x00020000);
  const int lane = threadIdx.x & 63;
  const float* __restrict__ u = g_u_lds;
  const int32_t* __restrict__ col = a.gcol;
  const int32_t* __restrict__ rp = a.brp;
  const int32_t gs = a.gshift;
  auto x_of = [&](int32_t c) {
#ifdef WG_TIMING_PROBES
    if (a.probe_fold > 0 && c >= H && c != kPadCol) c = H + ((c - H) & (a.probe_fold - 1));
#endif
    WG_DCHECK(c == kPadCol || (c >= 0 && (c < H || (uint64_t)(c - gs) * 4u + 4u <= (uint64_t)a.u_bytes)),
              "hub teams: column %d (hub %d, shift %d) past the %u-byte gathered vector", c, H, gs, (unsigned)a.u_bytes);
    const float xl = u[min(c, H)];
    const uint32_t off = c >= H ? (uint32_t)(c - gs) * 4u : kDrop;
    const float xg = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
    return xl + xg;
  };
  // the column ids stream once per step (8M R-MAT: 1 GB against a 4 MB L2 per XCD): non-temporal
  // loads keep them from evicting the gathered u lines (8M R-MAT K=32 step 1030 vs 1147 us;
  // non-temporal u gathers instead: 2068 us; profiles/r03/s50_hub_nt)
  auto ld_id = [](const int32_t* p) { return __builtin_nontemporal_load(p); };
  for (;;) {
    int g = 0;
    if (lane == 0) g = atomicAdd(&s_next, 1);
    g = __builtin_amdgcn_readfirstlane(__shfl(g, 0, 64));
    if (g >= d.z) break;
    const int2 gd = a.groups[g];
    const int nrows = gd.y & 0xffff;
    const int ln = gd.y >> 16;
    const int sh = __ffs(ln) - 1;
    const int team = lane >> sh;
    const int q = lane & (ln - 1);
    const int32_t row = gd.x + team;
    const bool act = team < nrows;
    double acc = 0.0;
    if (act && a.csell) {
      // SELL-64 ids: turn i of this lane is slot (line + i) * 64 + lane -- the same entries in
      // the same order as the CSR walk below (pads: kPadCol, adding 0.0)
      const int2 gs = a.gsell[g];
      const int32_t* __restrict__ cs = a.csell + (int64_t)gs.x * 64 + lane;
      int32_t i = 0;
      for (; i + 3 < gs.y; i += 4) {
        const int32_t c0 = ld_id(cs + (int64_t)i * 64), c1 = ld_id(cs + (int64_t)(i + 1) * 64),
                      c2 = ld_id(cs + (int64_t)(i + 2) * 64), c3 = ld_id(cs + (int64_t)(i + 3) * 64);
        const float x0 = x_of(c0), x1 = x_of(c1), x2 = x_of(c2), x3 = x_of(c3);
        acc += (double)x0;
        acc += (double)x1;
        acc += (double)x2;
        acc += (double)x3;
      }
      for (; i < gs.y; ++i) acc += (double)x_of(ld_id(cs + (int64_t)i * 64));
    } else if (act) {
      const int32_t e1 = rp[row + 1];
      int32_t e = rp[row] + q;
      for (; e + 3 * ln < e1; e += 4 * ln) {
        const int32_t c0 = ld_id(col + e), c1 = ld_id(col + e + ln), c2 = ld_id(col + e + 2 * ln),
                      c3 = ld_id(col + e + 3 * ln);
        const float x0 = x_of(c0), x1 = x_of(c1), x2 = x_of(c2), x3 = x_of(c3);
        acc += (double)x0;
        acc += (double)x1;
        acc += (double)x2;
        acc += (double)x3;
      }
      for (; e < e1; e += ln) acc += (double)x_of(ld_id(col + e));
    }
    for (int o = ln >> 1; o >= 1; o >>= 1) acc += __shfl_down(acc, o, 64);
    if (act && q == 0) lds1_epilogue(a, row, acc);
  }
}


// SELL-64 ids of the hub teams: one wave per row group; lane = team * ln + q takes entries
// rp[row] + q + i * ln, i < turns (pads: kPadCol)
__global__ void sell_fill_kernel(int32_t n_groups, const int2* __restrict__ groups, const int2* __restrict__ gsell,
                                 const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                 int32_t* __restrict__ out) {
  const int32_t g = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (g >= n_groups) return;
  const int2 gd = groups[g], gs = gsell[g];
  const int nrows = gd.y & 0xffff, ln = gd.y >> 16;
  const int team = lane / ln, q = lane % ln;
  const int32_t row = gd.x + team;
  const int32_t e0 = team < nrows ? rowptr[row] + q : 0, e1 = team < nrows ? rowptr[row + 1] : 0;
  int32_t* dst = out + (int64_t)gs.x * 64 + lane;
  for (int32_t i = 0; i < gs.y; ++i) {
    const int32_t e = e0 + i * ln;
    dst[(int64_t)i * 64] = e < e1 ? col[e] : kPadCol;
  }
}

// a row shard's hub plan: column c -> its LDS slot when it is a hub column, else c + hub.
// g (device, 3 * ng + 1 ints): [0, ng] halo group offsets, [ng + 1, 2 ng] hub length per
// group, [2 ng + 1, 3 ng] first slot per group.
__global__ void hub_remap_kernel(int64_t nnz, int32_t n_own, int32_t h1, int32_t hub, int32_t ng,
                                 const int32_t* __restrict__ g, const int32_t* __restrict__ col,
                                 int32_t* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const int32_t c = col[e];
  int32_t slot = -1;
  if (c < n_own) {
    slot = c < h1 ? c : -1;
  } else {
    const int32_t h = c - n_own;
    int lo = 0, hi = ng;  // group q with g[q] <= h < g[q + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (g[mid] <= h) lo = mid;
      else hi = mid;
    }
    const int32_t idx = h - g[lo];
    slot = idx < g[ng + 1 + lo] ? g[2 * ng + 1 + lo] + idx : -1;
  }
  out[e] = slot >= 0 ? slot : c + hub;
}

__global__ __launch_bounds__(256) void combine_lds1_kernel(Lds1Args a) {
  const int32_t row = blockIdx.x * 256 + threadIdx.x;
  if (row >= a.n) return;
  double acc = 0.0;
  for (int b = 0; b < a.nb; ++b) acc += (double)a.part[(int64_t)b * a.n + row];  // fixed block order
  lds1_epilogue(a, row, acc);
}

__global__ void scale_dinv_kernel(int64_t n, const float* __restrict__ x, const double* __restrict__ dinv,
                                  float* __restrict__ u) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) u[i] = (float)((double)x[i] * dinv[i]);
}

// block entry counts: cnt[b * n + r] = entries of row r in block b
__global__ __launch_bounds__(256) void lds1_count_kernel(int32_t n, int32_t nb, const int32_t* __restrict__ rowptr,
                                                        const int32_t* __restrict__ col, int32_t* __restrict__ cnt) {
  const int32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  for (int32_t e = rowptr[r] + lane; e < rowptr[r + 1]; e += 64) {
    const int32_t b = (col[e] >> 5) % nb;
    atomicAdd(cnt + (int64_t)b * n + r, 1);
  }
}

// block-major entries with local column ids, each (row, block) in CSR order
__global__ __launch_bounds__(256) void lds1_fill_kernel(int32_t n, int32_t nb, const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col, const int32_t* __restrict__ brp,
                                                       uint16_t* __restrict__ bcol) {
  const int32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  int32_t mypos = lane < nb ? brp[(int64_t)lane * n + r] : 0;  // lane b: next slot of block b
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int32_t e0 = rowptr[r], e1 = rowptr[r + 1];
  for (int32_t base = e0; base < e1; base += 64) {
    const int32_t e = base + lane;
    int32_t c = 0, blk = -1;
    if (e < e1) {
      c = col[e];
      blk = (c >> 5) % nb;
    }
    for (int bb = 0; bb < nb; ++bb) {
      const unsigned long long m = __ballot(blk == bb);
      if (!m) continue;
      const int32_t pos = __shfl(mypos, bb, 64);
      if (blk == bb) bcol[pos + __popcll(m & lt)] = (uint16_t)((((c >> 5) / nb) << 5) | (c & 31));
      if (lane == bb) mypos += __popcll(m);
    }
  }
}


// ---------------------------------------------------------------------------
// mode 2: chunk windows.  Every non-empty (row, block) segment is padded to a
// whole number of 8-id chunks (16 B; pad ids point at a zero LDS slot), and
// bit 15 of the first id of a segment flags its start.  A wave streams a
// contiguous chunk range, 64 chunks (512 ids, one 16-B load per lane) per
// window with the next two windows in flight; a lane sums its chunk's 8
// values, and a segmented inclusive scan over the wave (fixed shuffle order)
// gives each segment's sum, carried across windows in registers.  Each
// segment's sum goes to part[segment]; combine_lds2_kernel adds each row's
// segments in block order and runs the epilogue.
struct Lds2Args {
  const uint4* chunk;
  const int4* wdesc;
  const int32_t* wblock;
  const int32_t* pos;
  int32_t n_part;  // segments (part[] length)
  Lds1Args e;  // epilogue operands (+ u_in, part, nb, lchunks, n)
};

// Prefetch: an unconditional load from a clamped index (`last` is a valid
// chunk).  Chunks past the wave's range are replaced by pad ids where they are
// consumed (mask_chunk), not here: touching a loaded value right after the
// load (or loading inside a branch) makes the waitcnt pass drain every
// in-flight load, which serialises the prefetch.
__device__ __forceinline__ uint4 load_chunk(const uint4* __restrict__ ch, int32_t c, int32_t last) {
  return ch[min(c, last)];
}
__device__ __forceinline__ uint4 mask_chunk(const uint4 v, bool ok, uint32_t zz) {
  return make_uint4(ok ? v.x : zz, ok ? v.y : zz, ok ? v.z : zz, ok ? v.w : zz);
}

// One step of the segmented inclusive scan through DPP (VALU only, no LDS):
// add the value of the lane CTRL selects when it belongs to the same segment.
// Lanes without a source keep `old` (0.0 / an impossible segment id).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void seg_scan_step(double& s, int32_t pid) {
  const int lo = __double2loint(s), hi = __double2hiint(s);
  const int tlo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROWMASK, 0xf, false);
  const int thi = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROWMASK, 0xf, false);
  const int tp = __builtin_amdgcn_update_dpp(INT32_MIN, pid, CTRL, ROWMASK, 0xf, false);
  if (tp == pid) s += __hiloint2double(thi, tlo);
}

// Window scan (independent of the carry, so two windows' scans interleave):
// the lane's chunk sum of its 8 values, then a segmented inclusive scan over
// the wave -- row_shr 1/2/4/8 inside 16-lane rows, row_bcast 15 / 31 across
// rows, a fixed order.  lpid = segment starts at lanes <= lane (0: the
// segment open at the window start).
struct WinScan {
  double s;
  unsigned long long F;
  int32_t lpid;
};
__device__ __forceinline__ WinScan lds2_scan(const uint4 q, const float* __restrict__ u) {
  WinScan w;
  const bool flag = (q.x & 0x8000u) != 0u;
#ifdef WG_EXP_NOLDS  // timing-only experiment: no LDS reads (wrong results)
  double s = (double)(q.x & 0x7fffu) + (double)(q.y & 0xffffu) + (double)(q.z & 0xffffu) + (double)(q.w >> 16);
#else
  double s = (double)u[q.x & 0x7fffu];
  s += (double)u[q.x >> 16];
  s += (double)u[q.y & 0xffffu];
  s += (double)u[q.y >> 16];
  s += (double)u[q.z & 0xffffu];
  s += (double)u[q.z >> 16];
  s += (double)u[q.w & 0xffffu];
  s += (double)u[q.w >> 16];
#endif
  w.F = __ballot(flag);
#ifdef WG_EXP_NOSCAN  // timing-only experiment: no segmented scan (wrong results)
  w.lpid = 0;
  w.s = s;
  return w;
#endif
  w.lpid = (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(w.F >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)w.F, 0u)) +
           (flag ? 1 : 0);
  seg_scan_step<0x111, 0xf>(s, w.lpid);  // row_shr:1
  seg_scan_step<0x112, 0xf>(s, w.lpid);  // row_shr:2
  seg_scan_step<0x114, 0xf>(s, w.lpid);  // row_shr:4
  seg_scan_step<0x118, 0xf>(s, w.lpid);  // row_shr:8
  seg_scan_step<0x142, 0xa>(s, w.lpid);  // row_bcast:15 -> rows 1, 3
  seg_scan_step<0x143, 0xc>(s, w.lpid);  // row_bcast:31 -> rows 2, 3
  w.s = s;
  return w;
}

// Window finish: segment sums to part[], the open one carried in (cur, carry).
// Branch-free: both stores are buffer stores every lane issues (the b32
// builtin takes integer data: store the float's bits), with an out-of-range
// offset (dropped by the hardware) where nothing is due, so the waitcnt pass
// sees the same memory-op count on every path.
__device__ __forceinline__ void lds2_finish(WinScan w, __amdgpu_buffer_rsrc_t part, int lane, int32_t first,
                                            int32_t& cur, double& carry) {
  constexpr uint32_t kDrop = 0x80000000u;
  const int32_t pid = cur + w.lpid;
  double s = w.s;
  if (w.lpid == 0) s += carry;  // continued from the last window
  // the open segment ended at the window boundary: lane 0 flushes the carry
  const bool flush = (w.F & 1ull) && lane == 0 && cur >= first;
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)carry), part, flush ? (uint32_t)cur * 4u : kDrop, 0, 0);
  // a segment ends at lane l < 63 when lane l + 1 starts one
  const bool end = lane < 63 && ((w.F >> (lane + 1)) & 1ull);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)s), part, end ? (uint32_t)pid * 4u : kDrop, 0, 0);
  cur += (int32_t)__popcll(w.F);
  const int lo = __builtin_amdgcn_readlane(__double2loint(s), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(s), 63);
  carry = __hiloint2double(hi, lo);
}

// D (even) windows in flight per wave, processed in pairs: both loads of the
// next pair are issued first, then the two scans (independent), then the two
// finishes.  The loop is unrolled so each window's registers are reloaded in
// place (no copy that would wait on a pending load).
template <int D>
__global__ __launch_bounds__(kLdsThreads) void cheb_lds2_kernel(Lds2Args A) {
  const Lds1Args& a = A.e;
  const int b = A.wblock[blockIdx.x];
  const int zslot = a.lchunks * 32;  // zero slot for pad ids
  {
    const int n4 = a.lchunks * 8;
    const float4* src = reinterpret_cast<const float4*>(a.u_in);
    float4* dst = reinterpret_cast<float4*>(g_u_lds);
    for (int i = threadIdx.x; i < n4; i += kLdsThreads) {
      const int64_t g4 = ((int64_t)(i >> 3) * a.nb + b) * 8 + (i & 7);
      dst[i] = src[g4];
    }
    if (threadIdx.x == 0) g_u_lds[zslot] = 0.0f;
  }
  const int lane = threadIdx.x & 63;
  const int4 wd = A.wdesc[blockIdx.x * (kLdsThreads / 64) + (threadIdx.x >> 6)];
  const int32_t c0 = wd.x, c1 = wd.y;
  const uint4* __restrict__ ch = A.chunk;
  const uint32_t zz = (uint32_t)zslot | ((uint32_t)zslot << 16);
  const int32_t last = max(c1 - 1, 0);
  const __amdgpu_buffer_rsrc_t part =
      __builtin_amdgcn_make_buffer_rsrc(a.part, 0, A.n_part * 4, 0x00020000);  // raw buffer, gfx9 dword 3
  uint4 q[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {  // overlaps the LDS fill
    q[i] = load_chunk(ch, c0 + 64 * i + lane, last);
    // the loop issues (load, store, store) per window; two dropped stores here give the
    // loop header the same in-flight pattern on entry, so its wait keeps D windows in flight
    __builtin_amdgcn_raw_buffer_store_b32(0u, part, 0x80000000u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(0u, part, 0x80000000u, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  const float* __restrict__ u = g_u_lds;
  int32_t cur = wd.z - 1;  // segment open at the window start (none yet)
  double carry = 0.0;
  // whole groups of D windows; windows past c1 are all pad ids (no flags, no stores)
  for (int32_t cw = c0; cw < c1; cw += 64 * D) {
#pragma unroll
    for (int i = 0; i < D; i += 2) {
      const int32_t w0 = cw + 64 * i, w1 = w0 + 64;
      const uint4 qa = mask_chunk(q[i], w0 + lane < c1, zz);
      const uint4 qb = mask_chunk(q[i + 1], w1 + lane < c1, zz);
      q[i] = load_chunk(ch, w0 + 64 * D + lane, last);
      q[i + 1] = load_chunk(ch, w1 + 64 * D + lane, last);
      __builtin_amdgcn_sched_barrier(0);  // issue the prefetches here, not after the windows
      const WinScan sa = lds2_scan(qa, u);
      const WinScan sb = lds2_scan(qb, u);
      lds2_finish(sa, part, lane, wd.z, cur, carry);
      lds2_finish(sb, part, lane, wd.z, cur, carry);
    }
  }
  if (lane == 0 && cur >= wd.z) a.part[cur] = (float)carry;
}

// ---------------------------------------------------------------------------
// K chunks per lane (K = 2, 4): a window is 64*K consecutive chunks, lane l
// holding chunks K*l .. K*l+K-1 in sequence order.  Segments that start and
// end inside a lane are summed sequentially and stored by that lane; one
// segmented scan over the lanes' tail sums per window (K times fewer scans
// per id than cheb_lds2_kernel).  Lane l's scan segment starts at the highest
// lane <= l holding a segment start (seg0); a scan step adds its source lane
// when the source is >= seg0.  Same fixed order on every run.
__device__ __forceinline__ double chunk_sum(const uint4 q, const float* __restrict__ u) {
  double s = (double)u[q.x & 0x7fffu];
  s += (double)u[q.x >> 16];
  s += (double)u[q.y & 0xffffu];
  s += (double)u[q.y >> 16];
  s += (double)u[q.z & 0xffffu];
  s += (double)u[q.z >> 16];
  s += (double)u[q.w & 0xffffu];
  s += (double)u[q.w >> 16];
  return s;
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ void seg_scan_step_src(double& s, int src, int seg0) {
  const int tlo = __builtin_amdgcn_update_dpp(0, __double2loint(s), CTRL, ROWMASK, 0xf, false);
  const int thi = __builtin_amdgcn_update_dpp(0, __double2hiint(s), CTRL, ROWMASK, 0xf, false);
  if (src >= seg0) s += __hiloint2double(thi, tlo);  // lanes without a source read 0.0
}

template <int K>
__device__ __forceinline__ void lds3_window(const uint4 (&q)[K], const float* __restrict__ u,
                                            __amdgpu_buffer_rsrc_t part, int lane, int32_t first, int32_t& cur,
                                            double& carry) {
  constexpr uint32_t kDrop = 0x80000000u;
  double sc[K];
  bool f[K];
  int32_t before = 0;  // segment starts in lanes < lane
  int32_t total = 0;   // segment starts in the window
#pragma unroll
  for (int j = 0; j < K; ++j) {
    f[j] = (q[j].x & 0x8000u) != 0u;
    sc[j] = chunk_sum(q[j], u);
    const unsigned long long B = __ballot(f[j]);
    before += (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(B >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B, 0u));
    total += (int32_t)__popcll(B);
  }
  const int32_t open = cur + before;  // segment open before this lane's first chunk
  // lane-local: head (chunks before the first start), segments inside the lane, tail
  double run = 0.0, head = 0.0;
  int nf = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {  // branch-free: a (possibly dropped) store per slot
    // a start after an earlier one in this lane ends a segment that lies inside the lane
    const bool inner = f[j] && nf > 0;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)run), part, inner ? (uint32_t)(open + nf) * 4u : kDrop,
                                          0, 0);
    head = (f[j] && nf == 0) ? run : head;
    run = f[j] ? 0.0 : run;
    nf += f[j] ? 1 : 0;
    run += sc[j];
  }
  const bool has = nf > 0;
  // scan over lanes: value = tail sum (whole lane when it holds no start)
  const unsigned long long H = __ballot(has);
  const unsigned long long le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
  const unsigned long long m = H & le;
  const int seg0 = m ? 63 - __clzll(m) : -1;
  double P = run;
  seg_scan_step_src<0x111, 0xf>(P, lane - 1, seg0);                     // row_shr:1
  seg_scan_step_src<0x112, 0xf>(P, lane - 2, seg0);                     // row_shr:2
  seg_scan_step_src<0x114, 0xf>(P, lane - 4, seg0);                     // row_shr:4
  seg_scan_step_src<0x118, 0xf>(P, lane - 8, seg0);                     // row_shr:8
  seg_scan_step_src<0x142, 0xa>(P, (lane & ~15) - 1, seg0);             // row_bcast:15 -> rows 1, 3
  seg_scan_step_src<0x143, 0xc>(P, 31, seg0);                           // row_bcast:31 -> rows 2, 3
  if (seg0 < 0) P += carry;  // the window's open segment
  // value of the segment open before this lane, at the end of lane - 1
  const int plo = __builtin_amdgcn_update_dpp(0, __double2loint(P), 0x138, 0xf, 0xf, false);  // wave_shr:1
  const int phi = __builtin_amdgcn_update_dpp(0, __double2hiint(P), 0x138, 0xf, 0xf, false);
  const double Pprev = (lane == 0) ? carry : __hiloint2double(phi, plo);
  // a lane holding a start completes the segment open before it
  const bool done = has && !(lane == 0 && open < first);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(Pprev + head)), part,
                                        done ? (uint32_t)open * 4u : kDrop, 0, 0);
  const int lo = __builtin_amdgcn_readlane(__double2loint(P), 63);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(P), 63);
  carry = __hiloint2double(hi, lo);
  cur += total;
}

template <int K>
__global__ __launch_bounds__(kLdsThreads) void cheb_lds3_kernel(Lds2Args A) {
  constexpr int D = 2;  // windows in flight
  const Lds1Args& a = A.e;
  const int b = A.wblock[blockIdx.x];
  const int zslot = a.lchunks * 32;
  {
    const int n4 = a.lchunks * 8;
    const float4* src = reinterpret_cast<const float4*>(a.u_in);
    float4* dst = reinterpret_cast<float4*>(g_u_lds);
    for (int i = threadIdx.x; i < n4; i += kLdsThreads) {
      const int64_t g4 = ((int64_t)(i >> 3) * a.nb + b) * 8 + (i & 7);
      dst[i] = src[g4];
    }
    if (threadIdx.x == 0) g_u_lds[zslot] = 0.0f;
  }
  const int lane = threadIdx.x & 63;
  const int4 wd = A.wdesc[blockIdx.x * (kLdsThreads / 64) + (threadIdx.x >> 6)];
  const int32_t c0 = wd.x, c1 = wd.y;
  const uint4* __restrict__ ch = A.chunk;
  const uint32_t zz = (uint32_t)zslot | ((uint32_t)zslot << 16);
  const int32_t last = max(c1 - 1, 0);
  const __amdgpu_buffer_rsrc_t part = __builtin_amdgcn_make_buffer_rsrc(a.part, 0, A.n_part * 4, 0x00020000);
  constexpr int W = 64 * K;  // chunks per window
  uint4 q[D][K];
#pragma unroll
  for (int i = 0; i < D; ++i) {
#pragma unroll
    for (int j = 0; j < K; ++j) q[i][j] = load_chunk(ch, c0 + W * i + K * lane + j, last);
#pragma unroll
    for (int j = 0; j < K + 1; ++j) __builtin_amdgcn_raw_buffer_store_b32(0u, part, 0x80000000u, 0, 0);  // loop's pattern
    __builtin_amdgcn_sched_barrier(0);
  }
  __syncthreads();
  const float* __restrict__ u = g_u_lds;
  int32_t cur = wd.z - 1;
  double carry = 0.0;
  for (int32_t cw = c0; cw < c1; cw += W * D) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int32_t w0 = cw + W * i;
      uint4 cq[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        cq[j] = mask_chunk(q[i][j], w0 + K * lane + j < c1, zz);
        q[i][j] = load_chunk(ch, w0 + W * D + K * lane + j, last);
      }
      __builtin_amdgcn_sched_barrier(0);
      lds3_window<K>(cq, u, part, lane, wd.z, cur, carry);
    }
  }
  if (lane == 0 && cur >= wd.z) a.part[cur] = (float)carry;
}

__global__ __launch_bounds__(256) void combine_lds2_kernel(Lds2Args A) {
  const Lds1Args& a = A.e;
  const int32_t row = blockIdx.x * 256 + threadIdx.x;
  if (row >= a.n) return;
  // 8 blocks at a time: all segment ids, then all partials, from clamped
  // indices (no load behind a branch, so they overlap); fixed block order
  double acc = 0.0;
  for (int b0 = 0; b0 < a.nb; b0 += 8) {
    int32_t p[8];
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = A.pos[(int64_t)min(b0 + j, a.nb - 1) * a.n + row];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = a.part[max(p[j], 0)];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (b0 + j < a.nb && p[j] >= 0) ? (double)v[j] : 0.0;
  }
  lds1_epilogue(a, row, acc);
}

// segment fill: wave per row; lane b owns the row's segment of block b
// (start chunk cpt[b * n + r]); ids keep CSR order, pad ids -> zero slot,
// bit 15 on the segment's first id
// perm = 1: a segment's k entries are dealt column-major over its nch = ceil(k/8)
// chunks (rank t -> chunk t % nch, slot t / nch), so one lane's chunks span
// the whole (column-sorted) segment instead of one narrow column range.
__global__ __launch_bounds__(256) void lds2_fill_kernel(int32_t n, int32_t nb, int32_t zslot, int32_t perm,
                                                       const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col, const int32_t* __restrict__ cpt,
                                                       const int32_t* __restrict__ cnt, uint16_t* __restrict__ ids) {
  const int32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const int64_t start = lane < nb ? (int64_t)cpt[(int64_t)lane * n + r] * 8 : 0;
  int64_t mypos = start;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int32_t e0 = rowptr[r], e1 = rowptr[r + 1];
  for (int32_t base = e0; base < e1; base += 64) {
    const int32_t e = base + lane;
    int32_t c = 0, blk = -1;
    if (e < e1) {
      c = col[e];
      blk = (c >> 5) % nb;
    }
    for (int bb = 0; bb < nb; ++bb) {
      const unsigned long long m = __ballot(blk == bb);
      if (!m) continue;
      const int64_t p0 = __shfl(mypos, bb, 64);
      const int64_t s0 = __shfl(start, bb, 64);
      if (blk == bb) {
        int64_t dst = p0 + __popcll(m & lt);
        uint32_t id = (uint32_t)((((c >> 5) / nb) << 5) | (c & 31));
        if (dst == s0) id |= 0x8000u;
        if (perm) {
          const int64_t rank = dst - s0;
          const int64_t nch = ((int64_t)cnt[(int64_t)bb * n + r] + 7) / 8;
          dst = s0 + (rank % nch) * 8 + rank / nch;
        }
        ids[dst] = (uint16_t)id;
      }
      if (lane == bb) mypos += __popcll(m);
    }
  }
  if (lane < nb) {
    const int32_t k = cnt[(int64_t)lane * n + r];
    const int64_t nch = ((int64_t)k + 7) / 8;
    for (int64_t q = 0; q < nch * 8; ++q)
      if (perm ? ((q >> 3) + (q & 7) * nch >= k) : (q >= k)) ids[start + q] = (uint16_t)zslot;
  }
}

// row groups of the teams kernels (modes 1 and 4) and their workgroup split.
// h: block-major row pointers [nb * n + 1] (entries of block b, row r =
// [h[b*n+r], h[b*n+r+1])).
int build_groups(wg_laplacian_s* L, Lds1Plan* p, const std::vector<int32_t>& h, int64_t nb, int32_t iter_knob) {
  const int64_t n = p->n;
  // row groups per block: 64/LN consecutive rows, LN lanes per row
  const int iter = std::max(1, iter_knob);
  std::vector<int2> groups;
  std::vector<int64_t> gcost;  // entries + per-row overhead, for the workgroup split
  std::vector<int64_t> bfirst(nb + 1);
  for (int64_t b = 0; b < nb; ++b) {
    bfirst[b] = (int64_t)groups.size();
    const int32_t* r = h.data() + b * n;
    auto len = [&](int64_t i) { return (int64_t)(r[i + 1] - r[i]); };
    int64_t i = 0;
    while (i < n) {
      int ln = 1;
      while (ln < 64 && (int64_t)ln * iter < len(i)) ln <<= 1;
      int rows = (int)std::min<int64_t>(64 / ln, n - i);
      // a longer row further in the group widens the team (rows are only roughly sorted per block)
      for (;;) {
        int64_t mx = 0;
        for (int j = 0; j < rows; ++j) mx = std::max(mx, len(i + j));
        if (ln >= 64 || mx <= 2 * (int64_t)ln * iter) break;
        ln <<= 1;
        rows = (int)std::min<int64_t>(64 / ln, n - i);
      }
      int64_t c = 16;
      for (int j = 0; j < rows; ++j) c += len(i + j) + 2;
      groups.push_back(make_int2((int32_t)i, rows | (ln << 16)));
      gcost.push_back(c);
      i += rows;
    }
  }
  bfirst[nb] = (int64_t)groups.size();
  p->n_groups = (int32_t)groups.size();
  // workgroups: about one per CU, split evenly over the blocks, each block's
  // groups cut into equal-cost contiguous ranges
  int n_wg = L->tune.lds_wg > 0 ? L->tune.lds_wg : n_cus(L->device);
  n_wg = (int)std::max<int64_t>(nb, std::min<int64_t>(n_wg, ceil_div(p->nnz + 2 * n, 4096)));
  std::vector<int4> wgs;
  for (int64_t b = 0; b < nb; ++b) {
    const int m = (int)(n_wg / nb + (b < n_wg % nb ? 1 : 0));
    int64_t tot = 0;
    for (int64_t g = bfirst[b]; g < bfirst[b + 1]; ++g) tot += gcost[g];
    int64_t g = bfirst[b], acc = 0;
    for (int w = 0; w < m; ++w) {
      const int64_t target = tot * (w + 1) / m;
      const int64_t g0 = g;
      while (g < bfirst[b + 1] && (acc + gcost[g] <= target || w == m - 1)) acc += gcost[g++];
      if (g > g0 || w == m - 1) wgs.push_back(make_int4((int)b, (int)g0, (int)g, 0));
    }
  }
  p->n_wg = (int32_t)wgs.size();
  int rc = 0;
  if ((rc = dmalloc(&p->groups, groups.size())) || (rc = dmalloc(&p->wgs, wgs.size())) ||
      (rc = dmalloc(&p->part, nb > 1 ? (size_t)(nb * n) : 1)))
    return rc;
  WG_HIP_TRY(hipMemcpy(p->groups, groups.data(), sizeof(int2) * std::max<size_t>(1, groups.size()),
                       hipMemcpyHostToDevice));
  WG_HIP_TRY(hipMemcpy(p->wgs, wgs.data(), sizeof(int4) * std::max<size_t>(1, wgs.size()), hipMemcpyHostToDevice));
  WG_HIP_TRY(hipDeviceSynchronize());
  return WG_OK;
}



// mode 2 plan: segment chunk offsets, segment ids, chunk array, wave ranges.
// `cnt` = entries per (block, row) (block-major), p->brp holds the same on the device.
int build_windows(wg_laplacian_s* L, Lds1Plan* p, const std::vector<int32_t>& cnt) {
  const int64_t n = p->n, nb = p->nb;
  p->mode = 2;
  std::vector<int32_t> cpt(nb * n), pos(nb * n);
  std::vector<int64_t> seg_chunk;  // first chunk of each segment (+ end sentinel)
  std::vector<int64_t> bseg(nb + 1);
  int64_t chunks = 0;
  for (int64_t b = 0; b < nb; ++b) {
    bseg[b] = (int64_t)seg_chunk.size();
    for (int64_t r = 0; r < n; ++r) {
      const int64_t i = b * n + r;
      const int64_t k = cnt[i];
      cpt[i] = (int32_t)chunks;
      if (k > 0) {
        pos[i] = (int32_t)seg_chunk.size();
        seg_chunk.push_back(chunks);
        chunks += (k + 7) / 8;
      } else {
        pos[i] = -1;
      }
    }
  }
  bseg[nb] = (int64_t)seg_chunk.size();
  seg_chunk.push_back(chunks);
  if (chunks >= INT32_MAX / 2) return fail(WG_ERR_UNSUPPORTED, "lds2 plan: too many chunks (%lld)", (long long)chunks);
  p->n_chunks = chunks;
  p->n_pairs = (int32_t)(seg_chunk.size() - 1);
  // waves: workgroups split evenly over the blocks, each block's segments cut
  // into 16 * (its workgroups) contiguous ranges of equal cost (chunks + 1 per segment)
  constexpr int kW = kLdsThreads / 64;
  int n_wg = L->tune.lds_wg > 0 ? L->tune.lds_wg : n_cus(L->device);
  n_wg = (int)std::max<int64_t>(nb, std::min<int64_t>(n_wg, ceil_div(chunks + p->n_pairs, 256)));
  // workgroups per block in proportion to the block's cost (the hub columns
  // make block 0 the heaviest), at least one each, largest remainders first
  std::vector<int64_t> bcost(nb);
  int64_t all = 0;
  for (int64_t b = 0; b < nb; ++b) {
    bcost[b] = (seg_chunk[bseg[b + 1]] - seg_chunk[bseg[b]]) + (bseg[b + 1] - bseg[b]);
    all += bcost[b];
  }
  std::vector<int> mb(nb, 1);
  {
    int left = n_wg - (int)nb;
    std::vector<std::pair<double, int64_t>> rem;
    for (int64_t b = 0; b < nb && all > 0; ++b) {
      const double want = (double)n_wg * bcost[b] / all - 1.0;
      const int extra = std::max(0, std::min(left, (int)want));
      mb[b] += extra;
      left -= extra;
      rem.push_back({want - extra, b});
    }
    std::sort(rem.begin(), rem.end(), [](auto& x, auto& y) { return x.first > y.first; });
    for (size_t i = 0; left > 0 && i < rem.size(); ++i, --left) ++mb[rem[i].second];
  }
  std::vector<int4> wd;
  std::vector<int32_t> wb;
  for (int64_t b = 0; b < nb; ++b) {
    const int m = mb[b];
    const int64_t s0 = bseg[b], s1 = bseg[b + 1];
    const int64_t tot = (seg_chunk[s1] - seg_chunk[s0]) + (s1 - s0);
    int64_t sg = s0;
    for (int w = 0; w < m * kW; ++w) {
      const int64_t target = tot * (w + 1) / (m * kW);
      const int64_t g0 = sg;
      while (sg < s1 && ((seg_chunk[sg + 1] - seg_chunk[s0]) + (sg + 1 - s0) <= target || w == m * kW - 1)) ++sg;
      wd.push_back(make_int4((int)seg_chunk[g0], (int)seg_chunk[sg], (int)g0, 0));
      if (w % kW == 0) wb.push_back((int32_t)b);
    }
  }
  p->n_wg = (int32_t)wb.size();
  int rc = 0;
  int32_t* cpt_d = nullptr;
  if ((rc = dmalloc(&p->chunk, (size_t)chunks + 1)) || (rc = dmalloc(&p->pos, (size_t)(nb * n))) ||
      (rc = dmalloc(&p->wdesc, wd.size())) || (rc = dmalloc(&p->wblock, wb.size())) ||
      (rc = dmalloc(&p->part, (size_t)std::max<int32_t>(1, p->n_pairs))) || (rc = dmalloc(&cpt_d, (size_t)(nb * n))))
    return rc;
  auto done = [&](int code) {
    (void)hipFree(cpt_d);
    return code;
  };
  if (hipMemcpy(cpt_d, cpt.data(), sizeof(int32_t) * nb * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->pos, pos.data(), sizeof(int32_t) * nb * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->wdesc, wd.data(), sizeof(int4) * wd.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->wblock, wb.data(), sizeof(int32_t) * wb.size(), hipMemcpyHostToDevice) != hipSuccess)
    return done(fail(WG_ERR_HIP, "lds2 plan: upload failed"));
  hipLaunchKernelGGL(lds2_fill_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, 0, (int32_t)n, (int32_t)nb,
                     p->lchunks * 32, L->tune.lds_perm, L->rowptr, L->col, cpt_d, p->brp, reinterpret_cast<uint16_t*>(p->chunk));
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return done(fail(WG_ERR_HIP, "lds2 plan: fill failed"));
  done(0);
  char buf[256];
  snprintf(buf, sizeof(buf),
           "lds1: windows rows=%lld cols=%d nnz=%lld blocks=%lld lds_floats=%d segments=%d chunks=%lld "
           "(pad %.1f%%) workgroups=%d (+combine)\n",
           (long long)n, p->n_cols, (long long)p->nnz, (long long)nb, p->lchunks * 32, p->n_pairs, (long long)chunks,
           p->nnz ? 100.0 * (8.0 * chunks - p->nnz) / p->nnz : 0.0, p->n_wg);
  p->text = buf;
  for (int64_t b = 0; b < nb; ++b) {
    snprintf(buf, sizeof(buf), "  block %lld: cost %lld (%.1f%%) workgroups %d\n", (long long)b, (long long)bcost[b],
             all ? 100.0 * bcost[b] / all : 0.0, mb[b]);
    p->text += buf;
  }
  return WG_OK;
}
}  // namespace

void Lds1Plan::release() {
  for (void* p : {(void*)brp, (void*)bcol, (void*)groups, (void*)wgs, (void*)part, (void*)chunk, (void*)pos,
                  (void*)wdesc, (void*)wblock, (void*)hcol, (void*)hranges, (void*)gsell,
                  (void*)csell})
    (void)hipFree(p);
  hcol = nullptr;
  gsell = nullptr;
  csell = nullptr;
  hranges = nullptr;
  n_hranges = 0;
  chunk = nullptr;
  pos = nullptr;
  wdesc = nullptr;
  wblock = nullptr;
  brp = nullptr;
  bcol = nullptr;
  groups = nullptr;
  wgs = nullptr;
  part = nullptr;
}

void release_lds1(wg_laplacian_s* L) {
  release_tiles(L);  // the hybrid step's plans are invalidated by the same events
  for (int i = 0; i < 2; ++i) {
    if (L->lds1[i]) {
      L->lds1[i]->release();
      delete L->lds1[i];
      L->lds1[i] = nullptr;
    }
    L->lds1_failed[i] = false;
  }
}

// A row shard's hub: the p->hub highest-degree columns among the own columns
// [0, n_rows) and each peer's halo group, each of which is a descending-degree
// list, so the choice is a prefix of each; LDS slots own prefix first, then the
// groups in peer order.  Builds the remapped column array the kernel reads.
static int build_shard_hub(wg_laplacian_s* L, Lds1Plan* p, int32_t nnz) {
  const int64_t n_own = L->n_rows, n_cols = L->n_cols;
  const int ng = (int)L->halo_off.size() - 1;
  const int64_t hmax = p->hub;
  std::vector<double> dinv(n_cols);
  WG_HIP_TRY(hipMemcpy(dinv.data(), L->dinv, sizeof(double) * n_cols, hipMemcpyDeviceToHost));
  // candidates: the first hmax of each list, by degree w = 1 / dinv^2 (largest first)
  std::vector<std::pair<double, int>> cand;  // (dinv: smaller = higher degree, list)
  auto add_list = [&](int64_t b, int64_t e, int id) {
    for (int64_t i = b; i < std::min(e, b + hmax); ++i) cand.push_back({dinv[i], id});
  };
  add_list(0, n_own, 0);
  for (int q = 0; q < ng; ++q) add_list(n_own + L->halo_off[q], n_own + L->halo_off[q + 1], q + 1);
  const int64_t take = std::min<int64_t>(hmax, (int64_t)cand.size());
  std::nth_element(cand.begin(), cand.begin() + std::max<int64_t>(take - 1, 0), cand.end(),
                   [](const std::pair<double, int>& x, const std::pair<double, int>& y) { return x.first < y.first; });
  std::vector<int32_t> cnt(ng + 1, 0);
  for (int64_t i = 0; i < take; ++i) ++cnt[cand[i].second];
  // slots: own prefix, then each group's prefix
  std::vector<int4> ranges;
  std::vector<int32_t> g(3 * ng + 1, 0);
  int32_t slot = 0;
  if (cnt[0] > 0) ranges.push_back(make_int4(0, 0, cnt[0], 0));
  slot = cnt[0];
  for (int q = 0; q < ng; ++q) {
    g[q] = (int32_t)L->halo_off[q];
    g[ng + 1 + q] = cnt[q + 1];
    g[2 * ng + 1 + q] = slot;
    if (cnt[q + 1] > 0) ranges.push_back(make_int4((int)(n_own + L->halo_off[q]), slot, cnt[q + 1], 0));
    slot += cnt[q + 1];
  }
  g[ng] = (int32_t)L->halo_off[ng];
  p->hub = slot;
  p->lchunks = slot / 32 + 2;  // + the zero slots (32 at slot `hub`)
  p->n_hranges = (int32_t)ranges.size();
  if (int rc = dmalloc(&p->hranges, std::max<size_t>(1, ranges.size()))) return rc;
  if (!ranges.empty())
    WG_HIP_TRY(hipMemcpy(p->hranges, ranges.data(), sizeof(int4) * ranges.size(), hipMemcpyHostToDevice));
  int32_t* gd = nullptr;
  if (int rc = dmalloc(&gd, g.size())) return rc;
  WG_HIP_TRY(hipMemcpy(gd, g.data(), sizeof(int32_t) * g.size(), hipMemcpyHostToDevice));
  if (int rc = dmalloc(&p->hcol, (size_t)nnz + 4)) {
    (void)hipFree(gd);
    return rc;
  }
  WG_HIP_TRY(hipMemset(p->hcol + nnz, 0, 4 * sizeof(int32_t)));
  if (nnz > 0)
    hipLaunchKernelGGL(hub_remap_kernel, dim3((unsigned)ceil_div(nnz, 256)), dim3(256), 0, 0, (int64_t)nnz,
                       (int32_t)n_own, cnt[0], p->hub, ng, gd, L->col, p->hcol);
  const hipError_t e1 = hipGetLastError();
  const hipError_t e2 = hipDeviceSynchronize();
  (void)hipFree(gd);
  if (e1 != hipSuccess || e2 != hipSuccess) return fail(WG_ERR_HIP, "hub_remap: %s", hipGetErrorString(e1 ? e1 : e2));
  return WG_OK;
}

int get_lds1_plan(wg_laplacian_s* L, bool active_only, Lds1Plan** out) {
  *out = nullptr;
  active_only = active_only && L->reordered;
  const int slot = active_only ? 1 : 0;
  if (L->lds1[slot]) {
    *out = L->lds1[slot];
    return WG_OK;
  }
  if (!L->unit || !L->dinv || L->tune.lds == 0 || L->lds1_failed[slot]) return WG_OK;
  const int64_t n = active_only ? L->n_active : L->n_rows;
  const int64_t n_cols = active_only ? L->n_active : L->n_cols;
  // mode: 1 row teams, 2 chunk windows; 3 = auto (measured, profiles/r01/s14): one column
  // block -> teams (one launch, epilogue in place: PubMed 6.0 vs 6.8 us gather, 12.2
  // windows); several blocks -> windows on long rows (avg >= 64 per row: Reddit 60 vs 588
  // us), else the gather kernel (ogbn-arxiv F=1, avg 25: 12.5 vs 14.0 / 14.6 us)
  int mode = L->tune.lds;
  int32_t nnz_rows = 0;
  if (n > 0) WG_HIP_TRY(hipMemcpy(&nnz_rows, L->rowptr + n, sizeof(int32_t), hipMemcpyDeviceToHost));
  int32_t hub = std::max(32, std::min(40672, L->tune.lds_cb / 32 * 32));
  if (mode == 3) {
    const int64_t nb1 = ceil_div(ceil_div(std::max<int64_t>(n_cols, 1), 32), 40704 / 32);
    // hub teams when every workgroup's entries outnumber the hub floats it stages 8 to 1
    // (8M R-MAT K=32: 1219 vs 1645 us gather; ogbn-arxiv-size F=1: 12.5-15.8 vs 11.6 us)
    const int64_t hub_auto = std::min<int64_t>(40672, (int64_t)nnz_rows / (8 * (int64_t)n_cus(L->device)) / 32 * 32);
    if (nb1 == 1) {
      mode = 1;
    } else if (n > 0 && nnz_rows / n >= 64) {
      mode = 2;
    } else if (hub_auto >= 16384 && L->n_cols == L->n_rows) {
      // Row shards take the gather kernel.  Their halo groups are in descending degree
      // (wats_hip/dist.py), so the hot columns sit in few cache lines and the gather kernel
      // reads them from L2: 8M R-MAT 8-way shard 211 us per step vs 282 us with the hub
      // kernel staging the shard's own + every group's top columns (lds = 4, ranged hub);
      // 4-way 425 vs 767, 2-way 822 vs 837 (profiles/r02/s10_shard_probe_8m.log)
      mode = 4;
      hub = (int32_t)hub_auto;
    } else {
      mode = 0;
    }
  }
  if (mode == 0 || n == 0 || (mode == 4 && (int64_t)n_cols * 4 >= ((int64_t)1 << 31))) {
    L->lds1_failed[slot] = true;
    return WG_OK;
  }
  if (mode == 4) {
    // hub teams: one "block" of the hub columns, the operator's own CSR
    auto* p = new Lds1Plan();
    p->mode = 4;
    p->n = (int32_t)n;
    p->n_cols = (int32_t)n_cols;
    p->nb = 1;
    p->nnz = nnz_rows;
    const int64_t cols32 = ceil_div(std::max<int64_t>(n_cols, 1), 32) * 32;
    p->hub = (int32_t)std::min<int64_t>(cols32, hub);
    p->lchunks = p->hub / 32 + 1;  // + the zero slot (and padding)
    p->ulen = cols32;
    std::vector<int32_t> h(n + 1);
    WG_HIP_TRY(hipMemcpy(h.data(), L->rowptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
    int rc = build_groups(L, p, h, 1, L->tune.hub_iter);
    if (!rc && L->n_cols > L->n_rows && !L->halo_off.empty() && !active_only) rc = build_shard_hub(L, p, nnz_rows);
    if (!rc && !p->hcol && L->tune.hub_sell && p->n_groups > 0) {
      // SELL-64 ids: turns per group = the longest team row / team width
      std::vector<int2> gr(p->n_groups), gs(p->n_groups);
      if (hipMemcpy(gr.data(), p->groups, sizeof(int2) * p->n_groups, hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(WG_ERR_HIP, "hub sell: copy");
      int64_t lines = 0;
      for (int32_t g = 0; g < p->n_groups && !rc; ++g) {
        const int nrows = gr[g].y & 0xffff, ln = gr[g].y >> 16;
        int64_t turns = 0;
        for (int t = 0; t < nrows; ++t) {
          const int64_t len = h[gr[g].x + t + 1] - h[gr[g].x + t];
          turns = std::max<int64_t>(turns, ceil_div(len, ln));
        }
        gs[g] = make_int2((int32_t)lines, (int32_t)turns);
        lines += turns;
      }
      if (!rc && lines * 64 >= ((int64_t)1 << 31)) rc = WG_ERR_UNSUPPORTED;  // stay on the CSR walk
      if (!rc) rc = dmalloc(&p->gsell, (size_t)p->n_groups);
      if (!rc) rc = dmalloc(&p->csell, (size_t)std::max<int64_t>(1, lines * 64));
      if (!rc && hipMemcpy(p->gsell, gs.data(), sizeof(int2) * p->n_groups, hipMemcpyHostToDevice) != hipSuccess)
        rc = fail(WG_ERR_HIP, "hub sell: copy");
      if (!rc) {
        hipLaunchKernelGGL(sell_fill_kernel, dim3((unsigned)ceil_div(p->n_groups, 4)), dim3(256), 0, nullptr,
                           p->n_groups, p->groups, p->gsell, L->rowptr, L->col, p->csell);
        const hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) rc = fail(WG_ERR_HIP, "hub sell: %s", hipGetErrorString(e));
      }
      if (rc == WG_ERR_UNSUPPORTED) {
        (void)hipFree(p->gsell);
        (void)hipFree(p->csell);
        p->gsell = nullptr;
        p->csell = nullptr;
        rc = WG_OK;
      }
      snprintf(p->sell_note, sizeof(p->sell_note), " sell_lines=%lld (ids %.2fx nnz)", (long long)lines,
               (double)lines * 64 / std::max<int64_t>(1, nnz_rows));
    }
    if (rc) {
      p->release();
      delete p;
      return rc;
    }
    char buf[256];
    snprintf(buf, sizeof(buf), "lds1: hub teams rows=%lld cols=%lld nnz=%d hub=%d groups=%d workgroups=%d ranges=%d%s\n",
             (long long)n, (long long)n_cols, nnz_rows, p->hub, p->n_groups, p->n_wg, p->n_hranges, p->sell_note);
    p->text = buf;
    L->lds1[slot] = p;
    *out = p;
    return WG_OK;
  }
  // + static LDS <= 160 KiB; windows: 15-bit local ids and a zero slot at 32 * lchunks
  const int cb = std::max(32, std::min(mode == 2 ? 32736 : 40704, L->tune.lds_cb / 32 * 32));
  const int64_t nchunks = ceil_div(std::max<int64_t>(n_cols, 1), 32);
  const int64_t nb = ceil_div(nchunks, cb / 32);
  if (n == 0 || nb > std::min(L->tune.lds_maxnb, 64)) {
    L->lds1_failed[slot] = true;
    return WG_OK;
  }
  auto* p = new Lds1Plan();
  p->n = (int32_t)n;
  p->n_cols = (int32_t)n_cols;
  p->nb = (int32_t)nb;
  p->lchunks = (int32_t)ceil_div(nchunks, nb);
  int rc = WG_OK;
  auto bail = [&](int code) {
    p->release();
    delete p;
    return code;
  };
  int32_t nnz = 0;
  WG_HIP_TRY(hipMemcpy(&nnz, L->rowptr + n, sizeof(int32_t), hipMemcpyDeviceToHost));
  p->nnz = nnz;
  const int64_t ncnt = nb * n + 1;
  if ((rc = dmalloc(&p->brp, ncnt))) return bail(rc);
  WG_HIP_TRY(hipMemset(p->brp, 0, sizeof(int32_t) * ncnt));
  const dim3 rgrid((unsigned)ceil_div(n, 4));
  hipLaunchKernelGGL(lds1_count_kernel, rgrid, dim3(256), 0, 0, (int32_t)n, (int32_t)nb, L->rowptr, L->col, p->brp);
  WG_LAUNCH_CHECK();
  // exclusive scan on the host (the plan is built once per graph; brp is small)
  std::vector<int32_t> h(ncnt);
  WG_HIP_TRY(hipMemcpy(h.data(), p->brp, sizeof(int32_t) * ncnt, hipMemcpyDeviceToHost));
  if (mode == 2) {
    rc = build_windows(L, p, h);
    if (rc) return bail(rc);
    L->lds1[slot] = p;
    *out = p;
    return WG_OK;
  }
  if ((rc = dmalloc(&p->bcol, (size_t)nnz + 8))) return bail(rc);
  WG_HIP_TRY(hipMemset(p->bcol, 0, sizeof(uint16_t) * ((size_t)nnz + 8)));
  {
    int64_t run = 0;
    for (int64_t i = 0; i < ncnt; ++i) {
      const int64_t c = h[i];
      h[i] = (int32_t)run;
      run += c;
    }
    if (run != nnz) return bail(fail(WG_ERR_HIP, "lds1 plan: entry count %lld != nnz %d", (long long)run, nnz));
  }
  WG_HIP_TRY(hipMemcpy(p->brp, h.data(), sizeof(int32_t) * ncnt, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(lds1_fill_kernel, rgrid, dim3(256), 0, 0, (int32_t)n, (int32_t)nb, L->rowptr, L->col, p->brp,
                     p->bcol);
  WG_LAUNCH_CHECK();

  if ((rc = build_groups(L, p, h, nb, L->tune.lds_iter))) return bail(rc);
  WG_HIP_TRY(hipDeviceSynchronize());
  char buf[256];
  snprintf(buf, sizeof(buf), "lds1: rows=%lld cols=%lld nnz=%d blocks=%lld lds_floats=%d groups=%d workgroups=%d%s\n",
           (long long)n, (long long)n_cols, nnz, (long long)nb, p->lchunks * 32, p->n_groups, p->n_wg,
           nb > 1 ? " (+combine)" : "");
  p->text = buf;
  L->lds1[slot] = p;
  *out = p;
  return WG_OK;
}

int launch_scale_dinv(wg_laplacian_s* L, int64_t n, const float* x, float* u, hipStream_t stream) {
  if (n <= 0) return WG_OK;
  hipLaunchKernelGGL(scale_dinv_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, stream, n, x, L->dinv, u);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int launch_lds1_step(wg_laplacian_s* L, Lds1Plan* p, int32_t k, const float* u_km1, const float* t_km1,
                     const float* t_km2, float* t_k, float* u_k, float* S, double alpha0, double alpha_k,
                     hipStream_t stream) {
  if (p->n == 0) return WG_OK;
  if (int rc = prof_mark(L, stream, true)) return rc;
  const size_t lds = (size_t)p->lchunks * 32 * sizeof(float);
  Lds1Args a{};
  a.brp = p->brp;
  a.bcol = p->bcol;
  a.groups = p->groups;
  a.wgs = p->wgs;
  a.u_in = u_km1;
  a.xm1 = t_km1;
  a.xm2 = t_km2;
  a.xk = t_k;
  a.u_out = u_k;
  a.S = S;
  a.part = p->part;
  a.dinv = L->dinv;
  a.iso = L->iso;
  a.n = p->n;
  a.nb = p->nb;
  a.lchunks = p->lchunks;
  a.k = k;
  a.alpha0 = alpha0;
  a.alpha_k = alpha_k;
  a.probe_fold = L->tune.probe_fold;
  if (p->mode == 4) {
    if (int rc = ensure_dyn_lds((const void*)cheb_hub1_kernel, 160 * 1024 - 64)) return rc;
    a.brp = L->rowptr;
    a.gcol = p->hcol ? p->hcol : L->col;
    a.hub = p->hub;
    a.u_bytes = (int32_t)(p->ulen * 4);
    a.gshift = p->hcol ? p->hub : 0;
    a.n_hranges = p->n_hranges;
    a.gsell = p->gsell;
    a.csell = p->csell;
    a.hranges = p->hranges;
    hipLaunchKernelGGL(cheb_hub1_kernel, dim3(p->n_wg), dim3(kLdsThreads), lds, stream, a);
    WG_LAUNCH_CHECK();
    return prof_mark(L, stream, false);
  }
  if (p->mode == 2) {
    const int depth = L->tune.lds_depth >= 8 ? 8 : L->tune.lds_depth >= 4 ? 4 : 2;
    const void* fn2 = depth == 8   ? (const void*)cheb_lds2_kernel<8>
                      : depth == 4 ? (const void*)cheb_lds2_kernel<4>
                                   : (const void*)cheb_lds2_kernel<2>;
    if (int rc = ensure_dyn_lds(fn2, 160 * 1024 - 64)) return rc;
    Lds2Args A{};
    A.chunk = p->chunk;
    A.wdesc = p->wdesc;
    A.wblock = p->wblock;
    A.pos = p->pos;
    A.n_part = p->n_pairs;
    A.e = a;
    const int kpl = L->tune.lds_k;
    if (kpl == 2 || kpl == 4) {
      const void* fn3 = kpl == 4 ? (const void*)cheb_lds3_kernel<4> : (const void*)cheb_lds3_kernel<2>;
      if (int rc = ensure_dyn_lds(fn3, 160 * 1024 - 64)) return rc;
      if (kpl == 4)
        hipLaunchKernelGGL(cheb_lds3_kernel<4>, dim3(p->n_wg), dim3(kLdsThreads), lds + sizeof(float), stream, A);
      else
        hipLaunchKernelGGL(cheb_lds3_kernel<2>, dim3(p->n_wg), dim3(kLdsThreads), lds + sizeof(float), stream, A);
    } else if (depth == 8)
      hipLaunchKernelGGL(cheb_lds2_kernel<8>, dim3(p->n_wg), dim3(kLdsThreads), lds + sizeof(float), stream, A);
    else if (depth == 4)
      hipLaunchKernelGGL(cheb_lds2_kernel<4>, dim3(p->n_wg), dim3(kLdsThreads), lds + sizeof(float), stream, A);
    else
      hipLaunchKernelGGL(cheb_lds2_kernel<2>, dim3(p->n_wg), dim3(kLdsThreads), lds + sizeof(float), stream, A);
    WG_LAUNCH_CHECK();
    hipLaunchKernelGGL(combine_lds2_kernel, dim3((unsigned)ceil_div(p->n, 256)), dim3(256), 0, stream, A);
    WG_LAUNCH_CHECK();
    return prof_mark(L, stream, false);
  }
  const bool direct = p->nb == 1;
  const void* fn = direct ? (const void*)cheb_lds1_kernel<true> : (const void*)cheb_lds1_kernel<false>;
  if (int rc = ensure_dyn_lds(fn, 160 * 1024 - 64)) return rc;
  if (direct)
    hipLaunchKernelGGL(cheb_lds1_kernel<true>, dim3(p->n_wg), dim3(kLdsThreads), lds, stream, a);
  else
    hipLaunchKernelGGL(cheb_lds1_kernel<false>, dim3(p->n_wg), dim3(kLdsThreads), lds, stream, a);
  WG_LAUNCH_CHECK();
  if (!direct) {
    hipLaunchKernelGGL(combine_lds1_kernel, dim3((unsigned)ceil_div(p->n, 256)), dim3(256), 0, stream, a);
    WG_LAUNCH_CHECK();
  }
  return prof_mark(L, stream, false);
}

}  // namespace wg
