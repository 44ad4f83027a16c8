// step_dev.h -- device-side pieces of the Chebyshev step kernels shared by step.hip
// (cheb_step_kernel and its plan) and hub.hip (the LDS-hub wave kernel): the launch
// arguments, the per-row epilogue (reference calibration/WATS.py:32-36 recurrence, :65-68
// heat sum, :71-72 normalisation) and the gather loops.
#pragma once

#include "internal.h"

namespace wg {

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
  const int32_t* out_perm;  // last step, finalize fused: S / H rows go to caller row out_perm[row] ...
  float* S_out;             // ... of S_out / H (internal S is only read)
  int64_t ld;         // row stride (floats) of every vector
  int32_t LF;         // lanes across the tile's columns (tile width = LF * VEC)
  int32_t k;          // step index (1 or >= 2)
  double alpha0;
  double alpha_k;
  const ChunkDesc* chunks;
  double* partial;
  const int2* rowchunks;  // split rows: {first chunk, chunk count}
  uint32_t* arrivals;     // split rows: in-kernel combine counters, 0 between launches (nullable = combine_kernel)
  int64_t seg_mask;
  int32_t nt;
  int32_t bcast;
  int32_t vidx;
  int32_t clen;        // 0 = forward recurrence + heat sum; 1 / 2 = Clenshaw step / final (ClenArgs)
  const float* x0;     // Clenshaw: X0 rows (internal order, stride ld)
  double ck, cacc;     // Clenshaw: out = ck * X0 + cacc * acc - xm2
  // Clenshaw on unweighted graphs (L_hat_ij = -dinv_i dinv_j): the chain carries u = b * dinv, so the
  // gathers need no values (val == nullptr: every value 1).  uin: xm1 holds u; uprev: xm2 holds u;
  // uout: xk gets u.
  const double* dinv;
  int32_t uin, uprev, uout;
  // hybrid step (tiles.hip; col = the tail-first column array, rsplit = each row's tail end):
  // phase 4 sums the tail [e0, rsplit[row]), adds part (the dense blocks' float64 sums, row
  // stride ld) to rows with dense entries and runs the epilogue.  0 = the whole row.
  int32_t phase;
  const int32_t* rsplit;
  const double* part;
  int32_t probe;  // timing probe (-DWG_TIMING_PROBES builds, knob "probe"): gathers only, acc stored to xk
  // timing probes of the gather's request count / footprint (-DWG_TIMING_PROBES, results wrong):
  // probe_h2: columns below it gather one aligned 128-B line (lanes of columns 32.. skip);
  // probe_fold: every gathered column folded into [0, probe_fold)
  int32_t probe_h2, probe_fold;
  int32_t probe_ns;  // -DWG_TIMING_PROBES: Clenshaw epilogue without its X0 (bit 0) / b_{k+2} (bit 1) row loads
  int32_t coldnt;  // -DWG_TIMING_PROBES: gathers of columns >= coldnt with the non-temporal hint (the hot rows
                   // are not evicted by once-used cold lines?), the others plain: two loads, one dropped
  // value-free gathers on the padded CSR (cheb_step_kernel<..., P4 = true>): each row's column ids
  // padded to a multiple of 4 with kPadCol (prp / pcol); the gathered vector xm1 as a raw buffer
  // of u_bytes bytes, so a pad id's offset falls outside it and its load returns 0 with no request
  const int32_t* prp;
  const int32_t* pcol;
  int32_t p4v;        // the padded-CSR loop variant (tuning key gather4; launch_main)
  uint32_t u_bytes;
  unsigned long long* trace;  // -DWG_TIMING_PROBES, knob "trace": per-wave timeline of one launch
  const int2* wmeta;  // team waves in SELL order (Plan::sell): per wave {first chunk, turns}
  const int4* sell;
  // the chain's FIRST value-free launch without a permute-in pass (team.hip, tuning key "fold"): the
  // gathers read the caller's X0 (xm1 = x0c) through ids already mapped to caller rows (sell = the
  // team table's sell0) and scale each gathered row by its column's dinv (sdinv: one float64 per id
  // slot), so u_0 = X0 * dinv is never stored; the epilogue reads its own X0 row at caller row
  // perm_in[row] and writes it to x0i (the internal X0 the later steps read)
  int32_t first;
  double* tsum;  // hybrid tail beside the dense blocks (hyb_conc): the row sums go here, no epilogue
  const double* sdinv;
  const float* x0c;
  float* x0i;
  const int32_t* perm_in;
#ifdef WG_DEBUG_BOUNDS
  uint64_t dbg_sell_bytes;  // bytes of sell (0: unchecked)
#endif
};

// a padded-CSR column id whose byte offset (id * row bytes <= 256) lies past every gathered buffer
constexpr int32_t kPadCol = 0xFFFFFF;
// kPadCol ids after the last row of pcol: a sub-group's id loads run up to (PF + 1) turns of CPT
// steps (<= 4096 ids each) past its range
constexpr int32_t kPcolTail = 65536;

// the entry range of a row (or of a split-row chunk) this launch's phase covers
__device__ __forceinline__ void phase_range(const StepArgs& a, int64_t row, int32_t& e0, int32_t& e1) {
  if (a.phase == 0) return;
  e1 = min(e1, a.rsplit[row]);
  if (e1 < e0) e1 = e0;
}

// the hybrid step: the dense blocks' sums, for rows with dense entries
template <int VEC>
__device__ __forceinline__ void part_add(const StepArgs& a, int64_t row, int fs, double (&acc)[VEC]) {
  if (a.phase != 4 || a.rsplit[row] == a.rowptr[row + 1]) return;
  const double* p = a.part + row * a.ld + (int64_t)fs * VEC;
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] += p[j];
}

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

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int VEC>
__device__ __forceinline__ void store_vec_nt(float* p, const double (&x)[VEC]) {
  if constexpr (VEC == 1) {
    __builtin_nontemporal_store((float)x[0], p);
  } else if constexpr (VEC == 2) {
    f32x2 v = {(float)x[0], (float)x[1]};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x2*>(p));
  } else {
    f32x4 v = {(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  }
}

// 16-B write-through (sc1) store: the line leaves the XCD's L2 instead of staying there
// (MI355X_MICROARCH.md, inter-workgroup visibility table), so a step's T_k stream does not evict
// the gathered rows of the same step from L2; other widths store plainly
template <int VEC>
__device__ __forceinline__ void store_vec_sc1(float* p, const double (&x)[VEC]) {
  if constexpr (VEC == 4) {
    f32x4 v = {(float)x[0], (float)x[1], (float)x[2], (float)x[3]};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    for (int j = 0; j < VEC; ++j) p[j] = (float)x[j];
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

// Per-row epilogue operands, loaded BEFORE the row's gathers so their latency
// overlaps the accumulation (they do not depend on it).
template <int VEC>
struct EpiIn {
  float prev[VEC];  // k == 1: T_0 own row (for S); k >= 2: T_{k-2} own row
  float sold[VEC];  // S own row (k >= 2); Clenshaw: X0 own row
  int iso;
  int32_t orow;     // out_perm[row] (finalize fused into the last step)
  double dinv;      // Clenshaw on u = b * dinv: dinv of the row
};

template <int VEC>
__device__ __forceinline__ void epi_prefetch(const StepArgs& a, int64_t row, int fs, EpiIn<VEC>& in) {
  if (a.probe) return;
  const int64_t off = row * a.ld + (int64_t)fs * VEC;
  in.iso = a.iso[row];
  in.orow = a.out_perm ? a.out_perm[row] : (int32_t)row;
  if (a.clen) {
    in.dinv = (a.uin | a.uprev | a.uout) ? a.dinv[row] : 1.0;
#ifdef WG_TIMING_PROBES
    if (a.probe_ns & 2) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) in.prev[j] = 0.0f;
    } else
#endif
    if (a.xm2) {
      load_vec<VEC>(a.xm2 + off, in.prev);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) in.prev[j] = 0.0f;
    }
    if (a.first) {  // the caller's X0 row (no permute-in pass)
      in.orow = a.perm_in[row];
      load_vec<VEC>(a.x0c + (int64_t)in.orow * a.ld + (int64_t)fs * VEC, in.sold);
      return;
    }
#ifdef WG_TIMING_PROBES
    if (a.probe_ns & 1) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) in.sold[j] = 0.0f;
    } else
#endif
    if (a.x0) {
      load_vec<VEC>(a.x0 + off, in.sold);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) in.sold[j] = 0.0f;
    }
    return;
  }
  load_vec<VEC>((a.k == 1 ? a.xm1 : a.xm2) + off, in.prev);
  if (a.S && a.k >= 2) load_vec<VEC>(a.S + off, in.sold);
}

// Per-row epilogue, run by the LF lanes holding the row's sums (`lane0` = wave
// lane of the row's first column slice, for the H shuffle): diagonal of
// isolated rows, recurrence, T_k store, heat sum, optional normalisation.
template <int VEC>
__device__ __forceinline__ void step_epilogue(const StepArgs& a, int64_t row, int fs, double (&acc)[VEC],
                                              const EpiIn<VEC>& in, int lane0) {
  const int64_t off = row * a.ld + (int64_t)fs * VEC;
  const bool nt_st = (a.nt & 4) != 0;
  if (a.probe) {  // timing probe: the row sums only (results are not the chain's)
    if (a.xk) store_vec<VEC>(a.xk + off, acc);
    return;
  }
  if (a.clen && a.uin) {  // sum of u_j over the row: L_hat b = -dinv_i * sum (off-diagonal part)
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] *= -in.dinv;
  }
  if (a.first) {  // the internal X0 row for the later steps; an isolated row's diagonal term is X0 itself
    if (a.x0i) {
      double x[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) x[j] = (double)in.sold[j];
      store_vec<VEC>(a.x0i + off, x);
    }
    if (in.iso) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] -= (double)in.sold[j];
    }
  } else if (in.iso) {  // L_hat_ii = -1 (scipy setdiag(1 - iso), then "- identity")
    float x[VEC];
    if (a.k == 1) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) x[j] = in.prev[j];
    } else {
      load_vec<VEC>(a.xm1 + off, x);
    }
    const double xs = (a.clen && a.uin) ? 1.0 / in.dinv : 1.0;  // own row of u -> b
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] -= (double)x[j] * xs;
  }
  double t[VEC];
  if (a.clen) {  // Clenshaw: b = ck * X0 + cacc * (L_hat b') - b''
    const double ps = a.uprev ? 1.0 / in.dinv : 1.0;
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      t[j] = a.ck * (double)in.sold[j] + a.cacc * acc[j] - (double)in.prev[j] * ps;
    if (a.uout && a.xk) {
      double u[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) u[j] = t[j] * in.dinv;
      if (nt_st) store_vec_nt<VEC>(a.xk + off, u);
      else if (a.nt & 8) store_vec_sc1<VEC>(a.xk + off, u);
      else store_vec<VEC>(a.xk + off, u);
      return;  // never the final step (S is written only there)
    }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = (a.k == 1) ? acc[j] : 2.0 * acc[j] - (double)in.prev[j];
  }
  if (a.xk) {
    if (nt_st) store_vec_nt<VEC>(a.xk + off, t);
    else if (a.nt & 8) store_vec_sc1<VEC>(a.xk + off, t);
    else store_vec<VEC>(a.xk + off, t);
  }
  if (a.S) {
    double s[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j)  // k == 1: S = alpha0*T_0 + alpha1*T_1; Clenshaw final: S = t
      s[j] = a.clen ? t[j]
                    : (a.k == 1) ? a.alpha0 * (double)in.prev[j] + a.alpha_k * t[j]
                                 : (double)in.sold[j] + a.alpha_k * t[j];
    // finalize fused (last step): the rows go straight to the caller's order
    const int64_t oo = a.out_perm ? (int64_t)in.orow * a.ld + (int64_t)fs * VEC : off;
    float* Sd = a.out_perm ? a.S_out : a.S;
    if (nt_st) store_vec_nt<VEC>(Sd + oo, s);
    else store_vec<VEC>(Sd + oo, s);
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
      store_vec<VEC>(a.H + oo, h);
    }
  }
}

// acc += sum over e = e, e+stride, ... < e1 of val[e] * x[col[e]].
// Default: float64 FMAs (a float32 x float32 product is exact in float64).
// -DWG_LANE_F32 (experimental build): each lane's short sequence (<= a few
// dozen terms) in float32, added to the float64 accumulator at the end.
template <int VEC>
__device__ __forceinline__ void accumulate(const StepArgs& a, int32_t e, int32_t e1, int32_t stride,
                                           const float* __restrict__ xb, double (&acc)[VEC]) {
  const int32_t* __restrict__ col = a.col;
  const float* __restrict__ val = a.val;
  const int64_t ld = a.ld;
#ifdef WG_LANE_F32
  float part[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) part[j] = 0.0f;
#define WG_FMA(j, vv, xx) part[j] = fmaf((vv), (xx), part[j])
#else
#define WG_FMA(j, vv, xx) acc[j] = fma((double)(vv), (double)(xx), acc[j])
#endif
  for (; e + 3 * stride < e1; e += 4 * stride) {
    int32_t c[4];
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = col[e + u * stride];
      v[u] = val ? val[e + u * stride] : 1.0f;
    }
    float x[4][VEC];
#pragma unroll
    for (int u = 0; u < 4; ++u) load_vec<VEC>(xb + (int64_t)c[u] * ld, x[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < VEC; ++j) WG_FMA(j, v[u], x[u][j]);
  }
  for (; e < e1; e += stride) {
    const int32_t c = col[e];
    const float v = val ? val[e] : 1.0f;
    float x[VEC];
    load_vec<VEC>(xb + (int64_t)c * ld, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) WG_FMA(j, v, x[j]);
  }
#undef WG_FMA
#ifdef WG_LANE_F32
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] += (double)part[j];
#endif
}

// Sum the partial sums of n lane sub-groups (lanes base + q*LF + fs, q < n)
// into sub-group 0, in a fixed order (tree for power-of-two n).  Must be
// called by every lane of the wave (uniform control flow).
template <int VEC>
__device__ __forceinline__ void reduce_subgroups(double (&acc)[VEC], int n, int LF, int base, int fs) {
  if (n <= 1) return;
  if ((n & (n - 1)) == 0) {
    for (int off = n >> 1; off >= 1; off >>= 1) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += __shfl_down(acc[j], off * LF, 64);
    }
  } else {
    double tot[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) tot[j] = acc[j];
    for (int q = 1; q < n; ++q) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) tot[j] += __shfl(acc[j], base + q * LF + fs, 64);
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = tot[j];
  }
}

// Dynamic LDS of cheb_step_hot_kernel: the hot-column cache.
extern __shared__ float g_hot_lds[];

// Two separate loads (LDS / global) behind a branch.  Written as a ternary,
// clang merges them into one flat load of a selected generic pointer, which
// both loses the LDS fast path and (ROCm 7.2) miscompiles the LDS-to-flat
// cast ("V_CMP_NE_U32 src_shared_base" illegal instruction).
__device__ __forceinline__ float hot_or_global(const float* hot, const float* __restrict__ xb, int32_t c, int32_t H,
                                               int64_t ld) {
  float x;
  if (c < H) {
    x = hot[c];
    asm volatile("" ::: "memory");
  } else {
    x = xb[(int64_t)c * ld];
    asm volatile("" ::: "memory");
  }
  return x;
}

// F == 1 with an LDS hot-column cache: columns [0, H) of T_{k-1} (the
// highest-degree rows after relabelling, which receive most gathers) are read
// from LDS, the rest from global memory.
__device__ __forceinline__ void accumulate_hot1(const StepArgs& a, int32_t e, int32_t e1, int32_t stride,
                                                const float* __restrict__ xb, int32_t H, double (&acc)[1]) {
  const float* hot = g_hot_lds;
  const int32_t* __restrict__ col = a.col;
  const float* __restrict__ val = a.val;
  const int64_t ld = a.ld;
  for (; e + 3 * stride < e1; e += 4 * stride) {
    int32_t c[4];
    float v[4], x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      c[u] = col[e + u * stride];
      v[u] = val ? val[e + u * stride] : 1.0f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = hot_or_global(hot, xb, c[u], H, ld);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[0] = fma((double)v[u], (double)x[u], acc[0]);
  }
  for (; e < e1; e += stride) {
    const int32_t c = col[e];
    const float x = hot_or_global(hot, xb, c, H, ld);
    acc[0] = fma((double)val[e], (double)x, acc[0]);
  }
}

// Sub-group cooperative index loads (LF > 1).  The LF lanes of a sub-group
// walk the same nonzero sequence e, e+stride, ...; instead of every lane
// issuing a dword load of the same col/val entry (10 identical addresses per
// sub-group at F=40: the texture-address unit was ~70 % busy, PMC s11), lane
// fs loads element t0+fs and the sub-group shares the LF (col, val) pairs
// through ds_bpermute, which runs on the LDS pipe.  Same elements, same
// order as accumulate() -> bitwise-identical sums.  U = gathers in flight.
#ifndef WG_BCAST_U  // gathers in flight per lane on the widths whose LF is not a multiple of 5
#define WG_BCAST_U 4
#endif
template <int VEC, int U>
__device__ __forceinline__ void accumulate_bcast(const StepArgs& a, int32_t e, int32_t e1, int32_t stride,
                                                 const float* __restrict__ xb, double (&acc)[VEC], int fs,
                                                 int base) {
  const int LF = a.LF;
  const int64_t ld = a.ld;
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
        const int src = base + min(j + u, LF - 1);  // stays inside the sub-group
        c[u] = __shfl(myc, src, 64);
        v[u] = __shfl(myv, src, 64);
      }
      float x[U][VEC];
#ifdef WG_TIMING_PROBES
      // branch-free timing probes: probe_fold = 2^m folds every column into [0, 2^m) (an AND);
      // probe_h2 > 0: columns below it gather ONE aligned 128-B line (lanes 8, 9 repeat lanes
      // 0, 1's addresses); probe_h2 < 0: no gathers at all (x = the column id)
      if (a.probe_fold > 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] &= a.probe_fold - 1;
      }
      if (a.probe_h2 < 0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int q = 0; q < VEC; ++q) x[u][q] = (float)(c[u] + q);
      } else if (a.probe_h2 > 0) {
        const float* base = xb - fs * VEC;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool one = c[u] < a.probe_h2;
          const int64_t off = one ? (int64_t)c[u] * 32 + (fs & 7) * 4 : (int64_t)c[u] * ld + fs * VEC;
          if (j + u < cnt) load_vec<VEC>(base + off, x[u]);
        }
      } else
#endif
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j + u < cnt) load_vec<VEC>(xb + (int64_t)c[u] * ld, x[u]);  // no dummy gathers
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

// F == 1: each lane takes 4 consecutive nonzeros with one 16-B int4 / float4
// load of col / val (4x fewer index instructions through the texture-address
// unit).  Chunks are 4-aligned in the CSR (arrays padded by 4 entries), lane
// ns of the row's team takes chunks ns, ns+stride, ...; elements outside
// [e0, e1) are masked.  Different summation split than accumulate().
__device__ __forceinline__ void accumulate_vidx1(const StepArgs& a, int32_t e0, int32_t e1, int32_t ns,
                                                 int32_t stride, const float* __restrict__ xb, double (&acc)[1]) {
  const int64_t ld = a.ld;
  const int32_t eb = e0 & ~3;
  for (int32_t q = eb + 4 * ns; q < e1; q += 4 * stride) {
    const int4 c = *reinterpret_cast<const int4*>(a.col + q);
    const float4 v = a.val ? *reinterpret_cast<const float4*>(a.val + q) : make_float4(1.f, 1.f, 1.f, 1.f);
    const int32_t cc[4] = {c.x, c.y, c.z, c.w};
    const float vv[4] = {v.x, v.y, v.z, v.w};
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = (q + u >= e0) && (q + u < e1);
      x[u] = ok ? xb[(int64_t)cc[u] * ld] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = (q + u >= e0) && (q + u < e1);
      if (ok) acc[0] = fma((double)vv[u], (double)x[u], acc[0]);
    }
  }
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// Value-free gathers (unweighted graphs, u = b * dinv), VEC = 4, on the padded CSR: a sub-group
// walks the 4-entry chunks q, q + step, ... of its range [q, e1) (multiples of 4), CPT chunks per
// turn.  Each lane loads a chunk's four ids with ONE 16-B load (the sub-group's lanes share the
// address: no index broadcast), gathers its 16-B slice of each entry's row as a raw buffer load
// (pad ids return 0 without a memory request), sums the turn's slices in float32 pairs
// (v_pk_add_f32, a fixed tree) and adds that to the float64 accumulators.  The ids of the next PF
// turns are in flight while a turn's gathers are consumed: a turn's wait is ONE memory latency
// under load, and a wave's time is its turns x that latency (DESIGN.md 4.1, r04 timelines).
template <int CPT, int PF>
__device__ __forceinline__ void accumulate_u4(const StepArgs& a, int32_t q, int32_t e1, int32_t step, int fs,
                                              double (&acc)[4]) {
  if (q >= e1) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.xm1), 0,
                                                                      (int)a.u_bytes, 0x00020000);
  const uint32_t rb = (uint32_t)a.ld * 4u;
  const uint32_t lo = (uint32_t)fs * 16u;
  const int32_t* __restrict__ pc = a.pcol;
  const int32_t T = CPT * step;  // entries between a sub-group's turns
#ifdef WG_TIMING_PROBES
  const int32_t idmask = a.probe_fold < 0 ? 1023 : -1;  // probe: ids from one 4-KB window
#else
  constexpr int32_t idmask = -1;
#endif
  // the ids as raw buffer loads with the volatile bit (aux bit 31): the compiler may not sink a
  // volatile load to its use in the next turn (MachineSink did, serialising id and gather latency)
  const __amdgpu_buffer_rsrc_t rpc = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(pc), 0, 0x7fffffff,
                                                                       0x00020000);
  auto ld_ids = [&](int32_t qq, int4 (&id)[CPT]) {  // unconditional: pcol is padded by kPcolTail ids
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rpc, (uint32_t)((qq + c * step) & idmask) * 4u, 0,
                                                              (int)(1u << 31));
      id[c] = make_int4((int)v.x, (int)v.y, (int)v.z, (int)v.w);
    }
  };
  int4 ids[PF + 1][CPT];
#pragma unroll
  for (int t = 0; t <= PF; ++t) ld_ids(q + t * T, ids[t]);
  // one turn on id slot S: gathers, the next-but-PF turn's ids into the slot, the sums
  auto turn = [&](int4 (&id)[CPT]) -> bool {
    int32_t cc[4 * CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const bool ok = q + c * step < e1;
      cc[4 * c + 0] = ok ? id[c].x : kPadCol;
      cc[4 * c + 1] = ok ? id[c].y : kPadCol;
      cc[4 * c + 2] = ok ? id[c].z : kPadCol;
      cc[4 * c + 3] = ok ? id[c].w : kPadCol;
    }
#ifdef WG_TIMING_PROBES
    if (a.probe_fold > 0) {
#pragma unroll
      for (int u = 0; u < 4 * CPT; ++u) cc[u] = cc[u] == kPadCol ? kPadCol : (cc[u] & (a.probe_fold - 1));
    }
#endif
    u32x4_t x[4 * CPT];
#ifdef WG_TIMING_PROBES
    if (a.probe_h2 < 0) {
#pragma unroll
      for (int u = 0; u < 4 * CPT; ++u) x[u] = u32x4_t{(uint32_t)cc[u], 0u, 0u, 0u};
    } else
#endif
#pragma unroll
    for (int u = 0; u < 4 * CPT; ++u)
      x[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, __umul24((uint32_t)cc[u], rb) + lo, 0, 0);
    ld_ids(q + (PF + 1) * T, id);
    f32x2 l2[4 * CPT], h2[4 * CPT];
#pragma unroll
    for (int u = 0; u < 4 * CPT; ++u) {
      l2[u] = f32x2{__uint_as_float(x[u].x), __uint_as_float(x[u].y)};
      h2[u] = f32x2{__uint_as_float(x[u].z), __uint_as_float(x[u].w)};
    }
#pragma unroll
    for (int w = 1; w < 4 * CPT; w *= 2)  // fixed pairwise tree
#pragma unroll
      for (int u = 0; u + w < 4 * CPT; u += 2 * w) {
        l2[u] += l2[u + w];
        h2[u] += h2[u + w];
      }
    acc[0] += (double)l2[0].x;
    acc[1] += (double)l2[0].y;
    acc[2] += (double)h2[0].x;
    acc[3] += (double)h2[0].y;
    q += T;
    return q < e1;
  };
  for (;;) {
    if (!turn(ids[0])) break;
    if (!turn(ids[1])) break;
    if constexpr (PF >= 2) {
      if (!turn(ids[2])) break;
    }
  }
}

// A wave's sub-group g on SELL-ordered ids (Plan::sell, team.hip): chunk k (4 ids) of every
// sub-group of the wave at off + k G + g, so a turn's id read is one coalesced G x 16-B block for
// the wave instead of G scattered 16-B reads; every sub-group runs the wave's chunk count wm.y
// (shorter ones padded with kPadCol chunks: dropped loads, no masking), two chunks per turn and a
// single-chunk last turn when the count is odd; the next turn's ids are in flight during this
// turn's gathers.  float32 tree per turn, float64 accumulation (as accumulate_u4).
__device__ __forceinline__ void sum_turn(const u32x4_t* x, int n, double (&acc)[4]) {
  f32x2 l2[8], h2[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (u < n) {
      l2[u] = f32x2{__uint_as_float(x[u].x), __uint_as_float(x[u].y)};
      h2[u] = f32x2{__uint_as_float(x[u].z), __uint_as_float(x[u].w)};
    }
  }
#pragma unroll
  for (int w = 1; w < 8; w *= 2)
#pragma unroll
    for (int u = 0; u + w < 8; u += 2 * w) {
      if (u + w < n) {
        l2[u] += l2[u + w];
        h2[u] += h2[u + w];
      }
    }
  acc[0] += (double)l2[0].x;
  acc[1] += (double)l2[0].y;
  acc[2] += (double)h2[0].x;
  acc[3] += (double)h2[0].y;
}

// CPT: chunks per turn (2: a turn of 8 gathers, a single chunk last when the count is odd; 1:
// turns of 4 gathers and fewer live registers)
// FIRST: u_0 = X0 * dinv on the fly: each gathered 16-B slice x of caller row perm[c] becomes
// fl32(x * dinv[c]) (scale_rows' rounding, so the sums are the permute-in path's bit for bit); the
// chunk's 4 dinv values (32 B per chunk at twice its id offset) are loaded with its gathers
__device__ __forceinline__ void scale_chunk(const __amdgpu_buffer_rsrc_t& rd, uint32_t off, u32x4_t* x) {
  WG_DCHECK((uint64_t)off < 0x40000000ull, "first launch: dinv slot at byte %llu past 2^31", 2ull * off);
  const u32x4_t d01 = __builtin_amdgcn_raw_buffer_load_b128(rd, 2u * off, 0, 0);
  const u32x4_t d23 = __builtin_amdgcn_raw_buffer_load_b128(rd, 2u * off + 16u, 0, 0);
  const double d[4] = {__hiloint2double((int)d01.y, (int)d01.x), __hiloint2double((int)d01.w, (int)d01.z),
                       __hiloint2double((int)d23.y, (int)d23.x), __hiloint2double((int)d23.w, (int)d23.z)};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    x[u].x = __float_as_uint((float)((double)__uint_as_float(x[u].x) * d[u]));
    x[u].y = __float_as_uint((float)((double)__uint_as_float(x[u].y) * d[u]));
    x[u].z = __float_as_uint((float)((double)__uint_as_float(x[u].z) * d[u]));
    x[u].w = __float_as_uint((float)((double)__uint_as_float(x[u].w) * d[u]));
  }
}

template <int CPT = 2, bool FIRST = false>
__device__ __forceinline__ void accumulate_sell(const StepArgs& a, int2 wm, int G, int g, int fs, double (&acc)[4]) {
  if (wm.y <= 0) return;
  const __amdgpu_buffer_rsrc_t rd =  // FIRST only (unused otherwise)
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.sdinv), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.xm1), 0,
                                                                      (int)a.u_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc(const_cast<int4*>(a.sell), 0, 0x7fffffff,
                                                                      0x00020000);
  const uint32_t rb = (uint32_t)a.ld * 4u;
  const uint32_t lo = (uint32_t)fs * 16u;
  uint32_t off = ((uint32_t)wm.x + (uint32_t)g) * 16u;  // byte offset of this sub-group's chunk 0
  const uint32_t cstep = (uint32_t)G * 16u;                // next chunk of the same sub-group
  // volatile (aux bit 31): the next turn's ids are not sunk to their use (accumulate_u4)
  auto ld = [&](uint32_t o) {
    WG_DCHECK(a.dbg_sell_bytes == 0 || (uint64_t)o + 16u <= a.dbg_sell_bytes, "SELL id load at byte %u of %llu", o,
              (unsigned long long)a.dbg_sell_bytes);
    return __builtin_amdgcn_raw_buffer_load_b128(ri, o, 0, (int)(1u << 31));
  };
  auto gather = [&](uint32_t c) -> u32x4_t {
    WG_DCHECK(c == (uint32_t)kPadCol || (uint64_t)c * rb + lo + 16u <= a.u_bytes,
              "gathered column %u (row bytes %u, lane offset %u) past the %u-byte gathered vector", c, rb, lo, a.u_bytes);
#ifdef WG_TIMING_PROBES
    if (a.probe_fold > 0 && c != (uint32_t)kPadCol) c &= (uint32_t)(a.probe_fold - 1);
    if (a.probe_h2 == -1) return u32x4_t{c, 0u, 0u, 0u};
#endif
#ifdef WG_TIMING_PROBES
    if (a.coldnt > 0) {
      const uint32_t off = __umul24(c, rb) + lo;
      const bool cold = c >= (uint32_t)a.coldnt;
      const u32x4_t h = __builtin_amdgcn_raw_buffer_load_b128(rs, cold ? 0xFFFFFFF0u : off, 0, 0);
      const u32x4_t q = __builtin_amdgcn_raw_buffer_load_b128(rs, cold ? off : 0xFFFFFFF0u, 0, 2);
      return h | q;
    }
#endif
    return __builtin_amdgcn_raw_buffer_load_b128(rs, __umul24(c, rb) + lo, 0, 0);
  };
  if constexpr (CPT == 1) {
    u32x4_t c0 = ld(off);  // the array is padded past its last wave
    for (int t = 0; t < wm.y; ++t) {
      off += cstep;
      const u32x4_t n0 = ld(off);
      const uint32_t cc[4] = {c0.x, c0.y, c0.z, c0.w};
      u32x4_t x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = gather(cc[u]);
      if constexpr (FIRST) scale_chunk(rd, off - cstep, x);
      sum_turn(x, 4, acc);
      c0 = n0;
    }
    return;
  }
  const int pairs = wm.y >> 1;
  u32x4_t c0 = ld(off), c1 = ld(off + cstep);  // the array is padded past its last wave
  for (int t = 0; t < pairs; ++t) {
    off += 2 * cstep;
    const u32x4_t n0 = ld(off), n1 = ld(off + cstep);
    const uint32_t cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    u32x4_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = gather(cc[u]);
    if constexpr (FIRST) {
      scale_chunk(rd, off - 2 * cstep, x);
      scale_chunk(rd, off - cstep, x + 4);
    }
#ifdef WG_TIMING_PROBES
    if (a.probe_h2 == -6) {  // one more id-load instruction per turn (its cost through the address unit)
      const u32x4_t e = ld(off + 2 * cstep);
      asm volatile("" ::"v"(e.x));
    } else if (a.probe_h2 == -7) {  // one more gather instruction per turn (same line: an L1 hit)
      const u32x4_t e = gather(cc[7]);
      asm volatile("" ::"v"(e.x));
    }
#endif
    sum_turn(x, 8, acc);
    c0 = n0;
    c1 = n1;
  }
  if (wm.y & 1) {  // the last, single chunk
    const uint32_t cc[4] = {c0.x, c0.y, c0.z, c0.w};
    u32x4_t x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = gather(cc[u]);
    if constexpr (FIRST) scale_chunk(rd, off, x);
    sum_turn(x, 4, acc);
  }
}

template <int VEC, bool BCAST, bool HOT>
__device__ __forceinline__ void acc_range(const StepArgs& a, int32_t e, int32_t e1, int32_t stride,
                                          const float* __restrict__ xb, double (&acc)[VEC], int32_t H, int fs,
                                          int base) {
  if constexpr (HOT && VEC == 1) {
    accumulate_hot1(a, e, e1, stride, xb, H, acc);
  } else if constexpr (BCAST) {
    if (a.LF % 5 == 0) accumulate_bcast<VEC, 5>(a, e, e1, stride, xb, acc, fs, base);
    else accumulate_bcast<VEC, WG_BCAST_U>(a, e, e1, stride, xb, acc, fs, base);
  } else {
    accumulate<VEC>(a, e, e1, stride, xb, acc);
  }
}

}  // namespace wg
