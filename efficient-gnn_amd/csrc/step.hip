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
//  * Block mode (long rows): a 256-lane workgroup = 4G sub-groups splits the
//    row; sub-groups reduce by shuffles inside each wave, the 4 wave sums meet
//    in LDS behind one barrier.
//  * Split mode (hub rows longer than CH nonzeros): one workgroup per CH-nnz
//    chunk writes a float64 partial.  The last chunk to arrive finishes the row
//    in the same kernel (inkernel_combine = 1, the default): partials are sc1
//    (write-through) stores drained by every storing wave (s_waitcnt
//    vmcnt(0)), then one agent-scope atomic add per chunk on a
//    per-row counter (the completing arrival resets it to 0); the workgroup whose add completes the row reads every
//    chunk's partial with sc1 loads, in chunk order, and runs the epilogue.
//    This relies on gfx950's cache behaviour (sc1 stores write through to L2,
//    sc1 loads bypass the L1), the hand-off of MI355X_MICROARCH.md's table
//    row 1 -- not on HIP memory-model release/acquire ordering, which would
//    need an agent-scope release per chunk (buffer_wbl2 of an XCD L2 full of
//    the step's dirty lines: 1.3-2.2x slower for the whole step, DESIGN.md
//    4.1).  inkernel_combine = 0 runs a separate combine_kernel instead.
//  * The hybrid step (tiles.hip) runs this kernel over each row's tail
//    entries only (phase 4) and adds the dense blocks' float64 sums.
// Row sums accumulate in float64 (products of two float32 are exact).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "internal.h"

#include "step_dev.h"

namespace wg {
namespace {

// One work unit of the plan (a group of team rows, a block row or a split
// chunk) processed by one workgroup of NW waves.
// P4: 0 = the gather loops of acc_range; else the padded-CSR value-free loop accumulate_u4 with
// P4 / 10 chunks per turn and the ids of P4 % 10 turns ahead in flight
template <int VEC, bool BCAST, int NW, bool HOT, int P4 = 0>
__device__ __forceinline__ void unit_body(const StepArgs& a, const Seg* __restrict__ segs, int nseg, int32_t unit,
                                          int32_t H) {
  __shared__ double red[NW * 64 * VEC];
  int si = 0;
  for (int i = 1; i < nseg; ++i)
    if (unit >= segs[i].blk_begin) si = i;
  const Seg seg = segs[si];
  if (!((a.seg_mask >> si) & 1)) return;  // timing attribution only
#ifdef WG_TIMING_PROBES
  if (a.probe_h2 == -4) return;  // skeleton probe: the unit lookup alone
#endif
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int LF = a.LF;
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;

  if (seg.mode == 0) {
    // ---------------- team mode: LN sub-groups per row, G/LN rows per wave
    const int LN = seg.ln;
    const int TS = LF * LN;
    const int tpw = 64 / TS;
    const int team = lane / TS;
    const int tl = lane - team * TS;
    const int ns = tl / LF;
    const int fs = tl - ns * LF;
    const int64_t row = (int64_t)seg.begin + (int64_t)(unit - seg.blk_begin) * (NW * tpw) + wave * tpw + team;
    const bool active = team < tpw && row < seg.end;
    EpiIn<VEC> in;
#ifdef WG_TIMING_PROBES
    if (a.probe_h2 == -3) {  // skeleton probe: no row work at all, one store per row
      float* dst = a.xk ? a.xk : a.S;  // the final step stores S (xk is null there)
      if (active && ns == 0 && dst) store_vec<VEC>(dst + row * a.ld + fs * VEC, acc);
      return;
    }
#endif
    if (active) {
      if (ns == 0) epi_prefetch<VEC>(a, row, fs, in);
#ifdef WG_TIMING_PROBES
      if (a.probe_h2 == -2) {  // skeleton probe: no ids or gathers (the row pointers, epilogue kept)
        acc[0] += (double)(a.prp[row + 1] - a.prp[row]);
      } else
#endif
      if constexpr (P4 && VEC == 4) {  // padded CSR: the row's 4-entry chunks ns, ns + LN, ...
        if (a.sell)  // the same chunks in the wave's SELL order (one coalesced id read per turn)
          accumulate_sell(a, a.wmeta[(int64_t)unit * NW + wave], 64 / LF, lane / LF, fs, acc);
        else
          accumulate_u4<P4 / 10, P4 % 10>(a, a.prp[row] + 4 * ns, a.prp[row + 1], 4 * LN, fs, acc);
      } else {
      int32_t e0 = a.rowptr[row], e1 = a.rowptr[row + 1];
      phase_range(a, row, e0, e1);
      if constexpr (VEC == 1 && !HOT) {
        if (a.vidx && LF == 1) accumulate_vidx1(a, e0, e1, ns, LN, a.xm1, acc);
        else acc_range<VEC, BCAST, HOT>(a, e0 + ns, e1, LN, a.xm1 + fs * VEC, acc, H, fs, lane - fs);
      } else {
        acc_range<VEC, BCAST, HOT>(a, e0 + ns, e1, LN, a.xm1 + fs * VEC, acc, H, fs, lane - fs);
      }
      }
    }
    reduce_subgroups<VEC>(acc, LN, LF, team * TS, fs);
    if (active && ns == 0) {
      part_add<VEC>(a, row, fs, acc);
      step_epilogue<VEC>(a, row, fs, acc, in, team * TS);
    }
    return;
  }

  // ---------------- workgroup modes: 4 waves x G sub-groups on one nnz range
  //   mode 1: a whole row (then the epilogue)
  //   mode 2: one chunk of a split row (then a float64 partial; finished by combine_kernel)
  int64_t row;
  int32_t e0, e1, cid = 0;
  if (seg.mode == 1) {
    row = (int64_t)seg.begin + (unit - seg.blk_begin);
    e0 = a.rowptr[row];
    e1 = a.rowptr[row + 1];
  } else {
    cid = seg.begin + (int32_t)(unit - seg.blk_begin);
    const ChunkDesc d = a.chunks[cid];
    row = d.row;
    e0 = d.e0;
    e1 = d.e1;
  }
  phase_range(a, row, e0, e1);
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  EpiIn<VEC> in;
  if (seg.mode == 1 && threadIdx.x < LF) epi_prefetch<VEC>(a, row, threadIdx.x, in);
  if constexpr (P4 && VEC == 4) {
    // padded CSR: a split chunk's range maps to the same offsets in the padded row (pads only at
    // its end; chunk lengths are multiples of 4); the workgroup's sub-groups deal its 4-entry chunks
    const int32_t pr0 = a.prp[row];
    const int32_t q0 = pr0 + (e0 - a.rowptr[row]);
    const int32_t q1 = (e1 == a.rowptr[row + 1]) ? a.prp[row + 1] : pr0 + (e1 - a.rowptr[row]);
    if (sg < G) accumulate_u4<P4 / 10, P4 % 10>(a, q0 + 4 * (wave * G + sg), q1, 4 * NW * G, fs, acc);
  } else if constexpr (VEC == 1 && !HOT) {
    if (a.vidx && LF == 1) {
      // chunk-aligned ranges: for split chunks e0 is a multiple of CH (>= 4) from the row start, so
      // neighbouring chunks never both take an aligned 4-group (masking keeps the bounds exact anyway)
      accumulate_vidx1(a, e0, e1, wave * G + sg, NW * G, a.xm1, acc);
    } else if (sg < G) {
      acc_range<VEC, BCAST, HOT>(a, e0 + wave * G + sg, e1, NW * G, a.xm1 + fs * VEC, acc, H, fs, lane - fs);
    }
  } else if (sg < G) {
    acc_range<VEC, BCAST, HOT>(a, e0 + wave * G + sg, e1, NW * G, a.xm1 + fs * VEC, acc, H, fs, lane - fs);
  }
  reduce_subgroups<VEC>(acc, G, LF, 0, fs);
  if (lane < LF) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) red[(wave * LF + lane) * VEC + j] = acc[j];
  }
  __syncthreads();
  if (threadIdx.x < LF) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = red[t * VEC + j];
#pragma unroll 1
    for (int w = 1; w < NW; ++w) {  // fixed wave order
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += red[(w * LF + t) * VEC + j];
    }
    if (seg.mode == 1) {
      part_add<VEC>(a, row, t, acc);
      step_epilogue<VEC>(a, row, t, acc, in, 0);
    } else {
      double* p = a.partial + (int64_t)cid * (LF * VEC) + t * VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        if (a.arrivals) __hip_atomic_store(p + j, acc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
        else p[j] = acc[j];
      }
    }
  }
  if (seg.mode == 2 && a.arrivals) {
    // In-kernel combine of a split row, fence-free (MI355X_MICROARCH.md, hand-off table row 1):
    // the partials are sc1 (write-through) stores drained by every storing wave, then ONE
    // agent-scope atomic per chunk; the workgroup whose add completes the row reads every
    // chunk's partial with sc1 loads, in chunk order (deterministic), after a barrier.
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int2 rc = a.rowchunks[row];
    if (threadIdx.x == 0) {
      // the arrival that completes the row resets its counter (uint32, equality: no history)
      const uint32_t old = __hip_atomic_fetch_add(a.arrivals + row, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old + 1u == (uint32_t)rc.y;
      if (s_last) __hip_atomic_store(a.arrivals + row, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_last && threadIdx.x < LF) {
      const int t = threadIdx.x;
      EpiIn<VEC> in2;
      epi_prefetch<VEC>(a, row, t, in2);
      double sum[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) sum[j] = 0.0;
      for (int q = 0; q < rc.y; ++q) {
        const double* pp = a.partial + (int64_t)(rc.x + q) * (LF * VEC) + t * VEC;
#pragma unroll
        for (int j = 0; j < VEC; ++j) sum[j] += __hip_atomic_load(pp + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      part_add<VEC>(a, row, t, sum);
      step_epilogue<VEC>(a, row, t, sum, in2, 0);
    }
  }
}

// the padded-CSR step held to 8 waves per SIMD (64 VGPRs; timing variant, gather4 = 121)
template <int NW, int P4>
__global__ __launch_bounds__(NW * 64, 8) void cheb_step_occ_kernel(StepArgs a, const Seg* __restrict__ segs, int nseg) {
  unit_body<4, false, NW, false, P4>(a, segs, nseg, (int32_t)blockIdx.x, 0);
}

template <int VEC, bool BCAST, int NW, int P4 = 0>
__global__ __launch_bounds__(NW * 64) void cheb_step_kernel(StepArgs a, const Seg* __restrict__ segs, int nseg) {
  // units are dealt to the 8 XCDs round-robin (blockIdx order): the units are in descending row
  // length, so an XCD-contiguous order gave one XCD every hub row (3x slower, r02_s65)
#ifdef WG_TIMING_PROBES
  const unsigned long long r0 = wall_clock64(), c0 = clock64();
#endif
  unit_body<VEC, BCAST, NW, false, P4>(a, segs, nseg, (int32_t)blockIdx.x, 0);
#ifdef WG_TIMING_PROBES
  // timeline probe: per wave {block | wave << 24 | xcc << 28 | hw_id << 32, start, end (100 MHz wall
  // clock), shader cycles}
  if (a.trace && (threadIdx.x & 63) == 0) {
    const unsigned long long r1 = wall_clock64(), c1 = clock64();
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned long long* t = a.trace + ((size_t)blockIdx.x * NW + (threadIdx.x >> 6)) * 4;
    t[0] = (unsigned long long)blockIdx.x | ((unsigned long long)(threadIdx.x >> 6) << 24) |
           ((unsigned long long)(xcc & 15) << 28) | ((unsigned long long)hw << 32);
    t[1] = r0;
    t[2] = r1;
    t[3] = c1 - c0;
  }
#endif
}

// Persistent F == 1 variant: one workgroup per CU stages T_{k-1}[0, H) in LDS
// once, then walks the plan's work units round-robin.
template <int NW>
__global__ __launch_bounds__(NW * 64) void cheb_step_hot_kernel(StepArgs a, const Seg* __restrict__ segs, int nseg,
                                                                int32_t total_units, int32_t H) {
  for (int32_t i = threadIdx.x; i < H; i += NW * 64) g_hot_lds[i] = a.xm1[(int64_t)i * a.ld];
  __syncthreads();
  for (int32_t unit = blockIdx.x; unit < total_units; unit += gridDim.x) {
    unit_body<1, false, NW, true>(a, segs, nseg, unit, H);
    __syncthreads();  // the block-mode LDS partials are reused by the next unit
  }
}

// Split rows: sum each row's chunk partials in chunk order, then the epilogue.
// Sub-group of LF lanes per row.
template <int VEC>
__global__ __launch_bounds__(kBlock) void combine_kernel(StepArgs a, int32_t n_split, const int2* __restrict__ rowchunks,
                                                         int64_t row0) {
  const int lane = threadIdx.x & 63;
  const int LF = a.LF;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int64_t lr = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + sg;  // split row of the plan
  if (sg >= G || lr >= n_split) return;
  const int2 rc = rowchunks[lr];
  const int64_t row = row0 + lr;
  const int width = LF * VEC;
  EpiIn<VEC> in;
  epi_prefetch<VEC>(a, row, fs, in);
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;
  for (int q = 0; q < rc.y; ++q) {
    const double* p = a.partial + (int64_t)(rc.x + q) * width + fs * VEC;
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] += p[j];
  }
  part_add<VEC>(a, row, fs, acc);
  step_epilogue<VEC>(a, row, fs, acc, in, sg * LF);
}

// internal S -> caller-order S and H = S / (||S||_1 + 1e-8); team of LF lanes per row.
// Rows >= closed_from are purely isolated (T_k = (-1)^k X0): S = coef * X0
// with coef = sum_k (-1)^k alpha_k, read from the untouched T_0 rows.
template <int VEC>
__global__ __launch_bounds__(kBlock) void finalize_kernel(int64_t n, int64_t F, int64_t ldi, int LF,
                                                          const int32_t* __restrict__ perm,
                                                          const float* __restrict__ Sint, const float* __restrict__ X0int,
                                                          int64_t closed_from, double coef, float* __restrict__ S,
                                                          float* __restrict__ H) {
  const int lane = threadIdx.x & 63;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + sg;
  const bool active = sg < G && row < n;
  const bool closed = row >= closed_from;
  float x[VEC];
  double s[VEC];
  double part = 0.0;
  if (active) {
    load_vec<VEC>((closed ? X0int : Sint) + row * ldi + fs * VEC, x);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      s[j] = closed ? coef * (double)x[j] : (double)x[j];
      part += fabs(s[j]);
    }
  }
  double tot = 0.0;
  for (int q = 0; q < LF; ++q) tot += __shfl(part, sg * LF + q, 64);
  if (!active) return;
  const int64_t r = perm ? perm[row] : row;
  double h[VEC];
  const double den = tot + 1e-8;
#pragma unroll
  for (int j = 0; j < VEC; ++j) h[j] = s[j] / den;
  if (S) store_vec<VEC>(S + r * F + fs * VEC, s);
  if (H) store_vec<VEC>(H + r * F + fs * VEC, h);
}

// wide-F fallback (F > 64*VEC): wave per row.
__global__ __launch_bounds__(kBlock) void finalize_wide_kernel(int64_t n, int64_t F, int64_t ldi,
                                                               const int32_t* __restrict__ perm,
                                                               const float* __restrict__ Sint,
                                                               const float* __restrict__ X0int, int64_t closed_from,
                                                               double coef, float* __restrict__ S,
                                                               float* __restrict__ H) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const int64_t r = perm ? perm[row] : row;
  const bool closed = row >= closed_from;
  const float* src = closed ? X0int : Sint;
  const double c = closed ? coef : 1.0;
  double part = 0.0;
  for (int64_t f = lane; f < F; f += 64) part += fabs(c * (double)src[row * ldi + f]);
  for (int off = 32; off >= 1; off >>= 1) part += __shfl_xor(part, off, 64);
  const double den = part + 1e-8;
  for (int64_t f = lane; f < F; f += 64) {
    const double s = c * (double)src[row * ldi + f];
    if (S) S[r * F + f] = (float)s;
    if (H) H[r * F + f] = (float)(s / den);
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

// Permute-in with the closed-form rows finished on the spot (finalize fused
// into the chain): internal rows < closed_from get T_0 = X0 (internal order);
// purely isolated rows >= closed_from never enter the chain, so their
// S = coef * X0 and H = S / (|S|_1 + 1e-8) are written to the caller's row
// directly (the finalize_kernel arithmetic, same order of the row sum).
// RG row groups per wave, their row ids and X0 rows loaded before any is used (the pass is
// latency-bound: one group per wave left each wave a dependent perm -> X0 -> store chain)
template <int VEC, int RG>
__global__ __launch_bounds__(kBlock) void permute_in_closed_kernel(int64_t n, int64_t F, int LF,
                                                                   const int32_t* __restrict__ perm,
                                                                   const float* __restrict__ src,
                                                                   float* __restrict__ dst, int64_t closed_from,
                                                                   double coef, float* __restrict__ S,
                                                                   float* __restrict__ H, const double* __restrict__ dinv,
                                                                   float* __restrict__ u, int64_t u_rows,
                                                                   float* __restrict__ zero) {
  const int lane = threadIdx.x & 63;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  int64_t rows[RG], rs[RG];
  bool act[RG];
  float x[RG][VEC];
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    rows[g] = (wave * RG + g) * G + sg;
    act[g] = sg < G && rows[g] < n;
    rs[g] = act[g] ? perm[rows[g]] : 0;
  }
#pragma unroll
  for (int g = 0; g < RG; ++g)
    if (act[g]) load_vec<VEC>(src + rs[g] * F + fs * VEC, x[g]);
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int64_t row = rows[g], r = rs[g];
    const bool active = act[g];
    const bool closed = row >= closed_from;
    double sv[VEC];
    double part = 0.0;
    if (active) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        sv[j] = closed ? coef * (double)x[g][j] : (double)x[g][j];
        part += fabs(sv[j]);
      }
      if (!closed) {
        if (dst) store_vec<VEC>(dst + row * F + fs * VEC, sv);  // (fold 2: u_0 only)
        if (u) {  // u_0 = X0 * dinv for the first value-free step (scale_rows_kernel's rounding)
          const double di = dinv[row];
          double uv[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) uv[j] = (double)x[g][j] * di;
          store_vec<VEC>(u + row * F + fs * VEC, uv);
        }
      }
    }
    // closed rows are the internal tail: most groups hold none and skip the row sums
    if (!__ballot(active && closed)) continue;
    double tot = 0.0;
    for (int q = 0; q < LF; ++q) tot += __shfl(part, sg * LF + q, 64);
    if (!active || !closed) continue;
    const double den = tot + 1e-8;
    double h[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) h[j] = sv[j] / den;
    store_vec<VEC>(S + r * F + fs * VEC, sv);
    store_vec<VEC>(H + r * F + fs * VEC, h);
    // a row shard's exchange slots (dist.hip): the closed rows' u rows zero in both slots (the
    // hybrid step's dense tiles stage whole 32-row column tiles: 0 x stale must not enter a sum)
    const double z[VEC] = {};
    if (u && row < u_rows) store_vec<VEC>(u + row * F + fs * VEC, z);
    if (zero) store_vec<VEC>(zero + row * F + fs * VEC, z);
  }
}

// caller rows (stride F) -> internal rows (stride Fp > F), the Fp - F pad columns zeroed
__global__ void permute_pad_kernel(int64_t n, int64_t F, int64_t Fp, const int32_t* __restrict__ perm,
                                   const float* __restrict__ src, float* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * Fp) return;
  const int64_t i = idx / Fp;
  const int64_t f = idx - i * Fp;
  dst[idx] = f < F ? src[(int64_t)perm[i] * F + f] : 0.0f;
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

// the hybrid step with its tail beside the dense blocks (tuning key hyb_conc): each row's tail sums
// (a.tsum, written by the team kernel on the second stream) + its dense blocks' sums (part_add) and the
// epilogue the tail pass would have run; LF lanes per row, G rows per wave
__global__ __launch_bounds__(kBlock) void hybrid_epilogue_kernel(StepArgs a, int64_t n_rows) {
  const int lane = threadIdx.x & 63;
  const int LF = a.LF;
  const int G = 64 / LF;
  const int sg = lane / LF, fs = lane - sg * LF;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + sg;
  if (sg >= G || row >= n_rows) return;  // whole sub-groups: the H shuffle stays within a row's lanes
  EpiIn<4> in;
  epi_prefetch<4>(a, row, fs, in);
  const double* p = a.tsum + row * a.ld + fs * 4;
  const double2 s01 = *reinterpret_cast<const double2*>(p), s23 = *reinterpret_cast<const double2*>(p + 2);
  double acc[4] = {s01.x, s01.y, s23.x, s23.y};
  part_add<4>(a, row, fs, acc);
  step_epilogue<4>(a, row, fs, acc, in, sg * LF);
}

// smallest divisor of G that is >= want (G itself if none smaller)
int divisor_at_least(int G, int64_t want) {
  for (int d = 1; d <= G; ++d)
    if (G % d == 0 && d >= want) return d;
  return G;
}

template <int VEC, int NW>
void launch_main(const Plan& plan, const StepArgs& a, hipStream_t stream) {
  const dim3 grid(plan.tab.total_blocks), block(NW * 64);
  if constexpr (VEC == 4) {
    if (a.pcol) {  // a.p4v: the padded-CSR loop variant (gather4 tuning value)
      const Seg* sg = plan.d_segs;
      switch (a.p4v) {
        case 121: hipLaunchKernelGGL((cheb_step_occ_kernel<NW, 21>), grid, block, 0, stream, a, sg, plan.tab.n); break;
        case 31: hipLaunchKernelGGL((cheb_step_kernel<4, false, NW, 31>), grid, block, 0, stream, a, sg, plan.tab.n); break;
        case 22: hipLaunchKernelGGL((cheb_step_kernel<4, false, NW, 22>), grid, block, 0, stream, a, sg, plan.tab.n); break;
        case 41: hipLaunchKernelGGL((cheb_step_kernel<4, false, NW, 41>), grid, block, 0, stream, a, sg, plan.tab.n); break;
        default: hipLaunchKernelGGL((cheb_step_kernel<4, false, NW, 21>), grid, block, 0, stream, a, sg, plan.tab.n);
      }
      return;
    }
  }
  if (a.bcast && a.LF > 1)
    hipLaunchKernelGGL((cheb_step_kernel<VEC, true, NW>), grid, block, 0, stream, a, (const Seg*)plan.d_segs,
                       plan.tab.n);
  else
    hipLaunchKernelGGL((cheb_step_kernel<VEC, false, NW>), grid, block, 0, stream, a, (const Seg*)plan.d_segs,
                       plan.tab.n);
}

template <int NW>
int launch_hot(const Plan& plan, const StepArgs& a, hipStream_t stream) {
  int dev = 0;
  WG_HIP_TRY(hipGetDevice(&dev));
  const int n_cu = n_cus(dev);
  const size_t lds = (size_t)plan.hot * sizeof(float);
  if (int rc = ensure_dyn_lds((const void*)cheb_step_hot_kernel<NW>, 160 * 1024 - NW * 64 * 8)) return rc;
  const int grid = std::min<int>(plan.tab.total_blocks, n_cu);
  hipLaunchKernelGGL(cheb_step_hot_kernel<NW>, dim3(grid), dim3(NW * 64), lds, stream, a, (const Seg*)plan.d_segs,
                     plan.tab.n, plan.tab.total_blocks, plan.hot);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

template <int VEC>
int launch_step_vec(const Plan& plan, const StepArgs& a, hipStream_t stream) {
  const SegTable& tab = plan.tab;
  if (VEC == 1 && plan.hot > 0 && tab.total_blocks > 0 && a.phase == 0) {
    int rc = plan.nw == 16 ? launch_hot<16>(plan, a, stream) : launch_hot<4>(plan, a, stream);
    if (rc) return rc;
  } else if (tab.total_blocks > 0) {
    if (plan.nw == 16) launch_main<VEC, 16>(plan, a, stream);
    else if (plan.nw == 8) launch_main<VEC, 8>(plan, a, stream);
    else launch_main<VEC, 4>(plan, a, stream);
    WG_LAUNCH_CHECK();
  }
  if (plan.n_split > 0 && !a.arrivals && ((a.seg_mask >> tab.n) & 1)) {
    const int G = 64 / a.LF;
    hipLaunchKernelGGL(combine_kernel<VEC>, dim3((unsigned)ceil_div(plan.n_split, 4 * G)), dim3(kBlock), 0, stream, a,
                       plan.n_split, plan.rowchunks, plan.row0);
    WG_LAUNCH_CHECK();
  }
  return WG_OK;
}

}  // namespace

namespace {
int upload_segs(Plan& p) {
  int rc = dmalloc(&p.d_segs, kMaxSeg);
  if (rc) return rc;
  WG_HIP_TRY(hipMemcpy(p.d_segs, p.tab.s, sizeof(Seg) * kMaxSeg, hipMemcpyHostToDevice));
  return WG_OK;
}
}  // namespace

void Plan::release() {
  team.release();
  (void)hipFree(wmeta);
  (void)hipFree(sell);
  wmeta = nullptr;
  sell = nullptr;
  (void)hipFree(d_segs);
  d_segs = nullptr;
  (void)hipFree(chunks);
  (void)hipFree(partial);
  (void)hipFree(rowchunks);
  (void)hipFree(arrivals);
  arrivals = nullptr;
  chunks = nullptr;
  partial = nullptr;
  rowchunks = nullptr;
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

// Defaults measured on MI355X (profiles/r01 sweeps): wide signals (G = 64/LF
// small, e.g. F = 40 -> G = 6) want long per-sub-group runs; F = 1 (G = 64)
// shorter ones.
// Wide tiles (F >= 16) on large graphs: one sub-group per row up to 192 entries per
// lane (ogbn-arxiv-size F=40: 41.8 vs 45.5 us per step with iter 96 vs 24; F=64 56.3
// vs 64.9; Reddit-size F=44 1732 vs 1817 us; with the value-free Clenshaw chain,
// s47-s49: 192 vs 96 -- arxiv F=40 37.3 vs 38.2, F=64 49.9 vs 51.8, Reddit-size F=44
// 1497 vs 1522; 256 jumps to 55 us) and long split-row chunks (Reddit-size
// F=44: 1625 us with chunk_iter 128 vs 1729 with 64) above 16 M nonzeros, 64 below
// (arxiv F=40 36.5 vs 37.1 us, F=64 neutral; profiles/r01/s55_chunk_sweep.log); small graphs
// keep more lanes per row for latency (PubMed-size F=40: 9.3 us with iter 24, 17.2
// with 96).  F = 1 from 1 M nonzeros: 8 entries per lane (ogbn-arxiv-size: 10.7 us per
// step vs 11.6 with 16, s34).
void default_knobs(const Tuning& t, int G, int64_t nnz, int* iter, int* block_iter, int* chunk_iter,
                   bool hybrid = false, int64_t rows = 0) {
  // the hybrid step's tail (~22 % of each row's entries) wants longer one-row
  // sub-groups and larger block / split units the more rows there are to fill the CUs with
  // (Reddit-size F=41, rows / (G x 256 CUs): 182 -> iter 6144: 784 vs 917 us per step with the
  // gather kernel's defaults; its 2-way shards (92) -> 1536: 415 vs 473; the 4-way shards (46)
  // keep the defaults: 1536 gives 232-234 vs 246-249 on three ranks but 312 vs 247 on the fourth
  // (a long-tailed row walked by one sub-group), the 8-way shards (23) 172 vs 156;
  // profiles/r02/s72-s76).  Only from 8 M nonzeros: on the arxiv-size graph (2.3 M, hub rows of
  // thousands of tail entries walked by one sub-group) the 1536 tier took 67.8 vs 38.6 us
  // (profiles/r03/s20-s21)
  const int64_t per_cu = rows / ((int64_t)G * 256);
  if (hybrid && per_cu >= 64 && nnz >= ((int64_t)8 << 20)) {
    const bool big = per_cu >= 128;
    *iter = t.iter > 0 ? t.iter : (big ? 6144 : 1536);
    *block_iter = t.block_iter > 0 ? t.block_iter : (big ? 4096 : 1024);
    *chunk_iter = t.chunk_iter > 0 ? t.chunk_iter : (big ? 4096 : 1024);
    return;
  }
  const bool wide = G <= 16;
  const bool big = nnz >= (int64_t)1 << 20;
  // from 8 M nonzeros: longer team runs and 256-iteration split-row chunks (Reddit-size F=41,
  // width 48: 1400 vs 1434 us per step; its 8-way shard, 14.3 M nonzeros: 195-200 vs 207-211
  // with the 1-16 M defaults, profiles/r02/s39-s40)
  const bool large = nnz >= (int64_t)1 << 23;
  *iter = t.iter > 0 ? t.iter : (wide ? (large ? 384 : big ? 192 : 24) : (G == 64 && big ? 8 : 16));
  *block_iter = t.block_iter > 0 ? t.block_iter : (wide ? 256 : 32);
  *chunk_iter = t.chunk_iter > 0 ? t.chunk_iter : (wide ? (large ? 256 : big ? 64 : 32) : 16);
}

// Build (once per tile shape) the segment table and the split-row chunk table.
//   team  rows: len <= G*iter              (LN sub-groups per row, LN | G)
//   block rows: len <= 4G*block_iter       (one workgroup per row)
//   split rows: longer                     (one workgroup per CH = 4G*chunk_iter nnz + combine_kernel)
// Classification is by power-of-two length bucket (rows are sorted by length).
int get_plan(wg_laplacian_s* L, int LF, int VEC, bool active_only, Plan** out, bool hybrid) {
  active_only = active_only && L->reordered;
  const int NW = (L->tune.waves == 16 || L->tune.waves == 8) ? L->tune.waves : 4;
  const int64_t key = (int64_t)(((LF * 8 + VEC) * 2 + (active_only ? 1 : 0)) * 32 + NW +
                                (L->tune.hot > 0 ? (1 << 28) : 0) + (hybrid ? (1 << 29) : 0));
  auto it = L->plans.find(key);
  if (it != L->plans.end()) {
    *out = &it->second;
    return WG_OK;
  }
  Plan p;
  p.width = LF * VEC;
  p.nw = NW;
  if (LF == 1 && VEC == 1 && L->tune.hot > 0)
    p.hot = (int32_t)std::min<int64_t>({(int64_t)L->tune.hot, L->n_cols, (int64_t)((160 * 1024 - NW * 64 * 8) / 4)});
  const int G = 64 / LF;
  const int64_t n = active_only ? L->n_active : L->n_rows;
  unsigned int bucket[kBuckets];
  const int64_t base = 0;  // first row of the plan
  for (int b = 0; b < kBuckets; ++b) bucket[b] = L->bucket[b];
  bucket[0] -= (unsigned int)(L->n_rows - n);  // closed-form rows: length 0, at the very end
  p.row0 = base;
  p.row1 = n;
  int iter, block_iter, chunk_iter;
  default_knobs(L->tune, G, L->nnz, &iter, &block_iter, &chunk_iter, hybrid, n);
  const int64_t team_max = (int64_t)G * iter;
  const int64_t block_max = (int64_t)NW * G * block_iter;
  const int64_t CH = (int64_t)NW * G * chunk_iter;
  SegTable& t = p.tab;
  char buf[256];
  if (!L->reordered) {
    // caller order: a single team segment sized by the average row length
    const int ln = divisor_at_least(G, ceil_div(std::max<int64_t>(1, L->avg_len), iter));
    const int tpw = G / ln;
    t.s[0] = Seg{0, (int32_t)n, 0, ln, 0};
    t.n = n > 0 ? 1 : 0;
    t.total_blocks = (int32_t)ceil_div(n, NW * tpw);
    snprintf(buf, sizeof(buf), "team rows[0,%lld) ln=%d (no reorder)\n", (long long)n, ln);
    p.text = buf;
    if (int rc2 = upload_segs(p)) return rc2;
    auto res = L->plans.emplace(key, p);
    *out = &res.first->second;
    return WG_OK;
  }
  int64_t n_split = 0, n_block = 0;
  for (int b = kBuckets - 1; b >= 0; --b) {
    const int64_t maxlen = (b == 0) ? 1 : (1ll << b);
    if (maxlen > block_max) n_split += bucket[b];
    else if (maxlen > team_max) n_block += bucket[b];
  }
  int nseg = 0;
  int32_t blk = 0;
  if (n_split > 0) {
    std::vector<int32_t> rp(n_split + 1);
    WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr + base, sizeof(int32_t) * (n_split + 1), hipMemcpyDeviceToHost));
    std::vector<ChunkDesc> ch;
    std::vector<int2> rc(n_split);
    for (int64_t r = 0; r < n_split; ++r) {
      const int64_t len = rp[r + 1] - rp[r];
      const int cnt = (int)std::max<int64_t>(1, ceil_div(len, CH));
      rc[r] = make_int2((int)ch.size(), cnt);
      for (int q = 0; q < cnt; ++q) {
        ChunkDesc d{};
        d.row = (int32_t)(base + r);
        d.e0 = (int32_t)(rp[r] + q * CH);
        d.e1 = (int32_t)std::min<int64_t>(rp[r + 1], rp[r] + (q + 1) * CH);
        ch.push_back(d);
      }
    }
    p.n_chunks = (int32_t)ch.size();
    p.n_split = (int32_t)n_split;
    int rc_ = dmalloc(&p.chunks, ch.size());
    if (!rc_) rc_ = dmalloc(&p.partial, ch.size() * (size_t)p.width);
    if (!rc_) rc_ = dmalloc(&p.rowchunks, rc.size());
    if (!rc_) rc_ = dmalloc(&p.arrivals, rc.size());
    if (!rc_ && hipMemset(p.arrivals, 0, sizeof(uint32_t) * rc.size()) != hipSuccess) rc_ = WG_ERR_HIP;
    if (rc_) {
      p.release();
      return rc_;
    }
    WG_HIP_TRY(hipMemcpy(p.chunks, ch.data(), sizeof(ChunkDesc) * ch.size(), hipMemcpyHostToDevice));
    WG_HIP_TRY(hipMemcpy(p.rowchunks, rc.data(), sizeof(int2) * rc.size(), hipMemcpyHostToDevice));
    t.s[nseg++] = Seg{0, p.n_chunks, 0, G, 2};
    blk = p.n_chunks;
    snprintf(buf, sizeof(buf), "split rows[%lld,%lld) chunks=%d CH=%lld (+combine)\n", (long long)base,
             (long long)(base + n_split), p.n_chunks, (long long)CH);
    p.text += buf;
  }
  if (n_block > 0) {
    t.s[nseg++] = Seg{(int32_t)(base + n_split), (int32_t)(base + n_split + n_block), blk, G, 1};
    blk += (int32_t)n_block;
    snprintf(buf, sizeof(buf), "block rows[%lld,%lld) (workgroup per row)\n", (long long)(base + n_split),
             (long long)(base + n_split + n_block));
    p.text += buf;
  }
  int32_t row = (int32_t)(base + n_split + n_block);
  const int first_team = nseg;
  for (int b = kBuckets - 1; b >= 0; --b) {
    const int32_t cnt = (int32_t)bucket[b];
    const int64_t maxlen = (b == 0) ? 1 : (1ll << b);
    if (!cnt || maxlen > team_max) continue;
    int ln = divisor_at_least(G, ceil_div(maxlen, iter));
    Seg* last = nseg > first_team ? &t.s[nseg - 1] : nullptr;
    if (last && (last->ln == ln || nseg == kMaxSeg)) {
      if (last->ln != ln) ln = last->ln;  // out of slots: extend
      last->end = row + cnt;
      blk = last->blk_begin + (int32_t)ceil_div(last->end - last->begin, NW * (G / ln));
    } else {
      t.s[nseg++] = Seg{row, row + cnt, blk, ln, 0};
      blk += (int32_t)ceil_div(cnt, NW * (G / ln));
    }
    row += cnt;
  }
  t.n = nseg;
  t.total_blocks = blk;
  for (int i = first_team; i < nseg; ++i) {
    snprintf(buf, sizeof(buf), "team rows[%d,%d) ln=%d blocks=%d\n", t.s[i].begin, t.s[i].end, t.s[i].ln,
             (i + 1 < nseg ? t.s[i + 1].blk_begin : blk) - t.s[i].blk_begin);
    p.text += buf;
  }
  if (int rc2 = upload_segs(p)) {
    p.release();
    return rc2;
  }
  auto res = L->plans.emplace(key, p);
  *out = &res.first->second;
  return WG_OK;
}

// Profiling: a pair of timing-only events around every step launch (both
// kernels of a split step).  hipEventDisableSystemFence: no system-scope
// release (cache write-back / invalidate) -- the events must not perturb the
// kernels they time.
int prof_mark(wg_laplacian_s* L, hipStream_t stream, bool start) {
  if (!L->prof) return WG_OK;
  if (start) {
    while (L->ev.size() < L->ev_used + 2) {
      hipEvent_t e;
      WG_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
      L->ev.push_back(e);
    }
    WG_HIP_TRY(hipEventRecord(L->ev[L->ev_used], stream));
  } else {
    WG_HIP_TRY(hipEventRecord(L->ev[L->ev_used + 1], stream));
    L->ev_used += 2;
  }
  return WG_OK;
}

// The padded CSR of the value-free VEC-4 gathers (accumulate_u4): every row's column ids padded
// to a multiple of 4 with kPadCol, row pointers prp, kPcolTail pad ids after the last row.  Built
// once per handle (host pass over the operator's CSR).
bool gather4_applies(const wg_laplacian_s* L, int64_t F) {
  return L->tune.gather4 && !L->tune.probe && L->tune.hot == 0 && F % 4 == 0 && F * 4 <= 256 &&
         F <= 64 * 4 && L->n_cols < kPadCol;
}

int build_pcol(wg_laplacian_s* L) {
  if (L->pcol) return WG_OK;
  const int64_t n = L->n_rows;
  std::vector<int32_t> rp(n + 1);
  WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  std::vector<int32_t> col(std::max<int64_t>(rp[n], 1));
  if (rp[n]) WG_HIP_TRY(hipMemcpy(col.data(), L->col, sizeof(int32_t) * rp[n], hipMemcpyDeviceToHost));
  std::vector<int32_t> prp(n + 1);
  prp[0] = 0;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t len = rp[r + 1] - rp[r];
    const int64_t padded = prp[r] + (len + 3) / 4 * 4;
    if (padded > INT32_MAX - kPcolTail) return fail(WG_ERR_INVALID, "build_pcol: padded CSR exceeds int32");
    prp[r + 1] = (int32_t)padded;
  }
  std::vector<int32_t> pc((size_t)prp[n] + kPcolTail, kPadCol);
  for (int64_t r = 0; r < n; ++r)
    std::copy(col.begin() + rp[r], col.begin() + rp[r + 1], pc.begin() + prp[r]);
  int32_t *dprp = nullptr, *dpc = nullptr;
  if (int rc = dmalloc(&dprp, prp.size())) return rc;
  if (int rc = dmalloc(&dpc, pc.size())) {
    (void)hipFree(dprp);
    return rc;
  }
  WG_HIP_TRY(hipMemcpy(dprp, prp.data(), sizeof(int32_t) * prp.size(), hipMemcpyHostToDevice));
  WG_HIP_TRY(hipMemcpy(dpc, pc.data(), sizeof(int32_t) * pc.size(), hipMemcpyHostToDevice));
  L->prp = dprp;
  L->pcol = dpc;
  return WG_OK;
}

// The SELL order of a plan's value-free team waves (accumulate_sell): for wave w = unit * NW + wave
// of a team segment, sub-group g (row begin + (unit - blk_begin) NW tpw + wave tpw + g / LN, share
// ns = g % LN of the row's 4-entry chunks: ns, ns + LN, ...), its k-th chunk at
// sell[wmeta[w].x + k G + g] with k = 2 t + c; every sub-group padded with kPadCol chunks to the
// wave's turn count wmeta[w].y (2 chunks per turn), plus 2 turns of pads after the last wave.
int build_sell(wg_laplacian_s* L, Plan* p, int LF) {
  if (p->sell) return WG_OK;
  const int G = 64 / LF;
  const int NW = p->nw;
  const int64_t n = L->n_rows;
  std::vector<int32_t> rp(n + 1);
  WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  std::vector<int32_t> col(std::max<int64_t>(rp[n], 1));
  if (rp[n]) WG_HIP_TRY(hipMemcpy(col.data(), L->col, sizeof(int32_t) * rp[n], hipMemcpyDeviceToHost));
  std::vector<int2> wm((size_t)p->tab.total_blocks * NW, int2{0, 0});
  std::vector<int4> sell;
  const int4 pad4{kPadCol, kPadCol, kPadCol, kPadCol};
  for (int si = 0; si < p->tab.n; ++si) {
    const Seg& sg = p->tab.s[si];
    if (sg.mode != 0) continue;
    const int LN = sg.ln, tpw = G / LN;
    const int32_t nblk = (si + 1 < p->tab.n ? p->tab.s[si + 1].blk_begin : p->tab.total_blocks) - sg.blk_begin;
    for (int32_t u = 0; u < nblk; ++u) {
      for (int w = 0; w < NW; ++w) {
        const int64_t r0 = (int64_t)sg.begin + (int64_t)u * NW * tpw + (int64_t)w * tpw;
        int64_t turns = 0;
        for (int g = 0; g < G; ++g) {  // the wave's longest sub-group
          const int64_t r = r0 + g / LN, ns = g % LN;
          if (g / LN >= tpw || r >= sg.end) continue;
          const int64_t nch = (rp[r + 1] - rp[r] + 3) / 4;
          const int64_t mine = ns < nch ? (nch - ns + LN - 1) / LN : 0;
          turns = std::max<int64_t>(turns, (mine + 1) / 2);
        }
        const size_t wi = (size_t)(sg.blk_begin + u) * NW + w;
        if (sell.size() + (size_t)(2 * G * (turns + 2)) >= ((size_t)1 << 27))  // 16-B chunks at 32-bit byte offsets
          return fail(WG_ERR_UNSUPPORTED, "build_sell: id array exceeds 2 GB (tuning key sell = 0)");
        wm[wi] = int2{(int)sell.size(), (int)(2 * turns)};  // chunk count (accumulate_sell)
        const size_t base = sell.size();
        sell.resize(base + (size_t)2 * turns * G, pad4);
        for (int g = 0; g < G; ++g) {
          const int64_t r = r0 + g / LN, ns = g % LN;
          if (g / LN >= tpw || r >= sg.end) continue;
          const int64_t len = rp[r + 1] - rp[r];
          const int64_t nch = (len + 3) / 4;
          for (int64_t k = 0; ns + k * LN < nch; ++k) {
            const int64_t ch = ns + k * LN;
            int32_t id[4];
            for (int i = 0; i < 4; ++i) id[i] = ch * 4 + i < len ? col[rp[r] + ch * 4 + i] : kPadCol;
            sell[base + (size_t)k * G + g] = int4{id[0], id[1], id[2], id[3]};
          }
        }
      }
    }
  }
  sell.resize(sell.size() + (size_t)4 * G, pad4);  // the next-turn id reads past the last wave
  auto undo = [&](int rc) {  // no half-built table: the next call builds both arrays again
    (void)hipFree(p->wmeta);
    (void)hipFree(p->sell);
    p->wmeta = nullptr;
    p->sell = nullptr;
    return rc;
  };
  if (int rc = dmalloc(&p->wmeta, wm.size())) return undo(rc);
  if (int rc = dmalloc(&p->sell, sell.size())) return undo(rc);
  if (hipMemcpy(p->wmeta, wm.data(), sizeof(int2) * wm.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(p->sell, sell.data(), sizeof(int4) * sell.size(), hipMemcpyHostToDevice) != hipSuccess)
    return undo(fail(WG_ERR_HIP, "build_sell: upload failed"));
  return WG_OK;
}

int launch_step(wg_laplacian_s* L, int32_t k, int64_t F, const float* xm1, const float* xm2, float* xk, float* S,
                float* H, double alpha0, double alpha_k, hipStream_t stream, bool active_only, float* S_out,
                const ClenArgs* cl) {
  if (L->n_rows == 0) return WG_OK;
  if (int rc = prof_mark(L, stream, true)) return rc;
  const int vec = pick_vec(F, {xm1, xm2, xk, S, H, S_out});
  int64_t max_tile = 64 * (int64_t)vec;  // LF <= 64
  if (L->tune.tile_f > 0) max_tile = std::max<int64_t>(vec, std::min<int64_t>(max_tile, L->tune.tile_f / vec * vec));
  const bool fuse_h = (H != nullptr) && F <= max_tile;
  if (S_out && !(fuse_h && S)) return fail(WG_ERR_INVALID, "launch_step: fused finalize needs one tile and S");
  // hyb: the hybrid step's tail pass (phase 4 over the tail-first columns, + the blocks' sums)
  // conc (hyb_conc): the hybrid tail's sums go to L->tsum on the second stream; its arguments are kept
  // for the epilogue pass (hybrid_epilogue_kernel) that follows the join
  StepArgs conc_args{}, conc_fused{};
  int64_t conc_rows = -1;
  const TeamPlan* conc_team = nullptr;
  // defer: build the tail's plan and arguments (conc_fused, conc_team) without launching (the fused launch)
  auto tiles_loop = [&](const TilePlan* hyb, hipStream_t tail_stream = nullptr, double* tsum = nullptr,
                        bool defer = false) -> int {
    if (!tail_stream) tail_stream = stream;
    for (int64_t f0 = 0; f0 < F; f0 += max_tile) {
      const int64_t fw = std::min<int64_t>(max_tile, F - f0);
      const int LF = (int)(fw / vec);
      Plan* plan = nullptr;
      if (int rc = get_plan(L, LF, vec, active_only, &plan, /*hybrid=*/hyb != nullptr)) return rc;
      int rc = WG_OK;
      StepArgs a{};
      a.rowptr = L->rowptr;
      a.col = hyb ? hyb->tcol : L->col;
      a.val = L->val;
      a.iso = L->iso;
      a.xm1 = xm1 + f0;
      a.xm2 = xm2 ? xm2 + f0 : nullptr;
      a.xk = xk ? xk + f0 : nullptr;
      a.S = S ? S + f0 : nullptr;
      a.H = fuse_h ? H + f0 : nullptr;
      a.out_perm = S_out ? L->perm : nullptr;
      a.S_out = S_out;
      a.ld = F;
      a.LF = LF;
      a.k = k;
      a.alpha0 = alpha0;
      a.alpha_k = alpha_k;
      if (cl) {  // Clenshaw: the generic (k >= 2) paths, S written only by the final step
        a.k = 2;
        a.clen = cl->final_ ? 2 : 1;
        a.x0 = cl->x0 ? cl->x0 + f0 : nullptr;
        a.ck = cl->ck;
        a.cacc = cl->cacc;
        if (!cl->final_) a.S = nullptr;
        a.dinv = L->dinv;
        a.uin = cl->uin;
        a.uprev = cl->uprev;
        a.uout = cl->final_ ? 0 : cl->uout;
        if (a.uin) a.val = nullptr;  // unweighted: the gathered u needs no values
      }
      if (hyb) {
        a.phase = 4;
        a.rsplit = hyb->tsplit;
        a.part = hyb->part + f0;
      }
      a.nt = L->tune.nt >= 0 ? L->tune.nt : 8;  // store policy (below), for the team kernel too
      // value-free steps at VEC 4: every row as independent waves on SELL-ordered
      // padded ids (team.hip; the hybrid step's tail too), or the workgroup kernel on the padded CSR
      // (accumulate_u4 / accumulate_sell); all columns in one tile, rows addressable by 24-bit ids
      const bool g4 = vec == 4 && a.uin && F == fw && gather4_applies(L, F);
      // the hybrid step's tail on independent waves up to team_tail entries: larger tails keep the
      // workgroup kernel and its tiered plan (Reddit-size F = 41, width 48: 1 / 2 / 4 / 8-way shards
      // 798 / 411 / 224 / 133 us per step with the team tail vs 719 / 367 / 233 / 145; r04 s38), up to
      // twice that where the fused launch takes the step (tiles.hip hybrid_tail_on_team)
      const bool team_here = L->tune.team && (!hyb || hybrid_tail_on_team(L, hyb, F));
      const bool fold = cl && cl->x0c;  // the folded chain's first launch (team kernel only)
      if (fold && !(g4 && team_here && !hyb && f0 == 0))
        return fail(WG_ERR_INVALID, "launch_step: a folded first launch needs the team kernel");
      if (g4 && team_here) {
        if (!plan->team.wd)
          if (int rc2 = build_team_waves(L, plan->row1, LF, hyb ? L->tune.hyb_iter : L->tune.team_iter, hyb ? hyb->tcol : L->col,
                                         hyb ? hyb->tsplit : nullptr,
                                         L->tune.team_order >= 0 ? L->tune.team_order : (hyb ? 0 : 2), &plan->team))
            return rc2;
        a.u_bytes = (uint32_t)(L->n_cols * F * 4);
        a.probe = L->tune.probe;
        a.probe_h2 = L->tune.probe_h2;
        a.probe_fold = L->tune.probe_fold;
        a.coldnt = L->tune.coldnt;
        a.probe_ns = L->tune.probe_ns;
        if (fold) {
          if (cl->closed.gather_x0) {
            if (32 * plan->team.n_sell > (int64_t)0x7fffffff)  // sdinv at 2 x the ids' 32-bit byte offsets
              return fail(WG_ERR_UNSUPPORTED, "launch_step: %lld id slots: the folded first launch cannot address "
                          "their dinv", (long long)(4 * plan->team.n_sell));
            if (int rc2 = build_team_first(L, &plan->team)) return rc2;
            a.xm1 = cl->x0c;
          }
          a.x0c = cl->x0c;
          a.x0i = cl->x0i;
          a.perm_in = L->perm;
          if (int rc2 = launch_team4(plan->team, a, L->tune.team, stream, &cl->closed)) return rc2;
          continue;
        }
        if (tsum) {
          conc_args = a;
          conc_rows = plan->row1;
          a.tsum = tsum;
          if (defer) {
            conc_fused = a;
            conc_team = &plan->team;
            continue;
          }
        }
        if (int rc2 = launch_team4(plan->team, a, L->tune.team, tail_stream)) return rc2;
        continue;
      }
      if (g4 && !hyb) {
        if (int rc2 = build_pcol(L)) return rc2;
        a.prp = L->prp;
        a.pcol = L->pcol;
        a.u_bytes = (uint32_t)(L->n_cols * F * 4);
        a.p4v = L->tune.gather4;  // the loop variant (launch_main)
        if (L->tune.sell && plan->tab.total_blocks > 0) {  // team waves on SELL-ordered ids
          if (int rc2 = build_sell(L, plan, LF)) return rc2;
          a.wmeta = plan->wmeta;
          a.sell = plan->sell;
        }
      }
#ifdef WG_TIMING_PROBES
      if (L->tune.trace && L->trace_seq++ == L->tune.trace - 1) {
        const size_t need = (size_t)plan->tab.total_blocks * plan->nw * 4;
        if (L->trace_n < (int64_t)need) {
          (void)hipFree(L->trace_buf);
          L->trace_buf = nullptr;
          L->trace_n = 0;
          if (int rc2 = dmalloc(&L->trace_buf, need)) return rc2;
          L->trace_n = (int64_t)need;
        }
        WG_HIP_TRY(hipMemsetAsync(L->trace_buf, 0, sizeof(unsigned long long) * L->trace_n, stream));
        a.trace = L->trace_buf;
      }
#endif
      a.probe = L->tune.probe;
      a.probe_h2 = L->tune.probe_h2;
      a.probe_fold = L->tune.probe_fold;
      if (a.probe && !a.xk) a.xk = S ? S + f0 : nullptr;  // the final step of a chain stores into S
      a.chunks = plan->chunks;
      a.partial = plan->partial;
      // split rows index rowchunks / arrivals by internal row; a row-block plan's start at row0
      a.rowchunks = plan->rowchunks ? plan->rowchunks - plan->row0 : nullptr;
      a.arrivals = (L->tune.inkernel_combine && plan->n_split > 0) ? plan->arrivals - plan->row0 : nullptr;
      a.seg_mask = L->tune.seg_mask;
      // T_k stores write-through (sc1: the line leaves the XCD's L2, so the step's output stream
      // does not evict the rows it is gathering): ogbn-arxiv F=40 37.59 / 37.61 vs 38.29 / 37.91 us
      // per step plain, F=64 51.74 vs 52.14, Reddit-size F=41 746.6-747.2 vs 748.3-748.4 with nt
      // stores (profiles/r03/s29).  Before: nt stores only for > 64 MB step streams (arxiv F=40
      // 40.6 us plain vs 42.0 nt; Reddit-size F=44, 82 MB: 1773 plain vs 1738 nt)
      a.nt = L->tune.nt >= 0 ? L->tune.nt : 8;
      a.bcast = L->tune.bcast;
      // F == 1 gathers on large graphs: int4 index loads and narrower teams (8M R-MAT 8-way
      // shard: 275.7 us per step with vidx + iter 8 vs 296.9 without; ogbn-arxiv-size F=1:
      // vidx 12.3 vs 11.5, so only from 16 M nonzeros)
      a.vidx = L->tune.vidx >= 0 ? L->tune.vidx : (L->nnz >= ((int64_t)16 << 20) ? 1 : 0);
      if (vec == 4) rc = launch_step_vec<4>(*plan, a, stream);
      else if (vec == 2) rc = launch_step_vec<2>(*plan, a, stream);
      else rc = launch_step_vec<1>(*plan, a, stream);
      if (rc) return rc;
    }
    return WG_OK;
  };
  auto finish = [&]() -> int {
    if (H && !fuse_h) {
      hipLaunchKernelGGL(l1_normalize_kernel, dim3(ceil_div(L->n_rows, 4)), dim3(kBlock), 0, stream, L->n_rows, F, S, H);
      WG_LAUNCH_CHECK();
    }
    return prof_mark(L, stream, false);
  };
  // hybrid step (tiles.hip): the value-free Clenshaw steps of wide signals on large unweighted
  // graphs sum their dense blocks on the matrix cores (part), then gather each row's tail
  if (cl && cl->uin && !L->tune.probe && tiles_wanted(L, F)) {
    TilePlan* tp = nullptr;
    if (int rc = get_tile_plan(L, active_only, F, &tp)) return rc;
    if (tp) {
      const bool conc = vec == 4 && F <= max_tile && hybrid_conc_applies(L, tp, F) && gather4_applies(L, F);
      if (conc) {  // the tail's sums on the second stream beside the dense blocks, then one epilogue pass
        if (!L->side) WG_HIP_TRY(hipStreamCreateWithFlags(&L->side, hipStreamNonBlocking));
        // device-local ordering only: no system-scope fence on the fork / join records
        const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
        if (!L->side_fork) WG_HIP_TRY(hipEventCreateWithFlags(&L->side_fork, evf));
        if (!L->side_join) WG_HIP_TRY(hipEventCreateWithFlags(&L->side_join, evf));
        const int64_t need = L->n_rows * F;
        if (L->tsum_n < need) {
          (void)hipFree(L->tsum);
          L->tsum = nullptr;
          L->tsum_n = 0;
          if (int rc = dmalloc(&L->tsum, (size_t)need)) return rc;
          L->tsum_n = need;
        }
        int frc = WG_ERR_UNSUPPORTED;
        if (L->tune.hyb_conc != 3) {  // one launch: the dense blocks' workgroups, then the tail's waves
          if (int rc = tiles_loop(tp, stream, L->tsum, /*defer=*/true)) return rc;
          if (!conc_team) return fail(WG_ERR_INVALID, "launch_step: the hybrid tail's plan was not built");
          frc = launch_hybrid_fused(L, tp, F, xm1, *conc_team, conc_fused, stream);
          if (frc && frc != WG_ERR_UNSUPPORTED) return frc;
          if (!frc) ++tp->form_launches[2];
        }
        if (frc == WG_ERR_UNSUPPORTED) {  // two streams
          WG_HIP_TRY(hipEventRecord(L->side_fork, stream));
          WG_HIP_TRY(hipStreamWaitEvent(L->side, L->side_fork, 0));
          if (int rc = tiles_loop(tp, L->side, L->tsum)) return rc;
          if (int rc = launch_tiles(L, tp, F, xm1, stream)) return rc;
          WG_HIP_TRY(hipEventRecord(L->side_join, L->side));
          WG_HIP_TRY(hipStreamWaitEvent(stream, L->side_join, 0));
          ++tp->form_launches[1];
        }
        if (conc_rows < 0) return fail(WG_ERR_INVALID, "launch_step: the concurrent hybrid tail did not run");
        if (conc_rows > 0) {
          const int G = 64 / conc_args.LF;
          conc_args.tsum = L->tsum;
          hipLaunchKernelGGL(hybrid_epilogue_kernel, dim3((unsigned)ceil_div(conc_rows, 4 * (int64_t)G)), dim3(kBlock), 0,
                             stream, conc_args, conc_rows);
          WG_LAUNCH_CHECK();
        }
        return finish();
      }
      if (int rc = launch_tiles(L, tp, F, xm1, stream)) return rc;
      if (int rc = tiles_loop(tp)) return rc;
      ++tp->form_launches[0];
      return finish();
    }
  }
  if (int rc = tiles_loop(nullptr)) return rc;
  return finish();
}

int launch_finalize(wg_laplacian_s* L, int64_t F, const float* Sint, const float* X0int, double closed_coef, float* S,
                    float* H, hipStream_t stream, int64_t ldi) {
  const int64_t closed_from = X0int ? L->n_active : L->n_rows;
  const int64_t n = L->n_rows;
  if (n == 0) return WG_OK;
  if (ldi <= 0) ldi = F;
  int vec = pick_vec(F, {Sint, X0int, S, H});
  while (vec > 1 && ldi % vec) vec >>= 1;
  if (F <= 64 * vec) {
    const int LF = (int)(F / vec);
    const int G = 64 / LF;
    const dim3 grid((unsigned)ceil_div(n, 4 * G));
    if (vec == 4)
      hipLaunchKernelGGL(finalize_kernel<4>, grid, dim3(kBlock), 0, stream, n, F, ldi, LF, L->perm, Sint, X0int,
                         closed_from, closed_coef, S, H);
    else if (vec == 2)
      hipLaunchKernelGGL(finalize_kernel<2>, grid, dim3(kBlock), 0, stream, n, F, ldi, LF, L->perm, Sint, X0int,
                         closed_from, closed_coef, S, H);
    else
      hipLaunchKernelGGL(finalize_kernel<1>, grid, dim3(kBlock), 0, stream, n, F, ldi, LF, L->perm, Sint, X0int,
                         closed_from, closed_coef, S, H);
  } else {
    hipLaunchKernelGGL(finalize_wide_kernel, dim3(ceil_div(n, 4)), dim3(kBlock), 0, stream, n, F, ldi, L->perm, Sint,
                       X0int, closed_from, closed_coef, S, H);
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

int launch_permute_pad(wg_laplacian_s* L, int64_t F, int64_t Fp, const float* src, float* dst, hipStream_t stream) {
  const int64_t n = L->n_rows;
  if (n == 0) return WG_OK;
  if (Fp == F) return launch_permute(L, 0, F, src, dst, stream);
  hipLaunchKernelGGL(permute_pad_kernel, dim3((unsigned)ceil_div(n * Fp, 256)), dim3(256), 0, stream, n, F, Fp, L->perm,
                     src, dst);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

bool step_single_tile(wg_laplacian_s* L, int64_t F, std::initializer_list<const void*> ptrs) {
  const int vec = pick_vec(F, ptrs);
  int64_t max_tile = 64 * (int64_t)vec;
  if (L->tune.tile_f > 0) max_tile = std::max<int64_t>(vec, std::min<int64_t>(max_tile, L->tune.tile_f / vec * vec));
  return F <= max_tile;
}

// u_0 = X0 * dinv of the active rows only, internal order (fold 2)
int launch_permute_u0(wg_laplacian_s* L, int64_t F, const float* src, float* u, hipStream_t stream) {
  const int64_t n = L->n_active;
  if (n == 0) return WG_OK;
  if (F % 4) return fail(WG_ERR_INVALID, "permute_u0: F %% 4 != 0");
  const int LF = (int)(F / 4);
  if (LF > 64) return fail(WG_ERR_INVALID, "permute_u0: F too wide");
  const int G = 64 / LF;
  constexpr int kRG = 4;
  const dim3 grid((unsigned)ceil_div(n, 4 * G * kRG));
  hipLaunchKernelGGL((permute_in_closed_kernel<4, kRG>), grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, src,
                     (float*)nullptr, n, 0.0, (float*)nullptr, (float*)nullptr, L->dinv, u, (int64_t)0, (float*)nullptr);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int launch_permute_in_closed(wg_laplacian_s* L, int64_t F, const float* src, float* dst, double coef, float* S,
                             float* H, float* u, hipStream_t stream, float* zero) {
  const int64_t n = L->n_rows;
  if (n == 0) return WG_OK;
  const int vec = pick_vec(F, {src, dst, S, H, u, zero});
  if (F > 64 * vec) return fail(WG_ERR_INVALID, "permute_in_closed: F too wide");
  const int LF = (int)(F / vec);
  const int G = 64 / LF;
  constexpr int kRG = 4;
  const dim3 grid((unsigned)ceil_div(n, 4 * G * kRG));
  if (vec == 4)
    hipLaunchKernelGGL((permute_in_closed_kernel<4, kRG>), grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, src, dst,
                       L->n_active, coef, S, H, L->dinv, u, zero ? n : 0, zero);
  else if (vec == 2)
    hipLaunchKernelGGL((permute_in_closed_kernel<2, kRG>), grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, src, dst,
                       L->n_active, coef, S, H, L->dinv, u, zero ? n : 0, zero);
  else
    hipLaunchKernelGGL((permute_in_closed_kernel<1, kRG>), grid, dim3(kBlock), 0, stream, n, F, LF, L->perm, src, dst,
                       L->n_active, coef, S, H, L->dinv, u, zero ? n : 0, zero);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

namespace {
// mean 128-B cache lines one gathered row of W floats spans (rows back to back from a
// 256-B aligned base; the offsets mod 128 repeat with period <= 32 rows)
double lines_per_row(int64_t W) {
  int64_t tot = 0;
  for (int64_t i = 0; i < 32; ++i) {
    const int64_t o = (4 * W * i) % 128;
    tot += (o + 4 * W + 127) / 128;
  }
  return tot / 32.0;
}
}  // namespace

int padded_features(const wg_laplacian_s* L, int64_t F) {
  if (F < 3) return (int)F;
  const int64_t f4 = (F + 3) / 4 * 4;
  const int knob = L ? L->tune.fpad : 0;
  if (knob == 4 || knob == 8 || knob == 16) return (int)((F + knob - 1) / knob * knob);
  // auto: the width (a multiple of 4, or of 8) whose rows span the fewest cache lines -- the
  // step kernel is bound by gathered-line requests: F = 44 -> 48 (2.25 -> 2
  // lines per row; Reddit-size F=41 1504 -> 1422 us per step, profiles/r02/s6), F = 40 stays 40
  const int64_t f8 = (F + 7) / 8 * 8;
  return (int)(lines_per_row(f8) < lines_per_row(f4) - 1e-9 ? f8 : f4);
}

int launch_l1_normalize(const float* S, float* H, int64_t n, int64_t F, hipStream_t stream) {
  hipLaunchKernelGGL(l1_normalize_kernel, dim3(ceil_div(n, 4)), dim3(kBlock), 0, stream, n, F, S, H);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // namespace wg
