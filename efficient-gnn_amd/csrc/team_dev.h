// team_dev.h -- the independent-wave unit of the value-free step (team.hip), shared with the
// hybrid step's fused launch (tiles.hip hybrid_fused_kernel): the wave table's descriptors, the
// closed-form rows of a folded chain's first launch, and one wave's rows.
#pragma once

#include "step_dev.h"

namespace wg {
namespace {

// wave descriptor (two int4 per wave):
//   d0 = {first SELL chunk, chunks per sub-group, first row, LN | rows << 8 | part << 16}
//   d1 = {part index, parts of the row, first partial slot, arrival counter}   (part waves only)
struct TeamArgs {
  StepArgs a;
  const int4* wd;
  int32_t n_waves;
  double* wpart;   // [slots][LF * 4] float64 partials of part waves
  uint32_t* warr;  // [long rows] arrival counters (0 between launches: the last arrival resets)
  // the first launch of a folded chain (a.first) also finishes the purely isolated rows [closed_from,
  // n_rows) in closed form, S = coef * X0 and H = S / (|S|_1 + 1e-8) at their caller rows (what the
  // permute-in pass did), in n_closed_waves extra waves after the table's
  int32_t n_closed_waves;
  int64_t closed_from, n_rows;
  double coef;
  float* cS;
  float* cH;
#ifdef WG_DEBUG_BOUNDS
  int64_t dbg_rows, dbg_slots, dbg_long;  // the table's rows, partial slots and long rows
#endif
};

// the debug variant's plan sizes (WG_DEBUG_BOUNDS; nothing in the shipped library)
inline void team_args_debug(TeamArgs& t, const TeamPlan& tp) {
#ifdef WG_DEBUG_BOUNDS
  t.dbg_rows = tp.n_rows;
  t.dbg_slots = tp.n_slots;
  t.dbg_long = tp.n_long;
  t.a.dbg_sell_bytes = 16ull * (uint64_t)tp.n_sell;
#else
  (void)t;
  (void)tp;
#endif
}

constexpr int kClosedRG = 4;  // row groups per closed-form wave (their loads all issued before any use)

// rows [closed_from, n_rows): one LF-lane sub-group per row, kClosedRG groups of G rows per wave
__device__ __forceinline__ void closed_wave(const TeamArgs& t, int64_t cw) {
  const StepArgs& a = t.a;
  const int lane = threadIdx.x & 63;
  const int LF = a.LF;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  int64_t rows[kClosedRG], rs[kClosedRG];
  bool act[kClosedRG];
  float x[kClosedRG][4];
#pragma unroll
  for (int q = 0; q < kClosedRG; ++q) {
    rows[q] = t.closed_from + (cw * kClosedRG + q) * G + sg;
    act[q] = sg < G && rows[q] < t.n_rows;
    rs[q] = act[q] ? a.perm_in[rows[q]] : 0;
  }
#pragma unroll
  for (int q = 0; q < kClosedRG; ++q)
    if (act[q]) load_vec<4>(a.x0c + rs[q] * a.ld + fs * 4, x[q]);
#pragma unroll
  for (int q = 0; q < kClosedRG; ++q) {
    double sv[4];
    double part = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sv[j] = t.coef * (double)x[q][j];
      part += fabs(sv[j]);
    }
    double tot = 0.0;  // the row's L1 norm, in column order (finalize_kernel's order)
    for (int r = 0; r < LF; ++r) tot += __shfl(part, sg * LF + r, 64);
    if (!act[q]) continue;
    const double den = tot + 1e-8;
    double h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = sv[j] / den;
    store_vec<4>(t.cS + rs[q] * a.ld + fs * 4, sv);
    store_vec<4>(t.cH + rs[q] * a.ld + fs * 4, h);
  }
}

// MINW: minimum waves per SIMD the registers are held to (6 = the natural 77 VGPRs); LATE: the
// epilogue's X0 / previous-row operands loaded after the gathers instead of before (fewer live
// registers in the loop)
template <bool LATE, int CPT, bool FIRST = false>
__device__ __forceinline__ void team_wave(const TeamArgs& t, int w) {
  const StepArgs& a = t.a;
#ifdef WG_TIMING_PROBES
  if (a.probe_h2 == -4) return;  // launch + wave dispatch only
#endif
  int4 d0 = t.wd[2 * w];  // uniform address: a scalar load
  const int lane = threadIdx.x & 63;
  const int LF = a.LF;
  const int G = 64 / LF;
  const int sg = lane / LF;
  const int fs = lane - sg * LF;
  const int LN = d0.w & 0xff;
  const int tpw = (d0.w >> 8) & 0xff;
  const bool part = (d0.w >> 16) & 1;
  const int team = sg / LN;
  const int ns = sg - team * LN;
  const int64_t row = (int64_t)d0.z + team;
  const bool active = sg < G && team < tpw;
  WG_DCHECK(d0.z >= 0 && (int64_t)d0.z + (part ? 1 : tpw) <= t.dbg_rows && d0.y >= 0 && LN >= 1 && (part || tpw * LN <= G),
            "wave %d: descriptor {%d, %d, %d, %#x} outside the %lld-row table", w, d0.x, d0.y, d0.z, d0.w,
            (long long)t.dbg_rows);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  EpiIn<4> in;
#ifdef WG_TIMING_PROBES
  if (a.probe_h2 == -3) {  // no ids, gathers or epilogue operands: one 16-B store per row
    if (active && ns == 0 && a.xk)
      *reinterpret_cast<float4*>(a.xk + row * a.ld + fs * 4) = float4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  if (a.probe_h2 == -2) d0.y = 0;  // no ids, no gathers
#endif
  if (active) {
    if (!LATE && ns == 0 && !part && !a.tsum) epi_prefetch<4>(a, row, fs, in);
    accumulate_sell<CPT, FIRST>(a, int2{d0.x, d0.y}, G, sg, fs, acc);
    if (LATE && ns == 0 && !part && !a.tsum) epi_prefetch<4>(a, row, fs, in);
  }
  reduce_subgroups<4>(acc, LN, LF, team * LN * LF, fs);  // every lane (shuffles)
  bool emit = active && ns == 0;
  int lane0 = team * LN * LF;
  if (part) {  // a share of a long row: float64 partial (sc1), drained, then one arrival per wave
    const int4 d1 = t.wd[2 * w + 1];
    const int width = LF * 4;
    WG_DCHECK(d1.x >= 0 && d1.x < d1.y && d1.z >= 0 && (int64_t)d1.z + d1.y <= t.dbg_slots && d1.w >= 0 &&
                  d1.w < t.dbg_long,
              "part wave %d: {%d, %d, %d, %d} outside %lld slots / %lld long rows", w, d1.x, d1.y, d1.z, d1.w,
              (long long)t.dbg_slots, (long long)t.dbg_long);
    if (lane < LF) {
      double* p = t.wpart + (int64_t)(d1.z + d1.x) * width + lane * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) __hip_atomic_store(p + j, acc[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int last = 0;
    if (lane == 0) {
      // the arrival that completes the row resets its counter: every launch starts from 0, whatever
      // the history of earlier launches (uint32, compared for equality: no wrap-around modulus)
      const uint32_t old = __hip_atomic_fetch_add(t.warr + d1.w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old + 1u == (uint32_t)d1.y;
      if (last) __hip_atomic_store(t.warr + d1.w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    last = __shfl(last, 0, 64);
    if (!last || lane >= LF) return;
    // the last arriver: lanes 0 .. LF-1 (sub-group 0: fs == lane) sum every part's partial in
    // part order (deterministic) and share the team rows' epilogue below (one inlined copy)
    if (!a.tsum) epi_prefetch<4>(a, row, lane, in);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = 0.0;
    for (int q = 0; q < d1.y; ++q) {
      const double* p = t.wpart + (int64_t)(d1.z + q) * width + lane * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += __hip_atomic_load(p + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    emit = true;
    lane0 = 0;
  }
  if (emit) {
    if (a.tsum) {  // the row's sums only (hybrid_epilogue_kernel adds the dense blocks and finishes the row)
      double* p = a.tsum + row * a.ld + fs * 4;
      *reinterpret_cast<double2*>(p) = double2{acc[0], acc[1]};
      *reinterpret_cast<double2*>(p + 2) = double2{acc[2], acc[3]};
      return;
    }
    part_add<4>(a, row, fs, acc);
    step_epilogue<4>(a, row, fs, acc, in, lane0);
  }
}

}  // namespace
}  // namespace wg
