// team.hip -- the value-free Chebyshev / Clenshaw step for VEC-4 signals as independent WAVES
// (reference calibration/WATS.py:32-36 recurrence, :65-68 heat sum by Clenshaw, :71-72
// normalisation fused into the last step).
//
// Why a second kernel.  cheb_step_kernel (step.hip) runs workgroup units of three kinds (team
// rows, a workgroup per long row, split-row chunks reduced through LDS) in one kernel: its
// register and scalar-register budget is the union of the three (106 SGPRs, 75 VGPRs: 6
// workgroups of 4 waves per CU), and a long row holds four waves until the slowest finishes.
// Here every wave is a unit of its own, described by one entry of a wave table built with the
// plan (build_team_waves):
//   * team waves: G / LN rows, LN sub-groups of LF lanes per row (LN | G = 64 / LF), the row's
//     4-entry chunks dealt to its sub-groups (ns, ns + LN, ...), summed by shuffles;
//   * part waves: one share of a long row (all G sub-groups on it); the wave writes its float64
//     partial with write-through (sc1) stores, drains them, and adds to the row's arrival
//     counter; the wave whose add completes the row sums every part's partial with sc1 loads in
//     part order and runs the epilogue (MI355X_MICROARCH.md, hand-off table row 1, as step.hip's
//     split rows, per wave instead of per workgroup).
// Every wave reads its column ids in SELL order (accumulate_sell: one coalesced id read per turn,
// pads are dropped loads), so the kernel has no LDS, no barrier and a lean register budget.
#include <algorithm>
#include <cmath>
#include <vector>

#include "internal.h"

#include "team_dev.h"

namespace wg {
namespace {

template <int MINW, bool LATE, int CPT = 2>
__global__ __launch_bounds__(256, MINW) void cheb_team4_kernel(TeamArgs t) {
  const int w = (int)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w < t.n_waves) team_wave<LATE, CPT>(t, w);
}

// the first launch of a folded chain (no permute-in pass): gathers of the caller's X0 scaled by
// dinv, the internal X0 written by the epilogues, and the closed-form rows after the table's waves
// GX: the gathers read the caller's X0 scaled by dinv (fold 1); else u_0 from a pass (fold 2)
template <bool GX>
__global__ __launch_bounds__(256, 6) void cheb_team4_first_kernel(TeamArgs t) {
  const int w = (int)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w < t.n_waves) team_wave<false, 2, GX>(t, w);
  else if (w < t.n_waves + t.n_closed_waves) closed_wave(t, w - t.n_waves);
}

}  // namespace

void TeamPlan::release() {
  for (void* q : {(void*)wd, (void*)sell, (void*)wpart, (void*)warr, (void*)sell0, (void*)sdinv}) (void)hipFree(q);
  *this = TeamPlan{};
}

// The first launch's id table (fold): the SELL ids mapped to caller rows (perm) and each id slot's
// dinv (float64; 0 for pads, whose gathers return 0)
int build_team_first(wg_laplacian_s* L, TeamPlan* tp) {
  if (tp->sell0) return WG_OK;
  if (!tp->sell || tp->n_sell <= 0) return fail(WG_ERR_INVALID, "team first: no wave table");
  std::vector<int4> sell(tp->n_sell);
  WG_HIP_TRY(hipMemcpy(sell.data(), tp->sell, sizeof(int4) * sell.size(), hipMemcpyDeviceToHost));
  std::vector<int32_t> perm(L->n_rows);
  std::vector<double> dinv(L->n_cols);
  if (L->n_rows) WG_HIP_TRY(hipMemcpy(perm.data(), L->perm, sizeof(int32_t) * perm.size(), hipMemcpyDeviceToHost));
  if (L->n_cols) WG_HIP_TRY(hipMemcpy(dinv.data(), L->dinv, sizeof(double) * dinv.size(), hipMemcpyDeviceToHost));
  std::vector<double> sd(sell.size() * 4, 0.0);
  for (size_t i = 0; i < sell.size(); ++i) {
    int32_t* id = &sell[i].x;
    for (int j = 0; j < 4; ++j) {
      if (id[j] == kPadCol) continue;
      if (id[j] < 0 || id[j] >= L->n_rows) return fail(WG_ERR_INVALID, "team first: column %d outside the rows", id[j]);
      sd[4 * i + j] = dinv[id[j]];
      id[j] = perm[id[j]];
    }
  }
  int rc = dmalloc(&tp->sell0, sell.size());
  if (!rc) rc = dmalloc(&tp->sdinv, sd.size());
  if (!rc && (hipMemcpy(tp->sell0, sell.data(), sizeof(int4) * sell.size(), hipMemcpyHostToDevice) ||
              hipMemcpy(tp->sdinv, sd.data(), sizeof(double) * sd.size(), hipMemcpyHostToDevice)))
    rc = fail(WG_ERR_HIP, "team first: upload failed");
  if (rc) {
    (void)hipFree(tp->sell0);
    (void)hipFree(tp->sdinv);
    tp->sell0 = nullptr;
    tp->sdinv = nullptr;
  }
  return rc;
}

// The wave table and SELL ids of the rows [0, n) of L's operator (internal order, rows by
// descending length) for LF-lane sub-groups: a row of nch 4-entry chunks gets LN sub-groups, the
// smallest divisor of G with ceil(nch / LN) <= tch chunks each (tch = iter / 4, even); consecutive
// rows with the same LN share a wave (G / LN rows); a row longer than G * tch chunks is dealt to
// ceil(nch / (G * tch)) part waves.  Every sub-group of a wave runs the wave's chunk count (two chunks per turn, a single one last when it is odd),
// shorter ones padded with kPadCol chunks.
int build_team_waves(wg_laplacian_s* L, int64_t n, int LF, int iter, const int32_t* dcol,
                     const int32_t* drsplit, int order, TeamPlan* tp) {
  const int G = 64 / LF;
  const int64_t tch = std::max<int64_t>(2, (iter / 4 + 1) / 2 * 2);
  std::vector<int32_t> rs(n + 1);  // row starts; the entries of row r are [rs[r], re[r])
  WG_HIP_TRY(hipMemcpy(rs.data(), L->rowptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  std::vector<int32_t> col(std::max<int32_t>(rs[n], 1));
  if (rs[n]) WG_HIP_TRY(hipMemcpy(col.data(), dcol, sizeof(int32_t) * rs[n], hipMemcpyDeviceToHost));
  std::vector<int32_t> re(rs.begin() + 1, rs.end());  // drsplit: the hybrid step's tail ends
  if (drsplit && n) WG_HIP_TRY(hipMemcpy(re.data(), drsplit, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  auto rlen = [&](int64_t r) -> int64_t { return re[r] - rs[r]; };
  std::vector<int> divs;
  for (int d = 1; d <= G; ++d)
    if (G % d == 0) divs.push_back(d);
  std::vector<int4> wd;
  std::vector<int4> sell;
  const int4 pad4{kPadCol, kPadCol, kPadCol, kPadCol};
  int32_t slots = 0, longs = 0;
  tp->max_parts = tp->npot_rows = 0;
  auto chunk = [&](int64_t r, int64_t ch) {  // the 4 ids of chunk ch of row r
    int32_t id[4];
    for (int i = 0; i < 4; ++i) {
      const int64_t e = (int64_t)rs[r] + ch * 4 + i;
      id[i] = e < re[r] ? col[e] : kPadCol;
    }
    return int4{id[0], id[1], id[2], id[3]};
  };
  auto fits = [&]() {
    return sell.size() < ((size_t)1 << 27);  // 16-B chunks at 32-bit byte offsets (accumulate_sell)
  };
  int64_t r = 0;
  while (r < n) {
    const int64_t nch0 = (rlen(r) + 3) / 4;
    if (nch0 > (int64_t)G * tch) {  // a long row: part waves, all G sub-groups on one share each
      const int64_t per = (int64_t)G * tch;
      const int32_t parts = (int32_t)((nch0 + per - 1) / per);
      for (int32_t q = 0; q < parts; ++q) {
        const int64_t c0 = q * per, c1 = std::min<int64_t>(nch0, c0 + per);
        const int64_t nchs = (c1 - c0 + G - 1) / G;  // chunks per sub-group
        wd.push_back(int4{(int32_t)sell.size(), (int32_t)nchs, (int32_t)r, G | (1 << 8) | (1 << 16)});
        wd.push_back(int4{q, parts, slots, longs});
        const size_t base = sell.size();
        sell.resize(base + (size_t)nchs * G, pad4);
        for (int64_t c = c0; c < c1; ++c) sell[base + (size_t)(c - c0)] = chunk(r, c);  // chunk k: k / G, k % G
        if (!fits()) return fail(WG_ERR_UNSUPPORTED, "team waves: id array exceeds 2 GB");
      }
      slots += parts;
      ++longs;
      tp->max_parts = std::max(tp->max_parts, parts);
      if (parts & (parts - 1)) ++tp->npot_rows;
      ++r;
      continue;
    }
    int LN = G;
    for (int d : divs)
      if ((nch0 + d - 1) / d <= tch) {
        LN = d;
        break;
      }
    const int tpw = G / LN;
    int rows = 0;
    while (rows < tpw && r + rows < n) {  // consecutive rows with the same LN
      const int64_t nch = (rlen(r + rows) + 3) / 4;
      if (nch > (int64_t)G * tch) break;
      int ln = G;
      for (int d : divs)
        if ((nch + d - 1) / d <= tch) {
          ln = d;
          break;
        }
      if (ln != LN) break;
      ++rows;
    }
    int64_t nchs = 0;  // chunks per sub-group: the wave's most (sub-group 0 of its longest row)
    for (int i = 0; i < rows; ++i) {
      const int64_t nch = (rlen(r + i) + 3) / 4;
      nchs = std::max<int64_t>(nchs, (nch + LN - 1) / LN);
    }
    wd.push_back(int4{(int32_t)sell.size(), (int32_t)nchs, (int32_t)r, LN | (rows << 8)});
    wd.push_back(int4{0, 0, 0, 0});
    const size_t base = sell.size();
    sell.resize(base + (size_t)nchs * G, pad4);
    for (int i = 0; i < rows; ++i) {
      const int64_t nch = (rlen(r + i) + 3) / 4;
      for (int ns = 0; ns < LN; ++ns)
        for (int64_t k = 0; ns + k * LN < nch; ++k)
          sell[base + (size_t)k * G + (size_t)(i * LN + ns)] = chunk(r + i, ns + k * LN);
    }
    if (!fits()) return fail(WG_ERR_UNSUPPORTED, "team waves: id array exceeds 2 GB");
    r += rows;
  }
  sell.resize(sell.size() + (size_t)4 * G, pad4);  // the next-turn id reads past the last wave
  if (order) {  // dispatch order of the waves (the table is built longest rows first)
    const size_t nw = wd.size() / 2;
    std::vector<int4> o;
    o.reserve(wd.size());
    // 1: reversed (shortest rows first); 2 ..: fa waves from the longest end, then fb from the
    // shortest, repeated.  2 (one and one) mixes long and short rows in every workgroup: arxiv
    // F = 40 33.9 vs 34.7 us; whole workgroups alternating (7) put every long row on every other
    // XCD (round-robin placement): 51.9 (r04 s28)
    static const int kFa[8] = {0, 0, 1, 2, 4, 1, 1, 4}, kFb[8] = {0, 0, 1, 1, 1, 2, 4, 4};
    size_t lo = 0, hi = nw;
    while (lo < hi) {
      if (order == 1) {
        --hi;
        o.push_back(wd[2 * hi]);
        o.push_back(wd[2 * hi + 1]);
        continue;
      }
      for (int q = 0; q < kFa[order] && lo < hi; ++q, ++lo) {
        o.push_back(wd[2 * lo]);
        o.push_back(wd[2 * lo + 1]);
      }
      for (int q = 0; q < kFb[order] && lo < hi; ++q) {
        --hi;
        o.push_back(wd[2 * hi]);
        o.push_back(wd[2 * hi + 1]);
      }
    }
    wd.swap(o);
  }
  tp->n_waves = (int32_t)(wd.size() / 2);
  tp->n_sell = (int64_t)sell.size();
  tp->n_rows = n;
  tp->n_slots = slots;
  tp->n_long = longs;
  tp->width = LF * 4;
  int rc = dmalloc(&tp->wd, std::max<size_t>(wd.size(), 2));
  if (!rc) rc = dmalloc(&tp->sell, sell.size());
  if (!rc) rc = dmalloc(&tp->wpart, (size_t)std::max(slots, 1) * tp->width);
  if (!rc) rc = dmalloc(&tp->warr, (size_t)std::max(longs, 1));
  if (!rc && ((!wd.empty() && hipMemcpy(tp->wd, wd.data(), sizeof(int4) * wd.size(), hipMemcpyHostToDevice)) ||
              hipMemcpy(tp->sell, sell.data(), sizeof(int4) * sell.size(), hipMemcpyHostToDevice) ||
              hipMemset(tp->warr, 0, sizeof(uint32_t) * std::max(longs, 1))))
    rc = fail(WG_ERR_HIP, "team waves: upload failed");
  if (rc) tp->release();  // no half-built table (wd non-null marks a built one)
  return rc;
}

int launch_team4(const TeamPlan& tp, const StepArgs& a, int variant, hipStream_t stream, const TeamFirst* first) {
  TeamArgs t{};
  t.a = a;
  t.wd = tp.wd;
  t.n_waves = tp.n_waves;
  t.wpart = tp.wpart;
  t.warr = tp.warr;
  t.a.sell = tp.sell;
  team_args_debug(t, tp);
  if (first) {  // the folded chain's first launch
    const bool gx = first->gather_x0;
    if (gx && !tp.sell0) return fail(WG_ERR_INVALID, "launch_team4: no first-launch table");
    const int G = 64 / a.LF;
    t.a.first = 1;
    if (gx) {
      t.a.sell = tp.sell0;
      t.a.sdinv = tp.sdinv;
    }
    t.closed_from = first->closed_from;
    t.n_rows = first->n_rows;
    t.coef = first->coef;
    t.cS = first->S;
    t.cH = first->H;
    const int64_t nc = std::max<int64_t>(0, first->n_rows - first->closed_from);
    t.n_closed_waves = (int32_t)ceil_div(nc, (int64_t)G * kClosedRG);
    if (nc && (!t.cS || !t.cH)) return fail(WG_ERR_INVALID, "launch_team4: closed-form rows need S and H");
    const int64_t nw = (int64_t)tp.n_waves + t.n_closed_waves;
    if (nw <= 0) return WG_OK;
    if (gx) hipLaunchKernelGGL(cheb_team4_first_kernel<true>, dim3((unsigned)ceil_div(nw, 4)), dim3(256), 0, stream, t);
    else hipLaunchKernelGGL(cheb_team4_first_kernel<false>, dim3((unsigned)ceil_div(nw, 4)), dim3(256), 0, stream, t);
    WG_LAUNCH_CHECK();
    return WG_OK;
  }
  if (tp.n_waves <= 0) return WG_OK;
  const dim3 grid((unsigned)ceil_div(tp.n_waves, 4)), block(256);
  switch (variant) {
    case 7: hipLaunchKernelGGL((cheb_team4_kernel<7, false>), grid, block, 0, stream, t); break;
    case 8: hipLaunchKernelGGL((cheb_team4_kernel<8, false>), grid, block, 0, stream, t); break;
    case 9: hipLaunchKernelGGL((cheb_team4_kernel<8, true>), grid, block, 0, stream, t); break;
    case 10: hipLaunchKernelGGL((cheb_team4_kernel<6, true>), grid, block, 0, stream, t); break;
    case 11: hipLaunchKernelGGL((cheb_team4_kernel<6, false, 1>), grid, block, 0, stream, t); break;
    case 12: hipLaunchKernelGGL((cheb_team4_kernel<8, false, 1>), grid, block, 0, stream, t); break;
    case 13: hipLaunchKernelGGL((cheb_team4_kernel<8, true, 1>), grid, block, 0, stream, t); break;
    default: hipLaunchKernelGGL((cheb_team4_kernel<6, false>), grid, block, 0, stream, t);
  }
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // namespace wg
