// capi.hip -- C ABI entry points of the chain (include/wats_hip.h):
// graph_wavelet_features (reference calibration/WATS.py:39-74), one
// chebyshev_polynomials step (WATS.py:29-37), row-L1 normalisation
// (WATS.py:71-72), row permutations, halo gather, profiling and tuning.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <tuple>
#include <vector>

#include "internal.h"

namespace wg {

namespace {
thread_local std::string g_err;
thread_local std::string g_text;

__global__ void gather_rows_kernel(int64_t n, int64_t F, const int32_t* __restrict__ rows, const float* __restrict__ src,
                                   float* __restrict__ dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * F) return;
  const int64_t i = idx / F;
  const int64_t f = idx - i * F;
  dst[idx] = src[(int64_t)rows[i] * F + f];
}
__global__ void map_rows_kernel(int64_t n, const int32_t* __restrict__ map, const int32_t* __restrict__ rows,
                                int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = map[rows[i]];
}
}  // namespace

int ensure_dyn_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  WG_HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_tuple(fn, dev, bytes);
  if (done.count(key)) return WG_OK;
  WG_HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert(key);
  return WG_OK;
}

int n_cus(int dev) {
  static int cached[64] = {0};
  if (dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cached[dev] = v;
  }
  return cached[dev];
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int launch_l1_normalize(const float* S, float* H, int64_t n, int64_t F, hipStream_t stream);

}  // namespace wg

using namespace wg;

extern "C" {

const char* wg_last_error(void) { return g_err.c_str(); }

int wg_abi_version(void) { return WG_ABI_VERSION; }

int wg_laplacian_get_info(wg_laplacian_t L, wg_laplacian_info* info) {
  if (!L || !info) return fail(WG_ERR_INVALID, "wg_laplacian_get_info: NULL argument");
  info->n_rows = L->n_rows;
  info->n_cols = L->n_cols;
  info->nnz_input = L->nnz_input;
  info->nnz = L->nnz;
  info->n_isolated = L->n_iso;
  info->max_row_nnz = L->max_row;
  info->n_segments = 0;
  for (auto& kv : L->plans) info->n_segments = std::max(info->n_segments, kv.second.tab.n);
  info->reordered = L->reordered ? 1 : 0;
  info->n_closed_form = L->n_closed;
  return WG_OK;
}

int wg_laplacian_tune(wg_laplacian_t L, const char* key, int64_t value) {
  if (!L || !key) return fail(WG_ERR_INVALID, "wg_laplacian_tune: NULL argument");
  // any knob -- plan-shaping or launch-time -- invalidates a chain captured into a
  // hipGraph (dist.hip keys its exec on this counter): plan buffers are freed below,
  // and launch-time knobs are baked into the captured kernel arguments
  ++L->tune_gen;
  L->chain1_off = false;  // any tune gives a one-launch chain that timed out another chance
  if (!strcmp(key, "iter")) {
    if (value < 1) return fail(WG_ERR_INVALID, "iter must be >= 1");
    L->tune.iter = (int32_t)value;
  } else if (!strcmp(key, "chunk_iter")) {
    if (value < 1) return fail(WG_ERR_INVALID, "chunk_iter must be >= 1");
    L->tune.chunk_iter = (int32_t)value;
  } else if (!strcmp(key, "block_iter")) {
    if (value < 1) return fail(WG_ERR_INVALID, "block_iter must be >= 1");
    L->tune.block_iter = (int32_t)value;
  } else if (!strcmp(key, "nt")) {
    L->tune.nt = (int32_t)value;
    return WG_OK;
  } else if (!strcmp(key, "waves")) {
    if (value != 4 && value != 8 && value != 16) return fail(WG_ERR_INVALID, "waves must be 4, 8 or 16");
    L->tune.waves = (int32_t)value;
  } else if (!strcmp(key, "hot")) {
    L->tune.hot = (int32_t)std::max<int64_t>(0, std::min<int64_t>(value, 40000));
  } else if (!strcmp(key, "vidx")) {
    L->tune.vidx = value < 0 ? -1 : (value ? 1 : 0);
    return WG_OK;
  } else if (!strcmp(key, "bcast")) {
    L->tune.bcast = value ? 1 : 0;
    return WG_OK;
  } else if (!strcmp(key, "tile_f")) {
    L->tune.tile_f = (int32_t)std::max<int64_t>(0, value);
  } else if (!strcmp(key, "lds")) {
    if (value < 0 || value > 4) return fail(WG_ERR_INVALID, "lds must be 0, 1, 2, 3 (auto) or 4");
    L->tune.lds = (int32_t)value;
  } else if (!strcmp(key, "lds_cb")) {
    if (value < 32 || value > 40704) return fail(WG_ERR_INVALID, "lds_cb must be in [32, 40704]");
    L->tune.lds_cb = (int32_t)value;
  } else if (!strcmp(key, "lds_iter")) {
    if (value < 1) return fail(WG_ERR_INVALID, "lds_iter must be >= 1");
    L->tune.lds_iter = (int32_t)value;
  } else if (!strcmp(key, "lds_wg")) {
    L->tune.lds_wg = (int32_t)std::max<int64_t>(0, value);
  } else if (!strcmp(key, "sortcols")) {
    if (value) {
      WG_HIP_TRY(hipDeviceSynchronize());
      if (int rc = sort_row_columns(L, nullptr)) return rc;
    }
  } else if (!strcmp(key, "clenshaw")) {
    L->tune.clenshaw = value ? 1 : 0;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "uscale")) {
    L->tune.uscale = value ? 1 : 0;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "inkernel_combine")) {
    L->tune.inkernel_combine = value ? 1 : 0;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "lds_k")) {
    if (value != 1 && value != 2 && value != 4) return fail(WG_ERR_INVALID, "lds_k must be 1, 2 or 4");
    L->tune.lds_k = (int32_t)value;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "lds_depth")) {
    L->tune.lds_depth = (int32_t)value;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "lds_maxnb")) {
    L->tune.lds_maxnb = (int32_t)std::max<int64_t>(1, std::min<int64_t>(value, 64));
  } else if (!strcmp(key, "fuse_finalize")) {
    L->tune.fuse_finalize = value ? 1 : 0;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "hub_iter")) {
    L->tune.hub_iter = (int32_t)std::max<int64_t>(1, std::min<int64_t>(value, 4096));
  } else if (!strcmp(key, "fpad")) {
    if (value != 0 && value != 4 && value != 8 && value != 16) return fail(WG_ERR_INVALID, "fpad must be 0, 4, 8 or 16");
    L->tune.fpad = (int32_t)value;
    return WG_OK;  // launch-time choice (workspace regrows on the next call)
  } else if (!strcmp(key, "hub_sell")) {
    L->tune.hub_sell = value ? 1 : 0;  // plan-time choice (the LDS plans are rebuilt)
  } else if (!strcmp(key, "tiles")) {
    if (value < -1 || value > 1) return fail(WG_ERR_INVALID, "tiles must be -1 (auto), 0 or 1");
    L->tune.tiles = (int32_t)value;
  } else if (!strcmp(key, "tile_th")) {
    if (value < 1 || value > 2048) return fail(WG_ERR_INVALID, "tile_th must be in [1, 2048]");
    L->tune.tile_th = (int32_t)value;
  } else if (!strcmp(key, "tile_rows")) {
    if (value != 64 && value != 128) return fail(WG_ERR_INVALID, "tile_rows must be 64 or 128");
    L->tune.tile_rows = (int32_t)value;
  } else if (!strcmp(key, "tile_rg")) {
    if (value != 1 && value != 2 && value != 4) return fail(WG_ERR_INVALID, "tile_rg must be 1, 2 or 4");
    L->tune.tile_rg = (int32_t)value;  // plans rebuilt (the fused launch's tile items)
  } else if (!strcmp(key, "tile_mfma")) {
    if (value != 0 && value != 16 && value != 32) return fail(WG_ERR_INVALID, "tile_mfma must be 0 (auto), 16 or 32");
    L->tune.tile_mfma = (int32_t)value;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "tile_max")) {
    if (value < 0 || value > 1024) return fail(WG_ERR_INVALID, "tile_max must be in [0 (auto), 1024]");
    L->tune.tile_max = (int32_t)value;
  } else if (!strcmp(key, "lds_perm")) {
    L->tune.lds_perm = value ? 1 : 0;
  } else if (!strcmp(key, "chain")) {
    if (value < -1 || value > 1) return fail(WG_ERR_INVALID, "chain must be -1 (auto), 0 or 1");
    L->tune.chain = (int32_t)value;
  } else if (!strcmp(key, "chain_wg")) {
    if (value < 0 || value > 1024) return fail(WG_ERR_INVALID, "chain_wg must be in [0 (auto), 1024]");
    L->tune.chain_wg = (int32_t)value;
  } else if (!strcmp(key, "chain_fault")) {
    if (value < 0 || value > kChainMaxK) return fail(WG_ERR_INVALID, "chain_fault must be in [0, %d]", kChainMaxK);
    L->tune.chain_fault = (int32_t)value;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "hyb_conc")) {
    if (value < 0 || value > 3) return fail(WG_ERR_INVALID, "hyb_conc must be 0, 1 (auto), 2 (always) or 3 (two streams)");
    L->tune.hyb_conc = (int32_t)value;  // plans rebuilt: the fused launch's tile items are longer
  } else if (!strcmp(key, "chain_solo")) {
    if (value < 0 || value > 2) return fail(WG_ERR_INVALID, "chain_solo must be 0, 1 (auto) or 2 (wherever it fits)");
    L->tune.chain_solo = (int32_t)value;  // plans rebuilt
  } else if (!strcmp(key, "chain_direct")) {
    L->tune.chain_direct = value ? 1 : 0;  // also the auto worker count: plans rebuilt
  } else if (!strcmp(key, "chain_xcd")) {
    L->tune.chain_xcd = value ? 1 : 0;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "gather4")) {
    if (value != 0 && value != 1 && value != 21 && value != 22 && value != 31 && value != 41 && value != 121)
      return fail(WG_ERR_INVALID, "gather4 must be 0 (off), 1 (default loop), 21, 22, 31, 41 or 121");
    L->tune.gather4 = (int32_t)(value == 1 ? 21 : value);
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "team")) {
    if (value < 0 || value > 13 || (value > 1 && value < 7))
      return fail(WG_ERR_INVALID, "team must be 0 (off), 1 (default) or 7 .. 13");
    L->tune.team = (int32_t)value;
    return WG_OK;  // launch-time choice (the wave table is built with the plan on first use)

  } else if (!strcmp(key, "team_tail")) {
    if (value < 0) return fail(WG_ERR_INVALID, "team_tail must be >= 0");
    L->tune.team_tail = value;
    return WG_OK;  // launch-time choice (each plan keeps its own wave table)
  } else if (!strcmp(key, "team_order")) {
    if (value < -1 || value > 7) return fail(WG_ERR_INVALID, "team_order must be -1 (auto) or in [0, 7]");
    L->tune.team_order = (int32_t)value;
  } else if (!strcmp(key, "fold")) {
    if (value < 0 || value > 2) return fail(WG_ERR_INVALID, "fold must be 0, 1 or 2");
    L->tune.fold = (int32_t)value;
    return WG_OK;  // launch-time choice
  } else if (!strcmp(key, "hyb_iter")) {
    if (value < 8 || value > 4096) return fail(WG_ERR_INVALID, "hyb_iter must be in [8, 4096]");
    L->tune.hyb_iter = (int32_t)value;
  } else if (!strcmp(key, "team_iter")) {
    if (value < 8 || value > 4096) return fail(WG_ERR_INVALID, "team_iter must be in [8, 4096]");
    L->tune.team_iter = (int32_t)value;
  } else if (!strcmp(key, "sell")) {
    L->tune.sell = value ? 1 : 0;
    return WG_OK;  // launch-time choice (the SELL arrays are built with the plan on first use)
  } else if (!strcmp(key, "graph")) {
    if (value < -1 || value > 1) return fail(WG_ERR_INVALID, "graph must be -1 (auto), 0 or 1");
    L->tune.graph = (int32_t)value;
    return WG_OK;  // launch-time choice (tune_gen: a captured chain is re-captured)
#ifdef WG_TIMING_PROBES
    // timing probes (results wrong or time inflated on purpose): only in a probe build
    // (make -C efficient-gnn_amd/csrc VARIANT=probes EXTRA_FLAGS=-DWG_TIMING_PROBES)
  } else if (!strcmp(key, "seg_mask")) {
    L->tune.seg_mask = value;  // plan segments launched (timing attribution)
    return WG_OK;
  } else if (!strcmp(key, "probe")) {
    L->tune.probe = value ? 1 : 0;  // the gathers alone: no epilogue operands
    return WG_OK;
  } else if (!strcmp(key, "trace")) {
    L->tune.trace = (int32_t)std::max<int64_t>(0, value);  // 1-based step launch to record, 0 = off
    L->trace_seq = 0;
    return WG_OK;
  } else if (!strcmp(key, "probe_h2")) {
    L->tune.probe_h2 = (int32_t)value;  // negative: the skeleton probes (step.hip, step_dev.h)
    return WG_OK;
  } else if (!strcmp(key, "probe_ns")) {
    L->tune.probe_ns = (int32_t)value;
    return WG_OK;
  } else if (!strcmp(key, "coldnt")) {
    L->tune.coldnt = (int32_t)std::max<int64_t>(0, value);
    return WG_OK;
  } else if (!strcmp(key, "probe_fold")) {
    L->tune.probe_fold = (int32_t)value;  // -1: ids from one 4-KB window (accumulate_u4)
    return WG_OK;
  } else if (!strcmp(key, "probe_tailwin")) {
    L->tune.probe_tailwin = (int32_t)std::max<int64_t>(0, std::min<int64_t>(value, 1024));  // plan-time
  } else if (!strcmp(key, "xdelay")) {
    L->tune.xdelay = (int32_t)std::max<int64_t>(0, std::min<int64_t>(value, 100000));  // simulated link us
    return WG_OK;
#endif
  } else {
    return fail(WG_ERR_INVALID, "wg_laplacian_tune: unknown key '%s'", key);
  }
  WG_HIP_TRY(hipDeviceSynchronize());
  for (auto& kv : L->plans) kv.second.release();
  L->plans.clear();
  release_lds1(L);
  release_chain1(L);
  return WG_OK;
}

int wg_laplacian_set_halo_groups(wg_laplacian_t L, int32_t n_groups, const int64_t* offsets) {
  if (!L || n_groups < 0 || (n_groups > 0 && !offsets))
    return fail(WG_ERR_INVALID, "wg_laplacian_set_halo_groups: bad arguments");
  if (n_groups > 0 && (offsets[0] != 0 || offsets[n_groups] != L->n_cols - L->n_rows))
    return fail(WG_ERR_INVALID, "wg_laplacian_set_halo_groups: offsets must run from 0 to the halo size %lld",
                (long long)(L->n_cols - L->n_rows));
  for (int32_t q = 0; q < n_groups; ++q)
    if (offsets[q + 1] < offsets[q]) return fail(WG_ERR_INVALID, "wg_laplacian_set_halo_groups: offsets decrease");
  WG_HIP_TRY(hipDeviceSynchronize());
  if (n_groups > 0) L->halo_off.assign(offsets, offsets + n_groups + 1);
  else L->halo_off.clear();
  release_lds1(L);
  return WG_OK;
}

const char* wg_laplacian_describe(wg_laplacian_t L, int64_t F) {
  g_text.clear();
  if (!L || F < 1) return "";
  const int vec = (F % 4 == 0) ? 4 : (F % 2 == 0) ? 2 : 1;
  const int LF = (int)(std::min<int64_t>(F, 64 * vec) / vec);
  Plan* p = nullptr;
  if (get_plan(L, LF, vec, true, &p)) return "";
  char buf[192];
  snprintf(buf, sizeof(buf), "F=%lld VEC=%d LF=%d segments=%d blocks=%d active_rows=%lld closed_form_rows=%lld\n",
           (long long)F, vec, LF, p->tab.n, p->tab.total_blocks, (long long)L->n_active, (long long)L->n_closed);
  g_text = buf + p->text;
  // split-row arrival counters left non-zero (each row's completing arrival resets its counter,
  // so a finished launch leaves none: tests read this after a device sync)
  auto pending = [](const uint32_t* d, int32_t n) -> int {
    if (!d || n <= 0) return 0;
    std::vector<uint32_t> h(n);
    if (hipMemcpy(h.data(), d, sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int)std::count_if(h.begin(), h.end(), [](uint32_t v) { return v != 0; });
  };
  if (p->team.wd) {  // the independent-wave step kernel's table, once a step has built it (team.hip)
    snprintf(buf, sizeof(buf), "team: waves=%d long_rows=%d part_slots=%d max_parts=%d npot_rows=%d pending_arrivals=%d\n",
             p->team.n_waves, p->team.n_long, p->team.n_slots, p->team.max_parts, p->team.npot_rows,
             pending(p->team.warr, p->team.n_long));
    g_text += buf;
  }
  if (p->arrivals && p->n_split > 0) {
    snprintf(buf, sizeof(buf), "split rows: %d pending_arrivals=%d\n", p->n_split, pending(p->arrivals, p->n_split));
    g_text += buf;
  }
  for (int i = 1; i >= 0; --i)  // the hybrid step's plan, once a chain has built it, and the forms it ran in
    if (L->tiles[i]) {
      const TilePlan* tp = L->tiles[i];
      g_text += tp->text;
      snprintf(buf, sizeof(buf), "hybrid forms: fused=%lld two_stream=%lld sequential=%lld\n",
               (long long)tp->form_launches[2], (long long)tp->form_launches[1], (long long)tp->form_launches[0]);
      g_text += buf;
    }
  if (F == 1) {
    Lds1Plan* lp = nullptr;
    if (!get_lds1_plan(L, true, &lp) && lp) g_text += lp->text;
    if (L->chain1) g_text += L->chain1->text;  // once a chain has built it
    if (L->chain1_timeouts || L->chain1_off) {
      snprintf(buf, sizeof(buf), "chain1 timeouts=%d%s\n", L->chain1_timeouts,
               L->chain1_off ? " (off: multi-launch path)" : "");
      g_text += buf;
    }
  }
  return g_text.c_str();
}

int wg_cheb_step(wg_laplacian_t L, int32_t k, int64_t F, const float* t_km1, const float* t_km2, float* t_k, float* S,
                 float* H, double alpha0, double alpha_k, void* stream_) {
  if (!L || k < 1 || F < 1 || !t_km1 || (k >= 2 && !t_km2) || (H && !S))
    return fail(WG_ERR_INVALID, "wg_cheb_step: bad arguments (k=%d F=%lld)", k, (long long)F);
  return launch_step(L, k, F, t_km1, t_km2, t_k, S, H, alpha0, alpha_k, as_stream(stream_));
}

int wg_clenshaw_step(wg_laplacian_t L, int64_t F, const float* b1, const float* b2, const float* x0, float* out,
                     double ck, double cacc, int32_t flags, void* stream_) {
  if (!L || F < 1 || (L->n_rows && (!b1 || !x0 || !out)) || (flags & ~31) ||
      ((flags & WG_CLEN_FINAL) && (flags & WG_CLEN_UOUT)) || ((flags & (WG_CLEN_UIN | WG_CLEN_UPREV)) && !L->unit))
    return fail(WG_ERR_INVALID, "wg_clenshaw_step: bad arguments (F=%lld flags=%d)", (long long)F, flags);
  const bool fin = (flags & WG_CLEN_FINAL) != 0;
  ClenArgs cl{x0, ck, cacc, fin ? 1 : 0};
  cl.uin = (flags & WG_CLEN_UIN) ? 1 : 0;
  cl.uprev = (flags & WG_CLEN_UPREV) ? 1 : 0;
  cl.uout = (flags & WG_CLEN_UOUT) ? 1 : 0;
  return launch_step(L, 2, F, b1, b2, fin ? nullptr : out, fin ? out : nullptr, nullptr, 1.0, 0.0, as_stream(stream_),
                     (flags & WG_CLEN_ACTIVE) != 0, nullptr, &cl);
}

int wg_cheb_u_len(wg_laplacian_t L, int64_t* len) {
  if (!L || !len) return fail(WG_ERR_INVALID, "wg_cheb_u_len: NULL argument");
  *len = 0;
  Lds1Plan* lp = nullptr;
  if (int rc = get_lds1_plan(L, /*active_only=*/false, &lp)) return rc;
  if (lp) *len = lp->u_floats();
  return WG_OK;
}

int wg_lds_plan_info(wg_laplacian_t L, int32_t active_only, int64_t* out) {
  if (!L || !out) return fail(WG_ERR_INVALID, "wg_lds_plan_info: NULL argument");
  for (int i = 0; i < 8; ++i) out[i] = 0;
  Lds1Plan* lp = nullptr;
  if (int rc = get_lds1_plan(L, active_only != 0, &lp)) return rc;
  if (!lp) return WG_OK;
  out[0] = lp->mode;
  out[1] = lp->nb;
  out[2] = lp->n;
  out[3] = lp->n_cols;
  out[4] = lp->nnz;
  out[5] = lp->mode == 2 ? lp->n_pairs : (lp->nb > 1 ? (int64_t)lp->nb * lp->n : 0);
  out[6] = lp->n_chunks;
  out[7] = lp->n_wg;
  return WG_OK;
}

int wg_scale_dinv(wg_laplacian_t L, const float* x, float* u, void* stream_) {
  if (!L || (L->n_rows && (!x || !u))) return fail(WG_ERR_INVALID, "wg_scale_dinv: bad arguments");
  return launch_scale_dinv(L, L->n_rows, x, u, as_stream(stream_));
}

int wg_cheb_step_u(wg_laplacian_t L, int32_t k, const float* u_km1, const float* t_km1, const float* t_km2,
                   float* t_k, float* u_k, float* S, double alpha0, double alpha_k, void* stream_) {
  if (!L || k < 1 || (L->n_rows && (!u_km1 || !t_km1)) || (k >= 2 && L->n_rows && !t_km2))
    return fail(WG_ERR_INVALID, "wg_cheb_step_u: bad arguments (k=%d)", k);
  Lds1Plan* lp = nullptr;
  if (int rc = get_lds1_plan(L, /*active_only=*/false, &lp)) return rc;
  if (!lp) return fail(WG_ERR_UNSUPPORTED, "wg_cheb_step_u: the LDS kernel does not apply to this handle");
  return launch_lds1_step(L, lp, k, u_km1, t_km1, k >= 2 ? t_km2 : nullptr, t_k, u_k, S, alpha0, alpha_k,
                          as_stream(stream_));
}

int wg_permute_rows(wg_laplacian_t L, int32_t direction, int64_t F, const float* src, float* dst, void* stream_) {
  if (!L || F < 1 || (direction != 0 && direction != 1) || (L->n_rows && (!src || !dst)))
    return fail(WG_ERR_INVALID, "wg_permute_rows: bad arguments");
  return launch_permute(L, direction, F, src, dst, as_stream(stream_));
}

}  // extern "C"

namespace wg {

void ChainGraph::release() {
  if (exec) (void)hipGraphExecDestroy(exec);
  if (fork) (void)hipEventDestroy(fork);
  if (join) (void)hipEventDestroy(join);
  if (cap) (void)hipStreamDestroy(cap);
  *this = ChainGraph{};
}

namespace {

// The whole graph_wavelet_features chain (WATS.py:39-74) enqueued on `stream`: permute in, K
// Chebyshev / Clenshaw steps, finalize.  Eager, or recorded into a hipGraph by the caller.
int wavelet_chain(wg_laplacian_t L, const float* X0, int64_t F, int32_t K, double s, float* S, float* H,
                  hipStream_t stream) {
  const int64_t n = L->n_rows;
  // small unweighted graphs, F == 1: the whole chain in one launch (chain.hip)
  if (F == 1 && K >= 1 && S && H) {
    ChainPlan* cp = nullptr;
    if (int rc0 = get_chain1_plan(L, F, K, &cp)) return rc0;
    if (cp) return launch_chain1(L, cp, X0, K, s, S, H, stream);
  }
  // F == 1 on an unweighted graph: the column-blocked LDS kernel (lds1.hip)
  Lds1Plan* lp = nullptr;
  if (F == 1 && K >= 1) {
    int rc0 = get_lds1_plan(L, /*active_only=*/true, &lp);
    if (rc0) return rc0;
  }
  // internal width: F padded to a multiple of 4 (zero columns) for float4 lanes
  const int64_t Fp = lp ? F : padded_features(L, F);
  // workspace: T ping-pong (2) + internal S [+ u ping-pong, padded to whole column blocks], 256-B aligned
  const size_t stride = ((size_t)n * Fp + 63) / 64 * 64;
  const size_t ustride = lp ? ((size_t)lp->u_floats() + 63) / 64 * 64 : 0;
  // the hybrid step (tiles.hip) gathers the first step's X0 value-free too, as u_0 = X0 * dinv
  TilePlan* tp0 = nullptr;  // the hybrid step's plan, when it applies (built here once, synchronous)
  if (!lp && L->tune.clenshaw && K >= 1 && L->unit && L->tune.uscale &&
      L->tune.hot == 0 && !L->tune.probe && tiles_wanted(L, Fp))
    if (int rc0 = get_tile_plan(L, /*active_only=*/true, Fp, &tp0)) return rc0;
  // the padded-CSR gathers (step.hip accumulate_u4) are value-free: the first step too, on u_0
  const bool g4 = !lp && !tp0 && L->tune.clenshaw && K >= 1 && L->unit && L->tune.uscale && L->tune.hot == 0 &&
                  gather4_applies(L, Fp) && step_single_tile(L, Fp, {L->ws});
  const bool u0 = tp0 != nullptr || g4;
  const size_t need = (u0 ? 4 : 3) * stride + 2 * ustride;
  if (L->ws_floats < need) {
    WG_HIP_TRY(hipStreamSynchronize(stream));
    (void)hipFree(L->ws);
    L->ws = nullptr;
    L->ws_floats = 0;
    WG_HIP_TRY(hipMalloc(&L->ws, need * sizeof(float)));
    L->ws_floats = need;
  }
  float* b0 = L->ws;               // T_0, then T_2, T_4, ... (in place)
  float* b1 = L->ws + stride;      // T_1, T_3, ...
  float* sint = L->ws + 2 * stride;
  // purely isolated rows (internal rows >= n_active) never enter the chain:
  // T_k = (-1)^k X0 exactly, so S = X0 * sum_k (-1)^k alpha_k (WATS.py:65-68)
  double coef = 0.0;
  for (int32_t k = 0; k <= K; ++k) coef += ((k & 1) ? -1.0 : 1.0) * std::exp(-s * (double)k);
  // finalize fused: the permute-in finishes the closed-form rows, the last step
  // writes S and H in the caller's order (no separate finalize pass)
  const bool fuse_fin = !lp && L->tune.fuse_finalize && Fp == F && K >= 1 && S && H &&
                        step_single_tile(L, F, {b0, b1, sint, S, H});
  // the first value-free Clenshaw step gathers u_0 = X0 * dinv: written by the same pass
  const bool u0_fused = fuse_fin && u0 && !lp && L->tune.clenshaw && K >= 1;
  // fold (tuning key "fold", default on): no permute-in pass at all.  The first step's team-kernel
  // launch gathers the caller's X0 through caller-row ids scaled by dinv (u_0 on the fly), reads its
  // own X0 rows at perm[row] and writes the internal X0 the later steps read, and finishes the
  // closed-form rows (team.hip cheb_team4_first_kernel): arxiv-size F = 40 -19.6 us of pass per chain
  // the first launch reads a float64 dinv per SELL id slot at twice the ids' 32-bit byte offset: the
  // slots (at most 2 nnz + 8 N with every row's padding) must stay within 2^31 bytes of it
  const bool fold_fits = 8 * (2 * L->nnz + 8 * n) < ((int64_t)1 << 31);
  const bool fold = u0_fused && g4 && !tp0 && L->tune.fold && L->tune.team && L->tune.uscale && fold_fits &&
                    pick_vec(F, {X0, b0, b1, sint, S, H}) == 4;
  const bool fold2 = fold && L->tune.fold == 2;  // a pass writes u_0 (internal order) only
  float* x0int = b0;  // the internal X0 the steps read (fold: written by the first launch)
  int rc = fold2 ? launch_permute_u0(L, F, X0, L->ws + 3 * stride, stream)
           : fold ? WG_OK
           : fuse_fin ? launch_permute_in_closed(L, F, X0, b0, coef, S, H, u0_fused ? L->ws + 3 * stride : nullptr,
                                                 stream)
                      : launch_permute_pad(L, F, Fp, X0, b0, stream);
  if (rc) return rc;
  if (K == 0) WG_HIP_TRY(hipMemcpyAsync(sint, b0, sizeof(float) * n * Fp, hipMemcpyDeviceToDevice, stream));
  if (lp) {
    float* u[2] = {L->ws + 3 * stride, L->ws + 3 * stride + ustride};  // u_{k-1} = T_{k-1} * dinv
    rc = launch_scale_dinv(L, lp->n, b0, u[0], stream);
    if (rc) return rc;
    for (int32_t k = 1; k <= K; ++k) {
      const float* xm1 = (k & 1) ? b0 : b1;
      const float* xm2 = (k == 1) ? nullptr : ((k & 1) ? b1 : b0);
      float* xk = (k == K) ? nullptr : ((k & 1) ? b1 : b0);
      rc = launch_lds1_step(L, lp, k, u[(k - 1) & 1], xm1, xm2, xk, (k == K) ? nullptr : u[k & 1], sint, 1.0,
                            std::exp(-s * (double)k), stream);
      if (rc) return rc;
    }
    return launch_finalize(L, F, sint, b0, coef, S, H, stream);
  }
  if (L->tune.clenshaw && K >= 1) {
    // Clenshaw's recurrence for S = sum_k c_k T_k(L_hat) X0, c_k = exp(-s k) (WATS.py:65-68):
    //   b_K = c_K X0 (never stored), b_k = c_k X0 + 2 L_hat b_{k+1} - b_{k+2} (k = K-1 .. 1),
    //   S = c_0 X0 + L_hat b_1 - b_2.
    // K SpMM steps as in the forward recurrence, but no S stream: each step reads X0 instead of
    // reading and writing S.  b_k is written in place over b_{k+2} (own rows only); the buffers
    // alternate so that b_1 sits in b1 and the final step may overwrite b_2 in sint.
    std::vector<double> c(K + 1);
    for (int32_t k = 0; k <= K; ++k) c[k] = std::exp(-s * (double)k);
    const float* bk1 = b0;           // b_{k+1} (b_K is implicit: c_K X0)
    float* bk2 = nullptr;            // b_{k+2} (nullptr: implicit, b_K, or 0)
    double cacc = 2.0 * c[K];        // the implicit b_K = c_K X0 enters through the SpMM scale
    float* bufs[2] = {(K & 1) ? sint : b1, (K & 1) ? b1 : sint};
    int nb = 0;
    // unweighted graphs: every stored b_k as u_k = b_k * dinv, so the gathers read no CSR values
    // (L_hat b = -dinv_i sum_j u_j); X0 itself stays unscaled (the first step reads the values)
    const int useu = (L->unit && L->tune.uscale && L->tune.hot == 0) ? 1 : 0;
    float* ub = u0 ? L->ws + 3 * stride : nullptr;  // u_0 = X0 * dinv (active rows)
    if (u0 && !u0_fused && !fold && (rc = launch_scale_rows(L, L->n_active, Fp, b0, ub, stream))) return rc;
    for (int32_t k = K - 1; k >= 1; --k) {
      float* out = bk2 ? bk2 : bufs[nb++];
      const double ck = c[k] - (bk2 == nullptr && k + 2 == K ? c[K] : 0.0);  // implicit b_{k+2} = c_K X0
      ClenArgs cl{x0int, ck, cacc, 0};
      cl.uin = useu && (bk1 != b0 || u0);
      cl.uprev = useu && bk2 != nullptr;
      cl.uout = useu;
      if (fold && bk1 == b0) {  // the first launch (fold): X0 in caller order, the internal copy written
        cl.x0c = X0;
        cl.x0i = x0int;
        cl.closed = TeamFirst{L->n_active, n, coef, S, H, !fold2};
      }
      rc = launch_step(L, 2, Fp, (bk1 == b0 && u0) ? (fold && !fold2 ? X0 : ub) : bk1, bk2, out, nullptr, nullptr, 1.0, 0.0,
                       stream, /*active_only=*/true, nullptr, &cl);
      if (rc) return rc;
      bk2 = const_cast<float*>(bk1 == b0 ? nullptr : bk1);
      bk1 = out;
      cacc = 2.0;
    }
    // final: S = c_0 X0 + L_hat b_1 - b_2 (K == 1: L_hat b_1 = c_1 L_hat X0; K == 2: b_2 = c_2 X0)
    const double c0 = c[0] - (K == 2 ? c[2] : 0.0);
    ClenArgs cl{x0int, c0, K == 1 ? c[1] : 1.0, 1};
    cl.uin = useu && (bk1 != b0 || u0);
    cl.uprev = useu && K >= 3;
    if (fold && bk1 == b0) {  // K == 1: the final step is the first launch
      cl.x0c = X0;
      cl.closed = TeamFirst{L->n_active, n, coef, S, H, !fold2};
    }
    rc = launch_step(L, 2, Fp, (bk1 == b0 && u0) ? (fold && !fold2 ? X0 : ub) : bk1, K >= 3 ? bk2 : nullptr, nullptr, sint, fuse_fin ? H : nullptr,
                     1.0, 0.0, stream, /*active_only=*/true, fuse_fin ? S : nullptr, &cl);
    if (rc) return rc;
  } else {
    for (int32_t k = 1; k <= K; ++k) {
      const float* xm1 = (k & 1) ? b0 : b1;
      const float* xm2 = (k == 1) ? nullptr : ((k & 1) ? b1 : b0);
      float* xk = (k == K) ? nullptr : ((k & 1) ? b1 : b0);  // T_K itself is never re-read
      const double ak = std::exp(-s * (double)k);             // WATS.py:65
      const bool last_fused = fuse_fin && k == K;
      rc = launch_step(L, k, Fp, xm1, xm2, xk, sint, last_fused ? H : nullptr, 1.0, ak, stream,
                       /*active_only=*/true, last_fused ? S : nullptr);
      if (rc) return rc;
    }
  }
  if (fuse_fin) return WG_OK;
  return launch_finalize(L, F, sint, b0, coef, S, H, stream, Fp);
}

}  // namespace
}  // namespace wg

extern "C" {

int wg_wavelet_features(wg_laplacian_t L, const float* X0, int64_t F, int32_t K, double s, float* S, float* H,
                        void* stream_) {
  if (!L || F < 1 || K < 0 || (!S && !H) || (L->n_rows && !X0))
    return fail(WG_ERR_INVALID, "wg_wavelet_features: bad arguments (F=%lld K=%d)", (long long)F, K);
  if (L->n_cols != L->n_rows)
    return fail(WG_ERR_INVALID, "wg_wavelet_features: sharded handle (halo columns); use wg_cheb_step");
  hipStream_t stream = as_stream(stream_);
  if (L->n_rows == 0) return WG_OK;
  if (int rc = chain1_check(L)) return rc;
  if (L->warm_gen != L->tune_gen) {  // a tune drops plans: every width builds again
    L->warm_widths.clear();
    L->warm_gen = L->tune_gen;
  }
  const bool warmed = std::find(L->warm_widths.begin(), L->warm_widths.end(), F) != L->warm_widths.end();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  WG_HIP_TRY(hipStreamIsCapturing(stream, &cs));
  if (cs != hipStreamCaptureStatusNone) {
    // the caller records the chain into its own graph: only widths whose plans and workspace
    // exist (plan building copies to the host and workspace growth synchronises)
    if (!warmed)
      return fail(WG_ERR_UNSUPPORTED,
                  "wg_wavelet_features: the first call with F=%lld builds its plans and workspace synchronously; "
                  "call it once on an uncaptured stream before capturing",
                  (long long)F);
    return wavelet_chain(L, X0, F, K, s, S, H, stream);
  }
  // small chains are launch-bound (PubMed-size: 19 launches of a few us): replay them as a hipGraph
  const int64_t work = std::max<int64_t>(L->nnz, 1) * padded_features(L, F);
  const bool use_graph = L->tune.graph == 1 || (L->tune.graph < 0 && work <= ((int64_t)1 << 22));
  if (!use_graph || L->prof || !warmed) {
    const int rc = wavelet_chain(L, X0, F, K, s, S, H, stream);
    if (!rc && !warmed) L->warm_widths.push_back(F);
    return rc;
  }
  ChainGraph& g = L->chain;
  if (g.x0 != X0 || g.S != S || g.H != H || g.ws != L->ws || g.F != F || g.K != K || g.s != s ||
      g.gen != L->tune_gen) {
    if (g.exec) {
      WG_HIP_TRY(hipStreamSynchronize(g.cap));
      (void)hipGraphExecDestroy(g.exec);
      g.exec = nullptr;
    }
    g.x0 = X0; g.S = S; g.H = H; g.ws = L->ws; g.F = F; g.K = K; g.s = s; g.gen = L->tune_gen;
    g.warm = 0;
  }
  if (!g.exec && g.warm < 2) {  // capture only arguments seen twice in a row (not alternating buffers)
    const int rc = wavelet_chain(L, X0, F, K, s, S, H, stream);
    if (!rc) ++g.warm;
    return rc;
  }
  if (!g.cap) {
    WG_HIP_TRY(hipStreamCreateWithFlags(&g.cap, hipStreamNonBlocking));
    WG_HIP_TRY(hipEventCreateWithFlags(&g.fork, hipEventDisableTiming));
    WG_HIP_TRY(hipEventCreateWithFlags(&g.join, hipEventDisableTiming));
  }
  // the chain runs on the handle's stream, joined to the caller's on both sides
  WG_HIP_TRY(hipEventRecord(g.fork, stream));
  WG_HIP_TRY(hipStreamWaitEvent(g.cap, g.fork, 0));
  if (!g.exec) {
    hipGraph_t gr = nullptr;
    WG_HIP_TRY(hipStreamBeginCapture(g.cap, hipStreamCaptureModeRelaxed));
    const int rc = wavelet_chain(L, X0, F, K, s, S, H, g.cap);
    const hipError_t ec = hipStreamEndCapture(g.cap, &gr);
    if (rc) {
      if (gr) (void)hipGraphDestroy(gr);
      return rc;
    }
    if (ec != hipSuccess) return fail(WG_ERR_HIP, "wg_wavelet_features: capture failed: %s", hipGetErrorString(ec));
    const hipError_t ei = hipGraphInstantiate(&g.exec, gr, nullptr, nullptr, 0);
    (void)hipGraphDestroy(gr);
    if (ei != hipSuccess) {
      g.exec = nullptr;
      return fail(WG_ERR_HIP, "wg_wavelet_features: graph instantiate: %s", hipGetErrorString(ei));
    }
  }
  WG_HIP_TRY(hipGraphLaunch(g.exec, g.cap));
  if (L->chain1) {  // the replay may hold the one-launch chain: wg_chain_status waits for this replay
    WG_HIP_TRY(hipEventRecord(L->chain1->done, g.cap));
    L->chain1->done_stale = false;
  }
  WG_HIP_TRY(hipEventRecord(g.join, g.cap));
  WG_HIP_TRY(hipStreamWaitEvent(stream, g.join, 0));
  return WG_OK;
}

#ifdef WG_TIMING_PROBES
// probe builds only (not in the ABI header): the recorded step-launch timeline, 4 x u64 per wave
int wg_probe_trace(wg_laplacian_t L, unsigned long long* host, int64_t n, int64_t* got) {
  if (!L || !got) return fail(WG_ERR_INVALID, "wg_probe_trace: NULL argument");
  WG_HIP_TRY(hipDeviceSynchronize());
  *got = std::min<int64_t>(n, L->trace_n);
  if (*got > 0 && host) WG_HIP_TRY(hipMemcpy(host, L->trace_buf, sizeof(unsigned long long) * *got, hipMemcpyDeviceToHost));
  return WG_OK;
}
#endif

int wg_chain_status(wg_laplacian_t L, int32_t* timed_out) {
  if (!L || !timed_out) return fail(WG_ERR_INVALID, "wg_chain_status: NULL argument");
  return chain1_status(L, timed_out);
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
    WG_HIP_TRY(hipEventSynchronize(L->ev[i + 1]));
    float ms = 0.0f;
    WG_HIP_TRY(hipEventElapsedTime(&ms, L->ev[i], L->ev[i + 1]));
    tot += ms;
    mx = std::max(mx, (double)ms);
  }
  *sum_ms = tot;
  *launches = (int64_t)(L->ev_used / 2);
  if (max_ms) *max_ms = mx;
  L->ev_used = 0;
  return WG_OK;
}

int wg_profile_durations(wg_laplacian_t L, double* ms, int64_t cap, int64_t* n) {
  if (!L || !n || (cap > 0 && !ms)) return fail(WG_ERR_INVALID, "wg_profile_durations: NULL argument");
  const int64_t have = (int64_t)(L->ev_used / 2);
  for (int64_t i = 0; i < have && i < cap; ++i) {
    WG_HIP_TRY(hipEventSynchronize(L->ev[2 * i + 1]));
    float t = 0.0f;
    WG_HIP_TRY(hipEventElapsedTime(&t, L->ev[2 * i], L->ev[2 * i + 1]));
    ms[i] = (double)t;
  }
  *n = have;
  L->ev_used = 0;
  return WG_OK;
}

int wg_row_l1_normalize(const float* S, float* H, int64_t n_rows, int64_t F, void* stream_) {
  if (n_rows < 0 || F < 1 || (n_rows && (!S || !H))) return fail(WG_ERR_INVALID, "wg_row_l1_normalize: bad arguments");
  if (n_rows == 0) return WG_OK;
  return launch_l1_normalize(S, H, n_rows, F, as_stream(stream_));
}

int wg_laplacian_map_rows(wg_laplacian_t L, int32_t direction, const int32_t* rows, int64_t n, int32_t* out,
                          void* stream_) {
  if (!L || n < 0 || (direction != 0 && direction != 1) || (n && (!rows || !out)))
    return fail(WG_ERR_INVALID, "wg_laplacian_map_rows: bad arguments");
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(map_rows_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream_), n,
                     direction == 0 ? L->iperm : L->perm, rows, out);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int wg_gather_rows(const float* src, const int32_t* rows, int64_t n, int64_t F, float* dst, void* stream_) {
  if (n < 0 || F < 1 || (n && (!src || !rows || !dst))) return fail(WG_ERR_INVALID, "wg_gather_rows: bad arguments");
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(ceil_div(n * F, 256)), dim3(256), 0, as_stream(stream_), n, F, rows, src,
                     dst);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // extern "C"
