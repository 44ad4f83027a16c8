// internal.h -- shared internals of libwats_hip (not part of the C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "wats_hip.h"

namespace wg {

int fail(int code, const char* fmt, ...);

// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) once per (kernel, current device):
// the attribute is per device, so a process-wide "done" flag would skip it on a second device
int ensure_dyn_lds(const void* fn, int bytes);
// compute units of device `dev` (cached per device)
int n_cus(int dev);

#define WG_HIP_TRY(expr)                                                                       \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return ::wg::fail(e_ == hipErrorOutOfMemory ? WG_ERR_OOM : WG_ERR_HIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                     \
  } while (0)

#define WG_LAUNCH_CHECK() WG_HIP_TRY(hipGetLastError())

// Device bounds checks of the debug variant (make VARIANT=debug EXTRA_FLAGS=-DWG_DEBUG_BOUNDS):
// gathered column ids against the gathered vector, wave descriptors against their plan, LDS indices
// against the staged sizes, halo rows against their slots.  A failed check prints where and what, then
// traps (the launch fails with a located message instead of a silent out-of-bounds access).  The shipped
// library compiles them out.
#ifdef WG_DEBUG_BOUNDS
#define WG_DCHECK(cond, fmt, ...)                                                                          \
  do {                                                                                                     \
    if (__builtin_expect(!(cond), 0)) {                                                                    \
      printf("WG_DEBUG_BOUNDS %s:%d block %d thread %d: " fmt "\n", __FILE__, __LINE__, (int)blockIdx.x,   \
             (int)threadIdx.x, ##__VA_ARGS__);                                                             \
      __builtin_trap();                                                                                    \
    }                                                                                                      \
  } while (0)
#else
#define WG_DCHECK(cond, fmt, ...) ((void)0)
#endif

constexpr int kBlock = 256;   // 4 waves of 64 lanes
constexpr int kMaxSeg = 24;
constexpr int kBuckets = 33;  // row-length buckets: b=0: len<=1; b>0: 2^(b-1) < len <= 2^b

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

template <typename T>
int dmalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  WG_HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return WG_OK;
}

// ---------------------------------------------------------------------------
// Step-kernel launch plan (per signal-tile shape), see step.hip.
// ---------------------------------------------------------------------------
struct Seg {
  int32_t begin;      // team mode: internal rows [begin, end); chunk mode: chunk ids
  int32_t end;
  int32_t blk_begin;  // first workgroup of this segment
  int32_t ln;         // team mode: lane sub-groups cooperating on one row
  int32_t mode;       // 0 = team, 1 = block (workgroup per row), 2 = split (workgroup per nnz chunk)
};

struct SegTable {
  Seg s[kMaxSeg];
  int32_t n;
  int32_t total_blocks;
};

struct ChunkDesc {  // one workgroup's share of a split row
  int32_t row;
  int32_t e0, e1;   // nnz range
  int32_t pad;
};

// the wave table of the value-free VEC-4 step as independent waves (team.hip)
struct TeamPlan {
  int4* wd = nullptr;        // device [2 * n_waves]: per wave {SELL offset, turns, row, LN | rows << 8 | part << 16},
                             // {part, parts, first slot, arrival counter}
  int4* sell = nullptr;      // device: the waves' column ids in SELL order (accumulate_sell)
  double* wpart = nullptr;   // device [n_slots][width]: long rows' float64 partials
  uint32_t* warr = nullptr;  // device [n_long]: arrival counters, reset by each row's last arrival
  int32_t n_waves = 0, n_slots = 0, n_long = 0, width = 0;
  int32_t max_parts = 0, npot_rows = 0;  // long rows: most parts; rows whose part count is not a power of 2
  int64_t n_sell = 0;        // int4 chunks in sell (its padding included)
  int64_t n_rows = 0;        // rows of the table ([0, n_rows): the debug variant checks descriptors against it)
  int4* sell0 = nullptr;     // device [n_sell]: sell with caller-row ids (the folded chain's first launch)
  double* sdinv = nullptr;   // device [4 n_sell]: dinv of each id slot of sell (0 for pads)
  void release();
};

struct Plan {
  SegTable tab{};
  int64_t row0 = 0, row1 = 0;   // the rows planned
  Seg* d_segs = nullptr;        // device copy of tab.s (read with scalar loads)
  int32_t n_chunks = 0;
  int32_t width = 0;            // LF * VEC doubles per partial
  int32_t nw = 4;               // waves per workgroup of the step kernel
  int32_t hot = 0;              // F == 1: columns [0, hot) of T_{k-1} staged in LDS (0 = off)
  int32_t n_split = 0;          // split rows = internal rows [0, n_split)
  ChunkDesc* chunks = nullptr;  // device [n_chunks]
  double* partial = nullptr;    // device [n_chunks][width]
  int2* rowchunks = nullptr;    // device [n_split] {first chunk, chunk count}
  uint32_t* arrivals = nullptr; // device [n_split] arrival counters, reset by each row's last arrival
  // value-free VEC-4 team waves (step.hip build_sell): each wave's column ids in SELL-G order --
  // turn t, chunk c (4 ids), sub-group g at sell[wmeta[w].x + (2 t + c) G + g] -- padded with
  // kPadCol to the wave's longest sub-group, wmeta[w] = {first chunk, turns} per wave w
  int2* wmeta = nullptr;        // device [total_blocks * nw]
  int4* sell = nullptr;         // device
  TeamPlan team;                // the same rows as independent waves (team.hip), lazily
  std::string text;
  void release();
};

// F == 1 column-blocked plan (lds1.hip): columns are dealt to NB blocks in
// 32-column chunks (chunk c -> block c % NB); each workgroup stages one
// block of the gather vector u = T_{k-1} * dinv in LDS and walks the entries
// of that block, stored block-major with 16-bit local column ids.
struct Lds1Plan {
  int32_t n = 0;              // rows
  int32_t n_cols = 0;         // column space
  int32_t nb = 0;             // column blocks
  int32_t lchunks = 0;        // 32-column chunks per block (LDS floats = 32 * lchunks)
  int32_t n_wg = 0;           // workgroups of the main kernel
  int32_t n_groups = 0;
  int64_t nnz = 0;
  int32_t* brp = nullptr;     // device [nb * n + 1]: block b row r = [brp[b*n+r], brp[b*n+r+1])
  uint16_t* bcol = nullptr;   // device [nnz + 8]: local column ids
  int2* groups = nullptr;     // device: {first row, rows | lanes-per-row << 16}
  // mode 4 (plain hub, tuning key "hub_sell"): the column ids in SELL-64 order -- per row
  // group, slot i * 64 + lane holds the id lane's team member reads in its i-th turn (pad:
  // kPadCol, lds1.hip), so every id load of a wave is one coalesced 256-B read
  int2* gsell = nullptr;      // device [n_groups]: {first 64-slot line, turns}
  int32_t* csell = nullptr;   // device [64 * lines]
  char sell_note[64] = "";
  int4* wgs = nullptr;        // device [n_wg]: {block, first group, end group, 0}
  float* part = nullptr;      // device: teams [nb * n] block partial sums (nb > 1); windows [n_pairs]
  // mode 2 (windows): (row, block) segments padded to 8-id chunks, bit 15 of a
  // segment's first id flags its start; one wave streams a contiguous chunk range
  int32_t mode = 1;           // 1 = row teams, 2 = chunk windows, 4 = hub teams
  int32_t hub = 0;            // mode 4: columns [0, hub) in LDS, the rest gathered from u
  int64_t ulen = 0;           // mode 4: floats of u (the column space, padded to 32)
  int64_t n_chunks = 0;
  int32_t n_pairs = 0;        // non-empty (row, block) segments
  uint4* chunk = nullptr;     // device [n_chunks]
  int32_t* pos = nullptr;     // device [nb * n]: segment id of (block, row), -1 if empty
  int4* wdesc = nullptr;      // device [n_wg * 16]: {first chunk, end chunk, first segment, 0}
  int32_t* wblock = nullptr;  // device [n_wg]: column block of each workgroup
  // mode 4 on a row shard: the hub is the highest-degree columns of the own range and of
  // each peer's halo group (prefixes: each is degree-ordered), staged from n_hranges
  // ranges; the kernel reads remapped columns hcol (hub column -> its LDS slot, any
  // other column c -> c + hub, gathered from u[c])
  int32_t* hcol = nullptr;    // device [nnz + 4]
  int4* hranges = nullptr;    // device [n_hranges]: {u begin, LDS slot begin, length, 0}
  int32_t n_hranges = 0;
  std::string text;
  void release();
  // floats of the gather vector u the kernel reads (padded column space)
  int64_t u_floats() const { return mode == 4 ? ulen : (int64_t)lchunks * nb * 32; }
};

// Hybrid step (tiles.hip) for wide signals on large unweighted graphs: internal rows in
// blocks of 64 or 128, columns in tiles of 32; each (row block, column tile) pair holding at
// least tile_th entries is a dense block, summed on the matrix cores from its row masks of
// 32 bits; the rest of each row (its "tail") comes first in the row's range of
// tcol and is gathered by the step kernel (phase 4), which adds the blocks' sums.
struct TilePlan {
  int64_t n_plan = 0;          // rows planned: [0, n_plan)
  int32_t rows = 64;           // rows per row block (64 or 128: 4 or 8 waves of 16 rows)
  int64_t col_limit = 0;       // column rows a block may read (rows >= col_limit of the tile read as 0)
  int32_t n_blocks = 0, n_items = 0, n_multi = 0, n_slots = 0;
  int64_t dense_nnz = 0;       // entries inside dense blocks
  int32_t* bct = nullptr;      // device [n_blocks]: column tile of each block
  uint32_t* bmask = nullptr;   // device [n_blocks][rows]: row masks (bit k = column 32 * tile + k)
  int4* items = nullptr;       // device [n_items]: {row block, first block, end block, slot or -1}
  int4* multi = nullptr;       // device [n_multi]: {row block, first slot, slots, 0}
  // the same blocks as work items of the fused launch (hybrid_fused_kernel: longer items beside the tail's
  // waves); equal to the set above when both sizes agree (an explicit tile_max)
  int32_t n_fitems = 0, n_fmulti = 0, n_fslots = 0;
  int4* fitems = nullptr;
  int4* fmulti = nullptr;
  int32_t* tcol = nullptr;     // device [nnz]: each row's tail entries first (the rest of its range unused)
  int32_t* tsplit = nullptr;   // device [n_rows]: end of each row's tail (== row end: no dense entries)
  int32_t width = 0;           // doubles per row of part / slots
  double* part = nullptr;      // device [n_rows][width]: the dense blocks' sums
  double* slots = nullptr;     // device [max(n_slots, n_fslots)][rows][width]
  // hybrid steps issued per form (captured launches count once, at capture): [0] sequential (the tile
  // kernel, then the tail with its epilogue), [1] two streams (the tail's sums beside the blocks), [2] fused
  // (hybrid_fused_kernel); wg_laplacian_describe names them
  int64_t form_launches[3] = {0, 0, 0};
  std::string text;
  void release();
};

struct Tuning {
  // 0 = shape-dependent default (see default_knobs in step.hip)
  int32_t iter = 0;          // team mode: target nonzeros per lane sub-group
  int32_t block_iter = 0;    // block mode: rows up to NW*G*block_iter nonzeros get one workgroup
  int32_t chunk_iter = 0;    // split mode: NW*G*chunk_iter nonzeros per workgroup chunk
  int32_t nt = -1;           // store hints: 4 = nt T_k / S stores, 8 = write-through (sc1) T_k stores;
                             // -1 = auto (8; step.hip)
  int32_t tile_f = 0;        // max signal columns per launch (0 = 64*VEC)
  int32_t bcast = 1;         // F > 1: sub-group cooperative index loads (ds_bpermute broadcast)
  int32_t vidx = -1;         // F == 1: 16-B aligned int4/float4 index loads; -1 = auto (on for nnz >= 16 M)
  int32_t waves = 4;         // waves per step-kernel workgroup: 4, 8 or 16
  int32_t hot = 0;           // F == 1: LDS hot-column cache size (columns), 0 = off
  int64_t seg_mask = -1;     // timing attribution only (-DWG_TIMING_PROBES): launch only these segments
  int32_t inkernel_combine = 1;  // split rows: last-arriving chunk combines (sc1 hand-off) vs combine_kernel
  int32_t lds = 3;           // F == 1, unit weights: LDS kernel (0 = off, 1 = row teams, 2 = chunk windows, 3 = auto)
  int32_t lds_cb = 32768;    // LDS floats per column block (multiple of 32, <= 40960)
  int32_t lds_iter = 8;      // target entries per lane per row team
  int32_t lds_wg = 0;        // workgroups of the LDS kernel (0 = auto)
  int32_t lds_maxnb = 16;    // largest block count the LDS kernel takes (else the gather kernel)
  int32_t lds_depth = 2;     // windows: 64-chunk windows in flight per wave (2, 4 or 8)
  int32_t lds_k = 4;         // windows: chunks per lane (1 = cheb_lds2_kernel, 2 / 4 = cheb_lds3_kernel)
  int32_t fuse_finalize = 1;  // wavelet_features: closed rows in the permute-in, S / H from the last step
  int32_t clenshaw = 1;      // wavelet_features (F > 1 / weighted): heat sum by Clenshaw's recurrence (no S stream)
  int32_t uscale = 1;        // Clenshaw on unweighted graphs: carry u = b * dinv, gathers read no CSR values
  int32_t hub_iter = 16;     // hub teams (lds mode 4): target entries per lane of a row team
  int32_t lds_perm = 1;      // windows: 1 = deal a segment's entries column-major over its chunks
  int32_t probe = 0;         // timing only (-DWG_TIMING_PROBES): gathers + one output stream, no epilogue
  int32_t hub_sell = 1;      // hub teams on plain hubs: column ids in SELL-64 order (coalesced id loads)
  int32_t xdelay = 0;        // timing only (-DWG_TIMING_PROBES): microseconds of simulated link time per
                             // sharded-chain exchange (one spinning wave on the stream)
  int32_t fpad = 0;          // internal signal width of F >= 3: 0 = auto (fewest cache lines per row), 4 / 8 / 16 = that multiple
  int32_t tiles = -1;        // hybrid step (tiles.hip): -1 = auto (unweighted, width % 16 == 0, >= 8 M nonzeros,
                             // >= 30 % of the entries in dense blocks), 0 = off, 1 = whenever it applies
  int32_t tile_th = 96;      // entries that make a (row block, 32-column tile) pair a dense block
  int32_t tile_max = 0;      // dense blocks per workgroup (longer row blocks split over slots);
                             // 0 = auto: 128 from 100 k rows, else 64 (tiles.hip, r02_s80-s81)
  int32_t tile_rows = 128;   // hybrid step: rows per row block (64 or 128)
  int32_t probe_tailwin = 0; // timing only (-DWG_TIMING_PROBES): the hybrid tail's columns folded into 1/n of them
  int32_t trace = 0;         // timing only (-DWG_TIMING_PROBES): record the trace-th step launch's per-wave timeline
  int32_t probe_h2 = 0;      // timing only (-DWG_TIMING_PROBES): see StepArgs
  int32_t probe_fold = 0;    // timing only (-DWG_TIMING_PROBES): see StepArgs
  int32_t probe_ns = 0;      // timing only (-DWG_TIMING_PROBES): Clenshaw epilogue row loads skipped (bits X0, b_{k+2})
  int32_t coldnt = 0;        // timing only (-DWG_TIMING_PROBES): team gathers of columns >= coldnt non-temporal
  int32_t tile_rg = 1;       // hybrid step, 128-row blocks: 16-row groups per wave (1: 8 waves, 2: 4 waves)
  int32_t tile_mfma = 0;     // hybrid step, 128-row blocks of width 48 / 64: 16 = v_mfma_f32_16x16x32_bf16,
                             // 32 = v_mfma_f32_32x32x16_bf16 (cheb_tiles32_kernel: each B read serves 32
                             // rows); 0 = auto (32 at width 64, else 16; tiles.hip launch_tiles)
  int32_t chain = -1;        // F == 1 small unweighted graphs: the whole chain in one launch (chain.hip); -1 = auto
                             // (<= 2^18 nonzeros, <= 24576 active rows), 0 = off, 1 = whenever it applies
  int32_t chain_wg = 0;      // chain.hip workers (workgroups of 1024 threads; doubled until a worker fits LDS);
                             // 0 = auto: one when its ids and two u buffers fit LDS (no exchange), else 64
                             // (PubMed-size K=16: 8 / 16 / 32 / 64 workers 187 / 139 / 119 / 113 us per chain,
                             // profiles/r03/s13_chain1_worker_sweep.log)
  int32_t chain_solo = 1;    // chain.hip: one workgroup, ids in registers (auto worker count only): 1 up to 2^15
                             // entries, 2 wherever it fits, 0 never
  int32_t chain_direct = 1;  // chain.hip: gathers read the granules straight from memory (no LDS staging of u)
  int32_t chain_xcd = 0;     // chain.hip: workers on one XCD (grid of 8 P, every 8th workgroup works; P <= 32)
  int32_t chain_fault = 0;   // chain.hip fault injection (tests of the timeout path): worker 0 does not publish
                             // phase chain_fault; the launch's S / H come out NaN and the next call fails
  int32_t gather4 = 21;      // value-free VEC-4 steps on the padded CSR (step.hip build_pcol / accumulate_u4):
                             // 0 = off, else 10 x chunks per turn + turns of ids in flight (21, 22, 31, 41)
  int32_t sell = 1;          // padded-CSR steps: team waves read their ids in SELL order (step.hip build_sell)
  int32_t team = 1;          // padded-CSR steps as independent waves (team.hip cheb_team4_kernel); 7 .. 13:
                             // register-budget / turn-size variants (team.hip launch_team4; all time the same)
                             // instead of Clenshaw's 3; 0 = Clenshaw
  int32_t fold = 1;          // wg_wavelet_features on the team kernel: no permute-in pass (the first launch
                             // gathers the caller's X0 scaled by dinv, writes the internal X0, finishes
                             // the closed-form rows; team.hip cheb_team4_first_kernel); 2 = a pass writes
                             // u_0 only (the first launch gathers it; the rest as 1); 0 = the full pass
  int32_t hyb_conc = 1;      // hybrid step with the team-kernel tail: the tail's row sums on a second stream
                             // beside the dense blocks, then one epilogue pass (step.hip); 1 = when the
                             // blocks leave the GPU half idle (tiles.hip hybrid_conc_applies), 2 = always;
                             // one fused launch where the tile shape allows, else (and with 3) two streams
  int32_t team_iter = 96;    // team.hip: target entries per lane sub-group
  int32_t hyb_iter = 128;    // the same for the hybrid step's tail (8 / 4 / 2-way Reddit-size shards and the
                             // whole graph, fused launch: 100.1 / 171.4 / 323.5 / 692 us per step vs 101.5 /
                             // 173.0 / 331.4 / 705 at 96, r05 s58-s65)
  int64_t team_tail = 8 << 20;  // the hybrid step's tail on the team kernel up to this many entries
  int32_t team_order = -1;   // team.hip: wave dispatch order (0 longest rows first, 1 reversed, 2 .. 7 mixed;
                             // -1 auto: 2 for plain steps, 0 for the hybrid step's tail)
  int32_t graph = 0;         // wg_wavelet_features: replay the chain as a hipGraph from its 3rd call with the same
                             // arguments (1 = on; -1 = small chains only, active nnz x width <= 2^22).  Off: the
                             // replay measured SLOWER than eager launches on this stack, +2.7 us per kernel node
                             // (PubMed K=16 145 vs 95 us, arxiv F=1 220 vs 170 us; profiles/r03/s3_graph_probe.log)
};

// The whole F = 1 chain of a small unweighted graph in one launch (chain.hip): P workgroups,
// each owning a cost-balanced range of active rows, u of every active row staged in LDS,
// a device-counter barrier between phases
constexpr int kChainMaxK = 64;
struct ChainPlan {
  int32_t P = 0, n_act = 0, lds_bytes = 0, ustride = 0;
  uint16_t* ids = nullptr;    // device [nnz_active]: 16-bit column ids in row order (P > 1: worker-local)
  uint16_t* wcols = nullptr;  // device: each worker's gathered columns, concatenated (P > 1)
  uint16_t* gids = nullptr;   // device [nnz_active]: global 16-bit column ids (direct mode)
  uint16_t* bcols = nullptr;  // device: each worker's back-edge columns, concatenated (P > 1)
  int32_t* bcol_off = nullptr;  // device [P + 1]
  int32_t* wcol_off = nullptr;  // device [P + 1]
  int4* wdesc = nullptr;      // device [P]: {row0, row1, e0, e1}
  int32_t* wpass = nullptr;   // device [P][17]: each worker's waves' ranges of passes
  int2* passes = nullptr;     // device: one wave pass {first row, rows | log2 team size << 8}
  int32_t* bar = nullptr;     // device [4]: [2] epoch + 1 of the last timed-out launch, [3] launch epoch
  int32_t* host_flag = nullptr;    // host-mapped (pinned): epoch of the last timed-out launch
  int32_t* d_host_flag = nullptr;  // its device address
  int32_t seen = 0;                // the host_flag value already reported
  hipEvent_t done = nullptr;       // recorded after every launch: chain1_status waits for it alone
  bool done_stale = false;         // the last launch was captured into a graph (its replay records done
                                   // when it is the handle's own, capi.hip; a caller's graph: a device sync)
  uint64_t* gbuf = nullptr;   // device [2][ustride]: tagged u granules {float bits, tag << 32}
  float* u0 = nullptr;        // device [n_act]: u_0 = X0 * dinv
  float* x0 = nullptr;        // device [n_act]: X0 in internal order
  // solo (one workgroup, chain.hip cheb_chain_solo_kernel): E register slots per lane
  int32_t solo_E = 0, solo_npass = 0;
  uint32_t* sids = nullptr;   // device [E / 2][threads]: two 16-bit LDS byte offsets (column * 4) per word
  int4* spass = nullptr;      // device: the waves' passes {first row, rows | log2 team size << 8, slots, 0}
  int32_t* swpass = nullptr;  // device [waves + 1]: each wave's pass range
  int32_t* swslots = nullptr; // device [waves]: the slots each wave uses
  std::string text;
  void release();
};

// wg_wavelet_features captured into a hipGraph (capi.hip): the launches of one chain, keyed by the
// call's arguments, the tuning generation and the workspace they were recorded with
struct ChainGraph {
  const void* x0 = nullptr;
  const void* S = nullptr;
  const void* H = nullptr;
  const void* ws = nullptr;
  int64_t F = 0;
  int32_t K = -1;
  double s = 0.0;
  int64_t gen = -1;
  int warm = 0;                   // eager calls with this key (the first builds plans and the workspace)
  hipGraphExec_t exec = nullptr;
  hipStream_t cap = nullptr;      // the handle's own non-blocking stream (capture and replay)
  hipEvent_t fork = nullptr, join = nullptr;
  void release();
};

}  // namespace wg

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
  unsigned int bucket[wg::kBuckets] = {0};  // rows per length bucket (internal rows sorted descending)
  int64_t avg_len = 0;
  int64_t n_active = 0;       // rows [0, n_active) enter the chain in wg_wavelet_features
  int64_t n_closed = 0;       // purely isolated rows at the end: T_k = (-1)^k X0 (closed form)
  wg::Tuning tune;
  int64_t tune_gen = 0;       // bumped by every wg_laplacian_tune: captured chains (dist.hip) re-capture
  std::map<int64_t, wg::Plan> plans;  // key: (LF * 8 + VEC) * 2 + active_only (...)
  // unweighted graph (every off-diagonal a_ij == 1): L_hat_ij = -dinv_i dinv_j
  // up to scipy's float32 rounding, so the F == 1 LDS kernel reads no values
  bool unit = false;
  bool cols_sorted = false;   // rows' entries in ascending internal column (sort_row_columns)
  bool values_null = false;   // created with values == NULL (unweighted by construction: every shard of the
                              // graph agrees, so a row-sharded chain may exchange u = b * dinv)
  double* dinv = nullptr;     // [n_cols] internal column order: 1 / sqrt(w_j) (w_j == 0 -> 1)
  unsigned long long* trace_buf = nullptr;  // -DWG_TIMING_PROBES timeline (knob "trace")
  int64_t trace_n = 0, trace_seq = 0;
  int32_t* prp = nullptr;     // padded CSR of the value-free VEC-4 gathers (build_pcol): row pointers
  int32_t* pcol = nullptr;    // ... and column ids, rows padded to multiples of 4 (lazily)
  std::vector<int64_t> halo_off;  // row shard: halo columns [n_rows + halo_off[q], n_rows + halo_off[q+1])
                                  // come from peer q, each group in descending degree (wg_dist_create)
  wg::Lds1Plan* lds1[2] = {nullptr, nullptr};  // [active_only]
  bool lds1_failed[2] = {false, false};        // not applicable (too many blocks): use the gather kernel
  wg::TilePlan* tiles[2] = {nullptr, nullptr};  // [active_only] hybrid step plans (released with lds1)
  bool tiles_failed[2] = {false, false};
  // workspace for wg_wavelet_features
  float* ws = nullptr;
  size_t ws_floats = 0;
  // widths F whose plans and workspace wg_wavelet_features has built (at tuning generation
  // warm_gen): only those may run on a stream the caller is capturing
  std::vector<int64_t> warm_widths;
  int64_t warm_gen = -1;
  wg::ChainGraph chain;  // small chains replayed as a hipGraph (tuning key "graph")
  wg::ChainPlan* chain1 = nullptr;  // the one-launch F = 1 chain (chain.hip), lazily
  bool chain1_failed = false;       // no plan (too large for resident workers / LDS): multi-launch path
  bool chain1_off = false;          // a launch timed out (the GPU is shared?): multi-launch path until a tune
  int32_t chain1_timeouts = 0;      // timed-out launches seen on this handle
  // the hybrid step's tail beside its dense blocks (tuning key hyb_conc): a second stream, its fork /
  // join events and the tail's float64 row sums
  hipStream_t side = nullptr;
  hipEvent_t side_fork = nullptr, side_join = nullptr;
  double* tsum = nullptr;
  int64_t tsum_n = 0;
  // live step-kernel timing (wg_profile_*)
  bool prof = false;
  std::vector<hipEvent_t> ev;  // pool of (start, stop) pairs
  size_t ev_used = 0;

  ~wg_laplacian_s();
};

namespace wg {
// prologue.hip
int build_operator(wg_laplacian_s* L, const int64_t* indptr, const int32_t* indices, const float* values,
                   const float* w_cols, bool raw, hipStream_t stream);
int sort_row_columns(wg_laplacian_s* L, hipStream_t stream);
// step.hip
int pick_vec(int64_t F, std::initializer_list<const void*> ptrs);
// hybrid: the plan of the hybrid step's tail (tiles.hip; its own key and larger work units)
int get_plan(wg_laplacian_s* L, int LF, int VEC, bool active_only, Plan** out, bool hybrid = false);
// S_out (finalize fused into the last step; needs S, H and F within one tile):
// the rows' final S and H go to caller row perm[row] of S_out / H
// Clenshaw form of the heat sum (wavelet_features): a step computes
//   out = ck * X0 + cacc * (L_hat . xm1) - xm2      (xm2 NULL = 0)
// into xk (final == 0), or into S [S_out / H] as the finished sum (final == 1).
// the folded chain's first launch (team.hip cheb_team4_first_kernel): closed-form rows and their outputs
struct TeamFirst {
  int64_t closed_from = 0, n_rows = 0;
  double coef = 0.0;
  float* S = nullptr;
  float* H = nullptr;
  bool gather_x0 = true;  // gathers of the caller's X0 scaled by dinv (else of u_0, from a pass)
};

struct ClenArgs {
  const float* x0;  // X0, internal order, same width / stride as the chain
  double ck;
  double cacc;
  int final_;
  // unweighted graphs (L->unit): the chain vectors as u = b * dinv (no CSR values read);
  // uin: xm1 is u, uprev: xm2 is u, uout: write u (not on the final step)
  int uin = 0, uprev = 0, uout = 0;
  // fold (the chain's first launch, team kernel only): gather the caller's X0 (x0c, caller rows) as
  // u = X0 * dinv on the fly, read the own X0 row at perm[row], write the internal X0 (x0i, read by
  // the later steps through x0), and finish the closed-form rows (closed.S / closed.H, caller order)
  const float* x0c = nullptr;
  float* x0i = nullptr;
  TeamFirst closed;
};
int launch_step(wg_laplacian_s* L, int32_t k, int64_t F, const float* xm1, const float* xm2, float* xk,
                float* S, float* H, double alpha0, double alpha_k, hipStream_t stream, bool active_only = false,
                float* S_out = nullptr, const ClenArgs* cl = nullptr);
int launch_finalize(wg_laplacian_s* L, int64_t F, const float* Sint, const float* X0int, double closed_coef,
                    float* S, float* H, hipStream_t stream, int64_t ldi = 0);  // ldi: internal row stride (0 = F)
// the internal signal width of an F-column chain: odd / 4-unaligned F >= 3 is
// padded to a multiple of 4 (zero columns), so the step kernel runs float4
// lanes (Reddit-size F = 41: 5383 -> 1878 us per step as F = 44)
int padded_features(const wg_laplacian_s* L, int64_t F);
// launch_step would run F columns as one tile (the condition for a fused H / finalize)
bool step_single_tile(wg_laplacian_s* L, int64_t F, std::initializer_list<const void*> ptrs);
// permute-in that also writes the closed-form rows' S and H in the caller's order
// u: also u_0 = X0 * dinv of the active rows (or nullptr); zero (a row shard's second exchange
// slot): the closed rows' u rows zeroed in u and in zero
int launch_permute_u0(wg_laplacian_s* L, int64_t F, const float* src, float* u, hipStream_t stream);
int launch_permute_in_closed(wg_laplacian_s* L, int64_t F, const float* src, float* dst, double coef, float* S,
                             float* H, float* u, hipStream_t stream, float* zero = nullptr);
// caller rows (stride F) -> internal rows (stride Fp), pad columns zeroed
int launch_permute_pad(wg_laplacian_s* L, int64_t F, int64_t Fp, const float* src, float* dst, hipStream_t stream);
int launch_permute(wg_laplacian_s* L, int direction, int64_t F, const float* src, float* dst, hipStream_t stream);
int build_pcol(wg_laplacian_s* L);
// team.hip: the wave table of rows [0, n) for LF-lane sub-groups, and its launch
// (dcol: the operator's column ids, or the hybrid step's tail-first copy, drsplit its rows' tail ends)
int build_team_waves(wg_laplacian_s* L, int64_t n, int LF, int iter, const int32_t* dcol,
                     const int32_t* drsplit, int order, TeamPlan* tp);
struct StepArgs;
int launch_team4(const TeamPlan& tp, const StepArgs& a, int variant, hipStream_t stream,
                 const TeamFirst* first = nullptr);
int build_team_first(wg_laplacian_s* L, TeamPlan* tp);
// the value-free VEC-4 gathers on the padded CSR apply to an F-wide (internal width) signal
bool gather4_applies(const wg_laplacian_s* L, int64_t F);
int launch_l1_normalize(const float* S, float* H, int64_t n, int64_t F, hipStream_t stream);
int prof_mark(wg_laplacian_s* L, hipStream_t stream, bool start);
// tiles.hip: the hybrid step's plan (*out = nullptr: not applicable) and its dense-block pass,
// which writes part = sum over the dense entries of u_j (value-free steps) for the planned rows
bool tiles_wanted(const wg_laplacian_s* L, int64_t F);
// the hybrid step runs its tail beside the dense blocks on a second stream (hyb_conc, a plan already built,
// not the fused launch's shape): a chain that would replay as a hipGraph runs eagerly instead (the
// captured fork / join replays slower, dist.hip)
bool hybrid_conc_in_use(const wg_laplacian_s* L, int64_t F);
bool hybrid_tail_on_team(const wg_laplacian_s* L, const TilePlan* tp, int64_t F);
bool hybrid_fused_shape(const wg_laplacian_s* L, const TilePlan* tp, int64_t F);
bool hybrid_conc_applies(const wg_laplacian_s* L, const TilePlan* tp, int64_t F);
int get_tile_plan(wg_laplacian_s* L, bool active_only, int64_t F, TilePlan** out);
int launch_tiles(wg_laplacian_s* L, TilePlan* p, int64_t F, const float* u, hipStream_t stream);
// the dense blocks and the team-kernel tail sums (a.tsum) in one launch, then the blocks' combine
// (WG_ERR_UNSUPPORTED: not the default tile shape)
int launch_hybrid_fused(wg_laplacian_s* L, TilePlan* p, int64_t F, const float* u, const TeamPlan& tp,
                        const StepArgs& a, hipStream_t stream);
void release_tiles(wg_laplacian_s* L);
// u = x * dinv for rows [0, n) of an F-wide signal (in place allowed): the hybrid chain's first
// step gathers u_0 = X0 * dinv value-free like every later step
int launch_scale_rows(wg_laplacian_s* L, int64_t n, int64_t F, const float* x, float* u, hipStream_t stream);
// chain.hip: the one-launch chain of a small graph (*out = nullptr: not applicable)
int get_chain1_plan(wg_laplacian_s* L, int64_t F, int32_t K, ChainPlan** out);
int launch_chain1(wg_laplacian_s* L, ChainPlan* p, const float* X0, int32_t K, double s, float* S, float* H,
                  hipStream_t stream);
void release_chain1(wg_laplacian_s* L);
int chain1_status(wg_laplacian_s* L, int32_t* timed_out);
// a launch timed out: the multi-launch path until the next tune; the tuning generation moves on, so a
// chain captured with the one-launch kernel (capi.hip ChainGraph) is dropped instead of replayed
void chain1_turn_off(wg_laplacian_s* L);
// WG_ERR_TIMEOUT (once) when a launch of the one-launch chain gave up a wait since the last report
int chain1_check(wg_laplacian_s* L);
// lds1.hip
int get_lds1_plan(wg_laplacian_s* L, bool active_only, Lds1Plan** out);  // *out = nullptr: not applicable
void release_lds1(wg_laplacian_s* L);
// u = x * dinv (float32), rows [0, n)
int launch_scale_dinv(wg_laplacian_s* L, int64_t n, const float* x, float* u, hipStream_t stream);
// one Chebyshev step, F == 1: gathers u_km1 (n_cols, padded to 32), own rows of t_km1 (iso), t_km2, writes t_k,
// u_k = t_k * dinv (nullable), S
int launch_lds1_step(wg_laplacian_s* L, Lds1Plan* p, int32_t k, const float* u_km1, const float* t_km1,
                     const float* t_km2, float* t_k, float* u_k, float* S, double alpha0, double alpha_k,
                     hipStream_t stream);
}  // namespace wg
