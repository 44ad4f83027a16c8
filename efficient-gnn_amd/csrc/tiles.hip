// tiles.hip -- the hybrid Chebyshev step for wide signals on large unweighted
// graphs: the dense part of L_hat on the matrix cores.
//
// On an unweighted graph the value-free Clenshaw step sums u_j = b_j * dinv_j
// over each row's columns (step.hip, reference calibration/WATS.py:32-36).  In
// descending-degree order the hub columns form dense blocks: on the Reddit-size
// R-MAT graph the (128-row block, 32-column tile) pairs holding >= 128 entries
// carry 78 % of the 114.6 M entries.  The gather kernel pays two L2 line
// requests per entry (a 192-B row of u each); a dense block instead reads its
// 32 rows of u once (6 KB, coalesced), shared by the 128 rows of the block.
//
//   part[row] = sum over the row's dense entries of u_j      (this file)
//   step      = cheb_step_kernel over the tail entries (each row's tail first in
//               tcol; its own plan, get_plan(hybrid)), + part, epilogue: phase 4
//               after the blocks (the tail on a side stream beside them measured
//               slower: Reddit-size F=41 1176 vs 1136 us, 8-way shard 158 vs 155)
//
// The block sum is a 128 x 32 by 32 x W product A.U with A a 0/1 matrix (exact in
// bf16).  U is split exactly into three bf16 pieces, u = hi + mid + lo
// (truncations: hi = u with the low 16 bits cleared, mid likewise of u - hi, and
// lo = u - hi - mid has at most 8 significant bits), so every product is exact
// and each v_mfma_f32_16x16x32_bf16 adds 32 of them in float32; the float32 sums
// of up to 4 blocks (<= 384 exact terms) are added to a float64 accumulator.
// Results differ from the all-float64 gather kernel by that float32 rounding
// only (6.7e-8 relative on Reddit-size F = 41; tests/test_tiles.py).
//
// Workgroup = 8 waves = one 128-row block (or a share of a long row block's
// dense blocks: those write float64 slots that tiles_combine_kernel sums in
// order).  Per dense block: the lanes load the 32 x W tile of u (float4) three
// tiles ahead in a register ring, split it into the three bf16 pieces in a
// double-buffered LDS image per piece (bank-conflict-free rows, img_row), and
// each wave multiplies its 16 rows: A fragments from a byte -> 8 x bf16 lookup
// table indexed by the row mask, B fragments by the transposed LDS read
// ds_read_b64_tr_b16 (two per fragment), three MFMAs (lo, mid, hi) per 16
// columns.  DESIGN.md 4.6 has the measurements and the variants kept as knobs.
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "internal.h"
#include "team_dev.h"

namespace wg {
namespace {

constexpr int kTC = 32;  // columns per tile (the MFMA's K)
constexpr int kItemMax = 1024;  // dense blocks per work item (tile_max <= 1024)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// LDS image of one bf16 piece of a 32-row tile: row r at dword r*S + X*bit3(r) + Y*bit4(r), so the
// transposed reads (two 16-lane groups of a 32-lane half read rows 8 apart) hit 64 distinct banks
// (searched exhaustively for each width; a plain [32][W] image is 2-way conflicted: 66 M
// SQ_LDS_BANK_CONFLICT cycles per launch, a third of the kernel, r02 pmc_tiles)
__host__ __device__ constexpr int img_s(int nfb) { return nfb == 1 ? 8 : nfb == 2 ? 16 : nfb == 3 ? 24 : 40; }
__host__ __device__ constexpr int img_x(int nfb) { return nfb == 2 ? 8 : 32; }
__host__ __device__ constexpr int img_y(int nfb) { return nfb == 2 ? 8 : nfb == 4 ? 24 : 32; }
__host__ __device__ constexpr int img_dwords(int nfb) { return 31 * img_s(nfb) + img_x(nfb) + img_y(nfb) + 8 * nfb; }
template <int NFB>
__device__ __forceinline__ int img_row(int r) {  // bf16 offset of row r
  return 2 * (r * img_s(NFB) + img_x(NFB) * ((r >> 3) & 1) + img_y(NFB) * ((r >> 4) & 1));
}

struct TileArgs {
  const float* u;        // gathered vector (rows = columns of L_hat), row stride ld
  int64_t ld;
  int64_t col_limit;     // rows of u that exist (tile rows beyond read as 0)
  int64_t n_plan;        // rows of part written
  const int32_t* bct;
  const uint32_t* bmask;
  const int4* items;
  double* part;          // [rows][ld]
  double* slots;         // [slot][rows per block][W]
#ifdef WG_DEBUG_BOUNDS
  int64_t dbg_blocks, dbg_slots;  // dense blocks and float64 slots of the plan
#endif
};

// u = hi + mid + lo exactly, each piece a bf16 (the high half of a float32)
__device__ __forceinline__ void split3(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
  const uint32_t hb = __float_as_uint(x) & 0xFFFF0000u;
  const float r1 = x - __uint_as_float(hb);
  const uint32_t mb = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(mb);
  h = hb >> 16;
  m = mb >> 16;
  l = __float_as_uint(r2) >> 16;
}

#ifndef WG_TILES_FLUSH  // computed tiles per float32 -> float64 flush of the block sums
#define WG_TILES_FLUSH 4  // 917 vs 928 us per step at 1 (Reddit-size F=41, r02_s70), same S to 1e-8
#endif
#ifndef WG_TILES_RING  // depth of the tile-load ring in barrier groups: 1 or 2 (3 spills at 80 VGPRs)
#define WG_TILES_RING 2
#endif
#ifndef WG_TILES_GROUP  // dense blocks multiplied per barrier (1 or 2; Reddit-size F = 41: 719 vs 726 us per
#define WG_TILES_GROUP 2  // step, tile kernel 278 vs 282 us, profiles/r03/s36_s39_tiles32)
#endif
#ifndef WG_TILES_MINW
#define WG_TILES_MINW 6
#endif
// NWV waves; FW = false: every wave multiplies all NFB column blocks for its RG groups of 16
// rows; FW = true: wave w multiplies column block w % NFB for RG row groups, so each B
// fragment read from LDS serves RG row groups (NFB * 8 / RG waves for 128 rows)
template <int NFB, int NWV, int RG, bool FW>
__device__ __forceinline__ void tiles_item(const TileArgs& t, int item) {
  constexpr int NRW = FW ? NWV / NFB : NWV;  // waves along the rows
  constexpr int NFW = FW ? 1 : NFB;          // column blocks per wave
  constexpr int TR = 16 * NRW * RG;    // rows per row block (RG groups of 16 per wave)
  constexpr int NT = 64 * NWV;         // threads
  constexpr int W = 16 * NFB;          // signal width
  constexpr int NV = kTC * W / 4;      // float4 per tile
  constexpr int PER = (NV + NT - 1) / NT;
  __shared__ uint4 lut[256];                                          // byte -> 8 bf16 (bit j ? 1.0 : 0)
  constexpr int PT = NFB < 4 ? WG_TILES_GROUP : 1;     // tiles per barrier group (width 64: VGPRs)
  constexpr int RD = PT == 1 ? WG_TILES_RING : 1;       // ring depth in groups
  static_assert(RD == 1 || RD == 2, "ring depth 1 or 2");
  __shared__ __attribute__((aligned(16))) uint16_t img[2][PT][3][2 * img_dwords(NFB)];  // [buffer][tile][piece hi/mid/lo][k, f]
  const int tid = threadIdx.x;
  for (int e = tid; e < 256; e += NT) {
    uint32_t d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d[q] = (((e >> (2 * q)) & 1) ? 0x3F80u : 0u) | (((e >> (2 * q + 1)) & 1) ? 0x3F800000u : 0u);
    lut[e] = make_uint4(d[0], d[1], d[2], d[3]);
  }
  const int4 it = t.items[item];
  const int64_t rb = it.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int rwave = FW ? wave / NFB : wave;        // the wave's slot along the rows
  const int fb0 = FW ? wave % NFB : 0;             // its first column block
  const int mrow = 16 * RG * rwave + (lane & 15);  // this lane's A row of row group 0 (of the block)
  const int mshift = 8 * (lane >> 4);              // its byte of the 32-bit row mask
  const int32_t b0 = it.y, n = it.z - it.y;  // n <= kItemMax (build_tile_plan)
  WG_DCHECK(b0 >= 0 && n >= 0 && n <= kItemMax && (int64_t)it.z <= t.dbg_blocks && it.w < (int)t.dbg_slots &&
                rb * TR < t.n_plan,
            "tile item %d: {%d, %d, %d, %d} outside %lld blocks / %lld slots / %lld rows", item, it.x, it.y, it.z, it.w,
            (long long)t.dbg_blocks, (long long)t.dbg_slots, (long long)t.n_plan);
  __shared__ int32_t sbct[kItemMax];         // the item's column tiles: no global load ahead of each tile load
  for (int e = tid; e < n; e += NT) {
    sbct[e] = t.bct[b0 + e];
    WG_DCHECK(sbct[e] >= 0 && (int64_t)sbct[e] * kTC < t.col_limit, "block %d: column tile %d past %lld columns",
              b0 + e, sbct[e], (long long)t.col_limit);
  }
  __syncthreads();

  // a tile's loads, in a register ring RD tiles deep: PER float4 of u (staged into LDS) and the
  // row masks of this lane's A rows (never staged: its A fragments are looked up before the
  // tile's barrier).  The loads are unconditional (threads past the tile and rows past
  // col_limit read a valid row, zeroed when staged) so that no branch makes the compiler wait
  // for them where they are issued.
  int koff[PER], kkv[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int v = (tid + i * NT) % NV;
    kkv[i] = v / (W / 4);
    koff[i] = (v % (W / 4)) * 4;
  }
  float4 xs[RD][PT][PER];
  uint32_t ws[RD][PT][RG] = {}, oks[RD][PT] = {};
  auto load = [&](float4 (&x)[PER], uint32_t (&w)[RG], uint32_t& ok, int32_t j) {
    const int64_t r0 = (int64_t)sbct[j] * kTC;
    ok = 0u;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int64_t r = r0 + kkv[i];
      ok |= (r < t.col_limit ? 1u : 0u) << i;
      x[i] = *reinterpret_cast<const float4*>(t.u + (r < t.col_limit ? r : t.col_limit - 1) * t.ld + koff[i]);
    }
#pragma unroll
    for (int g = 0; g < RG; ++g) w[g] = t.bmask[(int64_t)(b0 + j) * TR + mrow + 16 * g];
  };
  auto store = [&](const float4 (&x)[PER], uint32_t ok, int buf, int q) {
#ifdef WG_TILES_PROBE_NO_STORE  // timing attribution only (results wrong): the tile is loaded, not staged
    if (x[0].x == 12345.f) img[buf][q][0][tid] = 1;
    return;
#endif
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int v = tid + i * NT;
      if (v < NV) {
        const int kk = kkv[i], f = koff[i];
        const float4 xv = (ok >> i) & 1u ? x[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t h[4], m[4], l[4];
        split3(xv.x, h[0], m[0], l[0]);
        split3(xv.y, h[1], m[1], l[1]);
        split3(xv.z, h[2], m[2], l[2]);
        split3(xv.w, h[3], m[3], l[3]);
        const int o = img_row<NFB>(kk) + f;
        *reinterpret_cast<uint2*>(&img[buf][q][0][o]) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
        *reinterpret_cast<uint2*>(&img[buf][q][1][o]) = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
        *reinterpret_cast<uint2*>(&img[buf][q][2][o]) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
      }
    }
  };

  double acc[RG][NFW][4];
#pragma unroll
  for (int g = 0; g < RG; ++g)
#pragma unroll
    for (int fb = 0; fb < NFW; ++fb)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[g][fb][i] = 0.0;

  // transposed-read address of this lane: group q4 = lane >> 4 reads rows 8 q4 + q (+4), q = (lane & 15) >> 2,
  // columns 4 (lane & 3) .. +3 of each 16-column block
  const int trow = 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int tcolo = 4 * (lane & 3);
  const int tr_lo = img_row<NFB>(trow) + tcolo, tr_hi = img_row<NFB>(trow + 4) + tcolo;
  // float32 MFMA sums of the last <= WG_TILES_FLUSH computed tiles, added to the float64 acc
  f32x4 cacc[NFW][RG];
  int nacc = 0;
  auto flush = [&]() {
#pragma unroll
    for (int fb = 0; fb < NFW; ++fb)
#pragma unroll
      for (int g = 0; g < RG; ++g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[g][fb][i] += (double)cacc[fb][g][i];
        cacc[fb][g] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    nacc = 0;
  };
#pragma unroll
  for (int fb = 0; fb < NFW; ++fb)
#pragma unroll
    for (int g = 0; g < RG; ++g) cacc[fb][g] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf, int q, const bf16x8 (&a)[RG]) {
#pragma unroll
    for (int fw = 0; fw < NFW; ++fw) {
      const int fb = fb0 + fw;
      f32x4 (&c)[RG] = cacc[fw];
#pragma unroll
      for (int p = 2; p >= 0; --p) {  // lo, mid, hi: one B fragment read, RG row groups
#ifdef WG_TILES_PROBE_NO_TR  // timing attribution only (results wrong): no B reads from LDS
        const s16x4 lo4 = {(short)(p + fb), 0, 0, 0}, hi4 = {0, 0, 0, (short)lane};
#else
        const s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&img[buf][q][p][tr_lo + 16 * fb]));
        const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&img[buf][q][p][tr_hi + 16 * fb]));
#endif
        const s16x8 bv = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        const bf16x8 b = __builtin_bit_cast(bf16x8, bv);
#pragma unroll
        for (int g = 0; g < RG; ++g) {
#ifdef WG_TILES_PROBE_NO_MFMA  // timing attribution only (results wrong)
          c[g][0] += (float)b[0] * (float)a[g][1];
#else
          c[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[g], b, c[g], 0, 0, 0);
#endif
        }
      }
    }
    if (++nacc == WG_TILES_FLUSH) flush();
  };

  if (n <= 0) return;
  // every load unconditional (past the last tile: the last tile again), so the ring's registers
  // are written only by their loads and the compiler waits for each load only where it is staged
  // groups of PT tiles (the last group's missing tiles are never multiplied)
  const int32_t ng = (n + PT - 1) / PT;
  auto load_group = [&](int slot, int32_t g) {
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int32_t j = g * PT + q;
      load(xs[slot][q], ws[slot][q], oks[slot][q], j < n ? j : n - 1);
    }
  };
  auto store_group = [&](int slot, int buf) {
#pragma unroll
    for (int q = 0; q < PT; ++q) store(xs[slot][q], oks[slot][q], buf, q);
  };
#pragma unroll
  for (int r = 0; r < RD; ++r) load_group(r, r);
  store_group(0, 0);
  // group g (g % 2 == I): its A fragments looked up from register set I % RD, then (barrier) it
  // is multiplied from LDS buffer I % 2 while set I % RD is refilled with group g + RD; group
  // g + 1 is split into the other buffer after
  auto group = [&](auto I, int32_t g) {
    constexpr int i = decltype(I)::value;
    bf16x8 a[PT][RG];
    bool any[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      any[q] = false;
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        a[q][rg] = __builtin_bit_cast(bf16x8, lut[(ws[i % RD][q][rg] >> mshift) & 0xFFu]);
        any[q] = any[q] || ws[i % RD][q][rg] != 0u;
      }
      // some row of the wave has an entry in this tile (wave-uniform), and the tile exists
      any[q] = __any(any[q]) && g * PT + q < n;
    }
    __syncthreads();  // group g staged; the other buffer no longer read
    load_group(i % RD, g + RD < ng ? g + RD : ng - 1);
#pragma unroll
    for (int q = 0; q < PT; ++q)
      if (any[q]) compute(i % 2, q, a[q]);
    if (g + 1 < ng) store_group((i + 1) % RD, (i + 1) % 2);
  };
  for (int32_t g = 0; g < ng; g += 2) {
    group(std::integral_constant<int, 0>{}, g);
    if (g + 1 >= ng) break;
    group(std::integral_constant<int, 1>{}, g + 1);
  }
  if (nacc > 0) flush();
  // D layout of 16x16x32: column = lane & 15, row = 4 (lane >> 4) + i
#pragma unroll
  for (int g = 0; g < RG; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = 16 * (RG * rwave + g) + 4 * (lane >> 4) + i;
      const int64_t row = rb * TR + rl;
      if (it.w < 0 && row >= t.n_plan) continue;
      double* dst = it.w < 0 ? t.part + row * t.ld : t.slots + ((int64_t)it.w * TR + rl) * W;
#pragma unroll
      for (int fw = 0; fw < NFW; ++fw) dst[16 * (fb0 + fw) + (lane & 15)] = acc[g][fw][i];
    }
}

template <int NFB, int NWV, int RG, bool FW>
__global__ __launch_bounds__(64 * NWV, FW ? 2 : (NWV == 8 && NFB < 4 ? WG_TILES_MINW : 4)) void cheb_tiles_kernel(TileArgs t) {
  tiles_item<NFB, NWV, RG, FW>(t, (int)blockIdx.x);
}

// The hybrid step with its tail beside the dense blocks in ONE launch (tuning key hyb_conc): workgroups
// [0, n_items) are the tile kernel's items (128-row blocks, 8 waves), the rest are 8 team-kernel waves each
// summing rows' tails into a.tsum (team_wave with tsum: no epilogue).  Tiles first in dispatch order.  No
// stream fork / join (a captured or eager cross-stream join cost ~10 us per step, r05 s45-s46)
template <int NFB>
__global__ __launch_bounds__(512, NFB < 4 ? WG_TILES_MINW : 4) void hybrid_fused_kernel(TileArgs tt, TeamArgs ta,
                                                                                          int32_t n_items) {
  if ((int)blockIdx.x < n_items) {
    tiles_item<NFB, 8, 1, false>(tt, (int)blockIdx.x);
    return;
  }
  const int w = ((int)blockIdx.x - n_items) * 8 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w < ta.n_waves) team_wave<false, 2>(ta, w);
}

// The same product on v_mfma_f32_32x32x16_bf16 (tile_mfma = 32; widths 48 and 64, 128-row
// blocks).  Wave w multiplies rows 32 (w & 3) .. +31 by signal columns 32 (w >> 2) .. +31 (a
// 48-wide signal pads its second column block with zero columns whose sums are not stored):
// each B fragment (16 tile columns x 32 signal columns) read from LDS serves 32 rows instead of
// 16, so a tile costs 12 transposed reads per wave (48 KB per workgroup) against 18 (72 KB) at
// width 48 and 24 (96 KB) at width 64.  The LDS image rows are 96 bf16 (48 dwords) apart: the
// four rows a 16-lane group reads in one transposed read hit distinct banks.
constexpr int kImg32 = 96;  // bf16 per image row
#ifndef WG_TILES32_MINW
#define WG_TILES32_MINW 4  // 16 float64 sums per lane: 6 waves per SIMD (80 VGPRs) spills
#endif
template <int W>
__global__ __launch_bounds__(512, WG_TILES32_MINW) void cheb_tiles32_kernel(TileArgs t) {
  constexpr int NT = 512, TR = 128;
  constexpr int NV = kTC * W / 4;  // float4 per tile
  static_assert(NV <= NT && (W == 48 || W == 64), "one float4 of the tile per thread, two 32-column blocks");
  __shared__ uint4 lut[256];
  __shared__ __attribute__((aligned(16))) uint16_t img[2][3][kTC * kImg32];  // [buffer][piece][k * 96 + f]
  const int tid = threadIdx.x;
  for (int e = tid; e < 256; e += NT) {
    uint32_t d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d[q] = (((e >> (2 * q)) & 1) ? 0x3F80u : 0u) | (((e >> (2 * q + 1)) & 1) ? 0x3F800000u : 0u);
    lut[e] = make_uint4(d[0], d[1], d[2], d[3]);
  }
  if (W < 64)  // the padding columns W .. 63 of every image row: zero once (never stored to)
    for (int e = tid; e < 2 * 3 * kTC * (64 - W) / 8; e += NT) {
      const int q = e % ((64 - W) / 8), r = e / ((64 - W) / 8);  // r = (buffer, piece, k)
      *reinterpret_cast<uint4*>(&img[0][0][0] + r * kImg32 + W + 8 * q) = make_uint4(0u, 0u, 0u, 0u);
    }
  const int4 it = t.items[blockIdx.x];
  const int64_t rb = it.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int32_t b0 = it.y, n = it.z - it.y;
  WG_DCHECK(b0 >= 0 && n >= 0 && n <= kItemMax && (int64_t)it.z <= t.dbg_blocks && it.w < (int)t.dbg_slots,
            "tile item %d: {%d, %d, %d, %d} outside %lld blocks / %lld slots", (int)blockIdx.x, it.x, it.y, it.z, it.w,
            (long long)t.dbg_blocks, (long long)t.dbg_slots);
  __shared__ int32_t sbct[kItemMax];
  for (int e = tid; e < n; e += NT) sbct[e] = t.bct[b0 + e];
  __syncthreads();
  const int rgrp = wave & 3, nb = wave >> 2;
  const int mrow = 32 * rgrp + (lane & 31);  // this lane's A row: tile columns 8 (lane >> 5) + 0..7 (+16)
  const int mshift = 8 * (lane >> 5);
  // the load ring of cheb_tiles_kernel (unconditional loads, the lane's own row mask)
  constexpr int RD = WG_TILES_RING;
  const int kk = (tid % NV) / (W / 4), f = ((tid % NV) % (W / 4)) * 4;
  float4 xs[RD];
  uint32_t ws[RD] = {}, oks[RD] = {};
  auto load = [&](float4& x, uint32_t& w, uint32_t& ok, int32_t j) {
    const int64_t r = (int64_t)sbct[j] * kTC + kk;
    ok = r < t.col_limit ? 1u : 0u;
    x = *reinterpret_cast<const float4*>(t.u + (r < t.col_limit ? r : t.col_limit - 1) * t.ld + f);
    w = t.bmask[(int64_t)(b0 + j) * TR + mrow];
  };
  auto store = [&](const float4& x0, uint32_t ok, int buf) {
    if (tid < NV) {
      const float4 x = ok ? x0 : make_float4(0.f, 0.f, 0.f, 0.f);
      uint32_t h[4], m[4], l[4];
      split3(x.x, h[0], m[0], l[0]);
      split3(x.y, h[1], m[1], l[1]);
      split3(x.z, h[2], m[2], l[2]);
      split3(x.w, h[3], m[3], l[3]);
      const int o = kk * kImg32 + f;
      *reinterpret_cast<uint2*>(&img[buf][0][o]) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
      *reinterpret_cast<uint2*>(&img[buf][1][o]) = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
      *reinterpret_cast<uint2*>(&img[buf][2][o]) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
    }
  };

  // B fragment of k-half h: lane holds tile columns k = 16 h + 8 (lane >> 5) + 0..7 of signal column
  // 32 nb + (lane & 31); its 16-lane group reads rows k0 + (lane & 15) / 4 (+4), 4 columns each
  const int tr_lo = (8 * (lane >> 5) + ((lane & 15) >> 2)) * kImg32 + 32 * nb + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const int tr_hi = tr_lo + 4 * kImg32;
  double acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0;
  f32x16 cacc = {};
  int nacc = 0;
  auto compute = [&](int buf, const bf16x8& a0, const bf16x8& a1) {
#pragma unroll
    for (int p = 2; p >= 0; --p) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const s16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&img[buf][p][tr_lo + 16 * h * kImg32]));
        const s16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&img[buf][p][tr_hi + 16 * h * kImg32]));
        const s16x8 bv = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        cacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(h ? a1 : a0, __builtin_bit_cast(bf16x8, bv), cacc, 0, 0, 0);
      }
    }
    if (++nacc == WG_TILES_FLUSH) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] += (double)cacc[i];
      cacc = f32x16{};
      nacc = 0;
    }
  };

  if (n <= 0) return;
  // every load unconditional (past the last tile: the last tile again), so the ring's registers
  // are written only by their loads and the compiler waits for each load only where it is staged
#pragma unroll
  for (int q = 0; q < RD; ++q) load(xs[q], ws[q], oks[q], q < n ? q : n - 1);
  store(xs[0], oks[0], 0);
  auto tile = [&](auto I, int32_t j) {
    constexpr int i = decltype(I)::value;
    const uint32_t mw = ws[i % RD];
    const bf16x8 a0 = __builtin_bit_cast(bf16x8, lut[(mw >> mshift) & 0xFFu]);
    const bf16x8 a1 = __builtin_bit_cast(bf16x8, lut[(mw >> (16 + mshift)) & 0xFFu]);
    const bool any = __any(mw != 0u);
    __syncthreads();
    load(xs[i % RD], ws[i % RD], oks[i % RD], j + RD < n ? j + RD : n - 1);
    if (any) compute(i % 2, a0, a1);
    if (j + 1 < n) store(xs[(i + 1) % RD], oks[(i + 1) % RD], (i + 1) % 2);
  };
  for (int32_t j = 0; j < n; j += 6) {
    tile(std::integral_constant<int, 0>{}, j);
    if (j + 1 >= n) break;
    tile(std::integral_constant<int, 1>{}, j + 1);
    if (j + 2 >= n) break;
    tile(std::integral_constant<int, 2>{}, j + 2);
    if (j + 3 >= n) break;
    tile(std::integral_constant<int, 3>{}, j + 3);
    if (j + 4 >= n) break;
    tile(std::integral_constant<int, 4>{}, j + 4);
    if (j + 5 >= n) break;
    tile(std::integral_constant<int, 5>{}, j + 5);
  }
  if (nacc > 0)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] += (double)cacc[i];
  // D layout of 32x32x16: column = lane & 31, row = 8 (i / 4) + 4 (lane >> 5) + i % 4
  const int col = 32 * nb + (lane & 31);
  if (col >= W) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int rl = 32 * rgrp + 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
    const int64_t row = rb * TR + rl;
    if (it.w < 0 && row >= t.n_plan) continue;
    double* dst = it.w < 0 ? t.part + row * t.ld : t.slots + ((int64_t)it.w * TR + rl) * W;
    dst[col] = acc[i];
  }
}

// row blocks split over several workgroups: part = their slots summed in slot order
// (blockIdx.y = the split row block, blockIdx.x = 256 of its 64 * W sums; the slot loads
// are independent, four in flight per thread)
template <int W>
__global__ __launch_bounds__(256) void tiles_combine_kernel(const int4* __restrict__ multi, const double* __restrict__ slots,
                                                            double* __restrict__ part, int64_t ld, int64_t n_plan, int TR) {
  const int4 mt = multi[blockIdx.y];
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= TR * W) return;
  const int rl = e / W, f = e - rl * W;
  const int64_t row = (int64_t)mt.x * TR + rl;
  if (row >= n_plan) return;
  const double* p = slots + ((int64_t)mt.y * TR + rl) * W + f;
  const int64_t step = (int64_t)TR * W;
  double s = 0.0;
  int q = 0;
  for (; q + 4 <= mt.z; q += 4) {
    const double v0 = p[q * step], v1 = p[(q + 1) * step], v2 = p[(q + 2) * step], v3 = p[(q + 3) * step];
    s += v0;
    s += v1;
    s += v2;
    s += v3;
  }
  for (; q < mt.z; ++q) s += p[q * step];
  part[row * ld + f] = s;
}

// u = x * dinv row-wise (float64 product rounded once, as the step epilogue stores u)
__global__ void scale_rows_kernel(int64_t n, int64_t F, const float* __restrict__ x, const double* __restrict__ dinv,
                                  float* __restrict__ u) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * F) return;
  u[i] = (float)((double)x[i] * dinv[i / F]);
}

template <typename T>
int upload(T** d, const std::vector<T>& h) {
  if (int rc = dmalloc(d, h.size())) return rc;
  if (!h.empty()) WG_HIP_TRY(hipMemcpy(*d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return WG_OK;
}

int build_tile_plan(wg_laplacian_s* L, bool active_only, TilePlan* p) {
  const int64_t n = L->n_rows, nnz = L->nnz;
  const int64_t n_plan = active_only ? L->n_active : n;
  // closed-form rows are never gathered: on a whole graph they end the column space; on a row shard
  // they sit between the active own rows and the halo (dist.hip keeps their u rows zero)
  const int64_t col_limit = (active_only && L->n_cols == L->n_rows) ? L->n_active : L->n_cols;
  const int th = std::max(1, L->tune.tile_th);
  int tmax = L->tune.tile_max;  // <= 0: auto (below)
  const int kTR = L->tune.tile_rows == 128 ? 128 : 64;
  p->rows = kTR;
  std::vector<int32_t> rp(n + 1), col(nnz);
  WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr, sizeof(int32_t) * (n + 1), hipMemcpyDeviceToHost));
  WG_HIP_TRY(hipMemcpy(col.data(), L->col, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
  const int64_t n_ct = ceil_div(L->n_cols, kTC);
  std::vector<int32_t> cnt(n_ct, 0), sel(n_ct, -1), touched, tmp;
  std::vector<int32_t> bct, tcol(col), tsplit(n);
  std::vector<uint32_t> bmask;
  std::vector<int4> items, multi;
  std::vector<int2> rbs;  // row blocks with dense blocks: {row block, first block}
  int32_t n_slots = 0;
  int64_t dense = 0;
  for (int64_t r = n_plan; r < n; ++r) tsplit[r] = rp[r + 1];  // unplanned rows: all tail
  const int64_t n_rb = ceil_div(n_plan, kTR);
  for (int64_t rb = 0; rb < n_rb; ++rb) {
    const int64_t r0 = rb * kTR, r1 = std::min<int64_t>(r0 + kTR, n_plan);
    touched.clear();
    for (int64_t r = r0; r < r1; ++r)
      for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
        const int32_t c = col[e];
        if (c < 0 || c >= col_limit) return fail(WG_ERR_INVALID, "tiles: column %d of row %lld outside [0, %lld)", c,
                                                 (long long)r, (long long)col_limit);
        if (cnt[c / kTC]++ == 0) touched.push_back(c / kTC);
      }
    std::sort(touched.begin(), touched.end());
    const int32_t first = (int32_t)bct.size();
    for (int32_t ct : touched)
      if (cnt[ct] >= th) {
        sel[ct] = (int32_t)bct.size();
        bct.push_back(ct);
      }
    bmask.resize(bct.size() * kTR, 0u);
    for (int64_t r = r0; r < r1; ++r) {
      tmp.clear();
      for (int32_t e = rp[r]; e < rp[r + 1]; ++e) {
        const int32_t c = col[e];
        const int32_t s = sel[c / kTC];
        if (s >= 0) {
          uint32_t& w = bmask[(size_t)s * kTR + (r - r0)];
          const uint32_t bit = 1u << (c % kTC);
          if (w & bit) {  // a repeated entry: a row mask cannot count it twice -- keep the gather kernel
            p->n_blocks = 0;
            return WG_OK;
          }
          w |= bit;
          ++dense;
        } else {
          tmp.push_back(c);
        }
      }
      if (L->tune.probe_tailwin > 0) {  // timing probe only (results wrong): every tail column folded
        const int64_t win = std::max<int64_t>(1, col_limit / L->tune.probe_tailwin);  // into one window
        for (auto& c : tmp) c = (int32_t)(col_limit / 2 + c % win < col_limit ? col_limit / 2 + c % win : c % win);
      }
      tsplit[r] = rp[r] + (int32_t)tmp.size();
      std::copy(tmp.begin(), tmp.end(), tcol.begin() + rp[r]);
    }
    for (int32_t ct : touched) {
      cnt[ct] = 0;
      sel[ct] = -1;
    }
    const int32_t nb = (int32_t)bct.size() - first;
    if (nb > 0) rbs.push_back(make_int2((int)rb, first));  // nb == 0: every entry is tail, no part added
  }
  // work items: a row block's dense blocks, split over several workgroups (slots) past tmax, one list
  // per form (the plan serves every width; hybrid_fused_shape picks the form per width at launch).  Auto
  // (tile_max <= 0) for the sequential and two-stream steps: 128 blocks per workgroup from 100 k rows, else 64
  // (Reddit-size F=41, width 48, us per step: whole graph 726 at 128 vs 735 at 192, 2-way shard 369 vs
  // 382; smaller shards want more workgroups, profiles/r02/s80-s81).  Where the fused launch takes the
  // plan (hybrid_fused_kernel: the tail's waves fill the GPU beside the items) fewer, longer items pay,
  // about n_plan / 310 blocks each: 8-way shard 101.6 at 96 vs 103.9 at 64 and 103.0 at 112, 4-way 173
  // at 128-192 vs 212.8 at 64 and 196 at 256, 2-way 326-331 at 384 vs 340 at 320 and 368-371 at 512,
  // whole graph 692-694 at 640-768 vs 705 at 512 and 745 at 1024 (r05 s55-s65)
  const int64_t nblk = (int64_t)bct.size();
  // one item list per form: {items, multi, slots}
  auto make_items = [&](int tm, std::vector<int4>& its, std::vector<int4>& mul) {
    tm = std::max(1, std::min(tm, kItemMax));
    int32_t ns = 0;
    for (size_t q0 = 0; q0 < rbs.size(); ++q0) {
      const int rb = rbs[q0].x, first = rbs[q0].y;
      const int32_t nb = (int32_t)((q0 + 1 < rbs.size() ? rbs[q0 + 1].y : nblk) - first);
      const int32_t k = (nb + tm - 1) / tm;
      if (k == 1) {
        its.push_back(make_int4(rb, first, first + nb, -1));
      } else {
        for (int32_t q = 0; q < k; ++q)
          its.push_back(make_int4(rb, first + (int32_t)((int64_t)nb * q / k), first + (int32_t)((int64_t)nb * (q + 1) / k),
                                  ns + q));
        mul.push_back(make_int4(rb, ns, k, 0));
        ns += k;
      }
    }
    return ns;
  };
  const int tseq = tmax > 0 ? tmax : (n_plan >= 100000 ? 128 : 64);
  const int tfus = tmax > 0 ? tmax : (int)std::min<int64_t>(kItemMax, std::max<int64_t>(96, n_plan / 310 / 16 * 16));
  n_slots = make_items(tseq, items, multi);
  std::vector<int4> fitems, fmulti;
  // the fused launch's items only where its tile shape can apply (hybrid_fused_shape decides per width)
  const bool fused_possible = kTR == 128 && L->tune.tile_rg == 1 && L->tune.team && L->tune.hyb_conc &&
                              L->tune.hyb_conc != 3;
  int32_t n_fslots = 0;
  if (fused_possible && tfus != tseq) n_fslots = make_items(tfus, fitems, fmulti);
  p->n_plan = n_plan;
  p->col_limit = col_limit;
  p->n_blocks = (int32_t)bct.size();
  p->n_items = (int32_t)items.size();
  p->n_multi = (int32_t)multi.size();
  p->n_slots = n_slots;
  p->dense_nnz = dense;
  int rc = upload(&p->bct, bct);
  if (!rc) rc = upload(&p->bmask, bmask);
  if (!rc) rc = upload(&p->items, items);
  if (!rc) rc = upload(&p->multi, multi);
  if (fitems.empty()) {  // the fused launch walks the same items
    p->fitems = p->items;
    p->fmulti = p->multi;
    p->n_fitems = p->n_items;
    p->n_fmulti = p->n_multi;
    p->n_fslots = p->n_slots;
  } else {
    if (!rc) rc = upload(&p->fitems, fitems);
    if (!rc) rc = upload(&p->fmulti, fmulti);
    p->n_fitems = (int32_t)fitems.size();
    p->n_fmulti = (int32_t)fmulti.size();
    p->n_fslots = n_fslots;
  }
  if (!rc) rc = upload(&p->tcol, tcol);
  if (!rc) rc = upload(&p->tsplit, tsplit);
  if (rc) return rc;
  char buf[256];
  snprintf(buf, sizeof(buf), "tiles: %d dense blocks (%dx32, >= %d entries) hold %lld of %lld entries (%.1f %%); %d items, %d split row blocks (fused launch: %d items, %d split)\n",
           p->n_blocks, kTR, th, (long long)dense, (long long)nnz, nnz ? 100.0 * dense / nnz : 0.0, p->n_items, p->n_multi,
           p->n_fitems, p->n_fmulti);
  p->text = buf;
  return WG_OK;
}

}  // namespace

void TilePlan::release() {
  (void)hipFree(bct);
  (void)hipFree(bmask);
  if (fitems != items) (void)hipFree(fitems);
  if (fmulti != multi) (void)hipFree(fmulti);
  (void)hipFree(items);
  (void)hipFree(multi);
  fitems = nullptr;
  fmulti = nullptr;
  (void)hipFree(tcol);
  (void)hipFree(tsplit);
  (void)hipFree(part);
  (void)hipFree(slots);
  bct = nullptr;
  bmask = nullptr;
  items = nullptr;
  multi = nullptr;
  tcol = nullptr;
  tsplit = nullptr;
  part = nullptr;
  slots = nullptr;
  width = 0;
}

void release_tiles(wg_laplacian_s* L) {
  for (int i = 0; i < 2; ++i) {
    if (L->tiles[i]) {
      L->tiles[i]->release();
      delete L->tiles[i];
      L->tiles[i] = nullptr;
    }
    L->tiles_failed[i] = false;
  }
}

int launch_scale_rows(wg_laplacian_s* L, int64_t n, int64_t F, const float* x, float* u, hipStream_t stream) {
  if (n <= 0) return WG_OK;
  if (n > L->n_cols) return fail(WG_ERR_INVALID, "launch_scale_rows: %lld rows > %lld columns", (long long)n,
                                 (long long)L->n_cols);
  hipLaunchKernelGGL(scale_rows_kernel, dim3((unsigned)ceil_div(n * F, 256)), dim3(256), 0, stream, n, F, x, L->dinv, u);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

bool tiles_wanted(const wg_laplacian_s* L, int64_t F) {
  if (L->tune.tiles == 0 || !L->unit || !L->reordered || F % 16 != 0 || F > 64) return false;
  return L->tune.tiles == 1 || L->nnz >= ((int64_t)8 << 20);
}

// the hybrid step's tail on the team kernel: up to team_tail entries in the sequential step (larger tails
// keep the workgroup kernel's tiered plan), any length where the fused launch takes the step (Reddit-size
// F = 41, us per step against the sequential workgroup tail: 2-way shard, 12.1 M tail entries, 323.5 vs
// 368.3; one GPU, 24.2 M, 692 vs 722 -- with longer tile items and hyb_iter 128, r05 s59-s65)
bool hybrid_tail_on_team(const wg_laplacian_s* L, const TilePlan* tp, int64_t F) {
  if (!tp || !L->tune.team) return false;
  if (L->nnz - tp->dense_nnz <= L->tune.team_tail) return true;
  return L->tune.hyb_conc && hybrid_fused_shape(L, tp, F);
}

bool hybrid_conc_applies(const wg_laplacian_s* L, const TilePlan* tp, int64_t F) {
  if (!tp || !L->tune.hyb_conc || !hybrid_tail_on_team(L, tp, F)) return false;
  if (L->tune.hyb_conc >= 2) return true;
  // auto: the one-launch form wherever its tile shape applies (Reddit-size F = 41 shards, step alone:
  // 8-way 102.0-102.5 vs 131.4-133.5 us, 4-way 208.4-209.3 vs 220.6, r05 s47-s48); the two-stream form
  // only for a plan whose dense blocks leave the GPU half idle (fewer work items than two per CU: the
  // 8-way shard 156.5 vs 168.7 us per step with its exchange, the 4-way one slower beside: 262.7 vs
  // 251.0, r05 s37-s38)
  if (hybrid_fused_shape(L, tp, F)) return true;
  return (int64_t)tp->n_items < 2 * (int64_t)n_cus(L->device);
}

// the fused launch's tile shape: 128-row blocks, one 16-row group per wave, the 16x16x32 MFMA
bool hybrid_fused_shape(const wg_laplacian_s* L, const TilePlan* tp, int64_t F) {
  const int shape = L->tune.tile_mfma > 0 ? L->tune.tile_mfma : (F == 64 ? 32 : 16);
  return tp && tp->rows == 128 && L->tune.tile_rg == 1 && shape == 16 && F % 16 == 0 && F <= 64 &&
         L->tune.hyb_conc != 3;
}

// a chain whose hybrid step forks a second stream (not the fused launch) runs eagerly
bool hybrid_conc_in_use(const wg_laplacian_s* L, int64_t F) {
  if (!tiles_wanted(L, F)) return false;
  const int64_t Fp = F + (-F % 16 + 16) % 16;  // the width the hybrid step runs at
  for (const TilePlan* tp : L->tiles)
    if (hybrid_conc_applies(L, tp, Fp) && !hybrid_fused_shape(L, tp, Fp)) return true;
  return false;
}

int get_tile_plan(wg_laplacian_s* L, bool active_only, int64_t F, TilePlan** out) {
  *out = nullptr;
  active_only = active_only && L->reordered;
  const int ai = active_only ? 1 : 0;
  if (L->tiles_failed[ai]) return WG_OK;
  if (!L->tiles[ai]) {
    auto* p = new TilePlan();
    int rc = build_tile_plan(L, active_only, p);
    if (rc) {
      p->release();
      delete p;
      return rc;
    }
    // auto: worth it only when the dense blocks carry a good share of the entries
    if (p->n_blocks == 0 || (L->tune.tiles < 0 && p->dense_nnz * 10 < L->nnz * 3)) {
      p->release();
      delete p;
      L->tiles_failed[ai] = true;
      return WG_OK;
    }
    L->tiles[ai] = p;
  }
  TilePlan* p = L->tiles[ai];
  if (p->width < F) {  // part / slots for this width
    (void)hipFree(p->part);
    (void)hipFree(p->slots);
    p->part = nullptr;
    p->slots = nullptr;
    p->width = 0;
    int rc = dmalloc(&p->part, (size_t)std::max<int64_t>(1, L->n_rows) * F);
    if (!rc) rc = dmalloc(&p->slots, (size_t)std::max(1, std::max(p->n_slots, p->n_fslots)) * p->rows * F);
    if (rc) return rc;
    p->width = (int32_t)F;
  }
  *out = p;
  return WG_OK;
}

namespace {
TileArgs tile_args(const TilePlan* p, int64_t F, const float* u, bool fused = false) {
  TileArgs t{};
  t.u = u;
  t.ld = F;
  t.col_limit = p->col_limit;
  t.n_plan = p->n_plan;
  t.bct = p->bct;
  t.bmask = p->bmask;
  t.items = fused ? p->fitems : p->items;
#ifdef WG_DEBUG_BOUNDS
  t.dbg_blocks = p->n_blocks;
  t.dbg_slots = fused ? p->n_fslots : p->n_slots;
#endif
  t.part = p->part;
  t.slots = p->slots;
  return t;
}

int launch_tiles_combine(const TilePlan* p, int64_t F, hipStream_t stream, bool fused = false) {
  const int32_t nm = fused ? p->n_fmulti : p->n_multi;
  const int4* multi = fused ? p->fmulti : p->multi;
  if (nm <= 0) return WG_OK;
  const dim3 grid((unsigned)ceil_div(p->rows * F, 256), nm), block(256);
  const int TR = p->rows;
  switch (F / 16) {
    case 1: hipLaunchKernelGGL(tiles_combine_kernel<16>, grid, block, 0, stream, multi, p->slots, p->part, F, p->n_plan, TR); break;
    case 2: hipLaunchKernelGGL(tiles_combine_kernel<32>, grid, block, 0, stream, multi, p->slots, p->part, F, p->n_plan, TR); break;
    case 3: hipLaunchKernelGGL(tiles_combine_kernel<48>, grid, block, 0, stream, multi, p->slots, p->part, F, p->n_plan, TR); break;
    default: hipLaunchKernelGGL(tiles_combine_kernel<64>, grid, block, 0, stream, multi, p->slots, p->part, F, p->n_plan, TR); break;
  }
  WG_LAUNCH_CHECK();
  return WG_OK;
}
}  // namespace

int launch_hybrid_fused(wg_laplacian_s* L, TilePlan* p, int64_t F, const float* u, const TeamPlan& tp,
                        const StepArgs& a, hipStream_t stream) {
  // the default tile shape only: 128-row blocks, one 16-row group per wave, the 16x16x32 MFMA
  if (!hybrid_fused_shape(L, p, F) || F > p->width || (reinterpret_cast<uintptr_t>(u) & 15) || !a.tsum ||
      tp.n_waves < 0)
    return WG_ERR_UNSUPPORTED;
  const TileArgs tt = tile_args(p, F, u, true);
  TeamArgs ta{};
  ta.a = a;
  ta.a.sell = tp.sell;
  ta.wd = tp.wd;
  ta.n_waves = tp.n_waves;
  ta.wpart = tp.wpart;
  ta.warr = tp.warr;
  team_args_debug(ta, tp);
  const int32_t ni = p->n_fitems;
  const int64_t nb = (int64_t)ni + ceil_div((int64_t)tp.n_waves, 8);
  if (nb > 0) {
    const dim3 grid((unsigned)nb), block(512);
    switch (F / 16) {
      case 1: hipLaunchKernelGGL(hybrid_fused_kernel<1>, grid, block, 0, stream, tt, ta, ni); break;
      case 2: hipLaunchKernelGGL(hybrid_fused_kernel<2>, grid, block, 0, stream, tt, ta, ni); break;
      case 3: hipLaunchKernelGGL(hybrid_fused_kernel<3>, grid, block, 0, stream, tt, ta, ni); break;
      default: hipLaunchKernelGGL(hybrid_fused_kernel<4>, grid, block, 0, stream, tt, ta, ni); break;
    }
    WG_LAUNCH_CHECK();
  }
  return launch_tiles_combine(p, F, stream, true);
}

int launch_tiles(wg_laplacian_s* L, TilePlan* p, int64_t F, const float* u, hipStream_t stream) {
  if (F % 16 != 0 || F > 64 || F > p->width || (reinterpret_cast<uintptr_t>(u) & 15))
    return fail(WG_ERR_INVALID, "launch_tiles: width %lld (need a multiple of 16 <= %d, 16-B aligned u)", (long long)F,
                std::min(64, (int)p->width));
  const TileArgs t = tile_args(p, F, u);
  if (p->n_items > 0) {
    // 128-row blocks: 8 waves of 16 rows, or (tile_rg = 2) 4 waves of two 16-row groups sharing
    // each B fragment (half the LDS reads)
    const int rg = p->rows == 128 ? L->tune.tile_rg : 1;
    const dim3 grid(p->n_items), block(4 * p->rows / rg);
    // 32x32x16 at width 64 by default (Reddit-size F = 64: 845 vs 872 us per step; at width 48
    // the padded shape loses, 785 vs 723: profiles/r03/s36_s39_tiles32)
    const int shape = L->tune.tile_mfma > 0 ? L->tune.tile_mfma : (F == 64 ? 32 : 16);
    const bool m32 = shape == 32 && p->rows == 128 && (F == 48 || F == 64);
#define WG_TILES(NFB)                                                                                  \
  if (p->rows == 64) hipLaunchKernelGGL((cheb_tiles_kernel<NFB, 4, 1, false>), grid, block, 0, stream, t);             \
  else if (rg == 4) hipLaunchKernelGGL((cheb_tiles_kernel<NFB, 2 * NFB, 4, true>), dim3(p->n_items), dim3(128 * NFB), 0, \
                                       stream, t);                                                                  \
  else if (rg == 2) hipLaunchKernelGGL((cheb_tiles_kernel<NFB, 4, 2, false>), grid, block, 0, stream, t);             \
  else hipLaunchKernelGGL((cheb_tiles_kernel<NFB, 8, 1, false>), grid, block, 0, stream, t);
    if (m32 && F == 48) hipLaunchKernelGGL(cheb_tiles32_kernel<48>, grid, dim3(512), 0, stream, t);
    else if (m32) hipLaunchKernelGGL(cheb_tiles32_kernel<64>, grid, dim3(512), 0, stream, t);
    else switch (F / 16) {
      case 1: WG_TILES(1) break;
      case 2: WG_TILES(2) break;
      case 3: WG_TILES(3) break;
      default: WG_TILES(4) break;
    }
#undef WG_TILES
    WG_LAUNCH_CHECK();
  }
  return launch_tiles_combine(p, F, stream);
}

}  // namespace wg
