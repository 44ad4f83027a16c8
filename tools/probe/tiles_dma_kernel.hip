// tiles_dma_kernel.hip -- measured and removed (r03 s25-s26; not built): the hybrid step's tile
// kernel (efficient-gnn_amd/csrc/tiles.hip) with its u tiles brought in by inline-asm LDS-DMA into
// a 4/6/8-deep ring, per-wave row masks and the 18 transposed B reads of a tile batched.  On the
// 8-way Reddit-size F=48 shard (tools/shard_probe.py) the tile kernel took 61.3-62.0 us at every
// depth with the first form and 66.0-68.2 us with the batched form, against 61.9 us for the
// 3-deep register ring; the full Reddit-size F=41 step 740-808 vs 749 us; bitwise equal results
// (tests/test_tiles.py at the time).  Timing-only builds of the register-ring kernel on the same
// shard: without the transposed B reads 29.3 us, without the MFMAs 52.6, without the split-and-
// stage writes 53.5 (profiles/r03/s27): the kernel is bound by its LDS B-fragment reads, not by
// the latency of its tile loads.  Kept for the record; it needs tiles.hip's helpers to compile.
// ---------------------------------------------------------------------------------------------
// The same block sums with the tiles of u brought in by LDS-DMA (global_load_lds_dwordx4) into a
// D-deep ring: a workgroup keeps D - 1 tiles in flight without holding them in registers, so a
// short row block (a shard's, or an ogbn-arxiv-size graph's: one or two workgroups per CU, tens of
// tiles each) is not paced by one load latency per two tiles as with the 3-deep register ring.
//
// Wave w < NUW brings 1 KiB of each 32 x W tile (its own 64 float4, the float4 index it splits
// later: lane l of wave w owns float4 w*64 + l), and every wave its own 16 row masks (lanes 0-3,
// 16 B each).  A wave reads back only bytes its own DMA wrote, after its own counted vmcnt wait,
// so the masks of tile j + 1 are read (and turned into the A fragment) while tile j is multiplied,
// and the only barrier per tile orders the split images.  The DMAs are inline asm, so the compiler
// inserts no vmcnt(0) before the ring's LDS reads (it would for the builtin), and the loop has no
// other vector-memory loads: the item's column tiles are staged into LDS first.  Dummy DMAs past
// the item's last tile re-read its last tile (never split), so every wave's wait count is the same
// every iteration; the ring drains before the workgroup ends.  Per tile a wave issues its 6 NFB
// transposed B reads together, then the 3 NFB MFMAs (one LDS latency per tile, not one per MFMA).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_base) {  // 16 B per lane -> [base + 16 lane]
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_base))
               : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {  // LDS writes visible; vector-memory DMAs stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

constexpr int kTileItemMax = 256;  // dense blocks per work item of the DMA kernel (its LDS column-tile list)

// waves per SIMD the LDS allows (2 per resident 512-thread workgroup), at most 4: the batched B
// fragments need ~110 VGPRs at W = 48 (at 80 the loop spills, and a scratch reload's vmcnt(0)
// would drain the DMA ring)
constexpr int tiles_dma_minw(int nfb, int d) {
  const int lds = 4096 + d * (kTC * 16 * nfb / 4) * 16 + d * 512 + 12 * 2 * img_dwords(nfb) + 4 * kTileItemMax;
  const int wg = 163840 / lds;
  const int cap = nfb == 4 ? 2 : 4;  // W = 64: 132 VGPRs
  return wg * 2 < cap ? wg * 2 : cap;
}

template <int NFB, int D>
__global__ __launch_bounds__(512, tiles_dma_minw(NFB, D)) void cheb_tiles_dma_kernel(TileArgs t) {
  constexpr int TR = 128;
  constexpr int NT = 512;
  constexpr int W = 16 * NFB;
  constexpr int NV = kTC * W / 4;  // float4 per tile
  constexpr int NUW = NV / 64;     // waves that bring (and split) a tile's u: 2, 4, 6, 8
  static_assert(NV % 64 == 0 && D >= 3, "tile shape");
  __shared__ uint4 lut[256];
  __shared__ __attribute__((aligned(16))) float4 raw[D][NV];
  __shared__ __attribute__((aligned(16))) uint32_t mring[D][TR];
  __shared__ __attribute__((aligned(16))) uint16_t img[2][3][2 * img_dwords(NFB)];
  __shared__ int32_t sbct[kTileItemMax];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int4 it = t.items[blockIdx.x];
  const int64_t rb = it.x;
  const int32_t b0 = it.y, n = it.z - it.y;
  for (int e = tid; e < 256; e += NT) {
    uint32_t d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      d[q] = (((e >> (2 * q)) & 1) ? 0x3F80u : 0u) | (((e >> (2 * q + 1)) & 1) ? 0x3F800000u : 0u);
    lut[e] = make_uint4(d[0], d[1], d[2], d[3]);
  }
  for (int e = tid; e < n; e += NT) sbct[e] = t.bct[b0 + e];
  __syncthreads();
  if (n <= 0) return;

  const bool uw = wave < NUW;
  const int kk = tid / (W / 4), f4 = (tid % (W / 4)) * 4;  // this lane's float4 of a tile (uw)
  // tile j's DMAs into ring slot j % D (j >= n: the last tile again, never split)
  auto issue = [&](int32_t j) {
    const int32_t jj = j < n ? j : n - 1;
    const int slot = j % D;
    if (uw) {
      int64_t row = (int64_t)sbct[jj] * kTC + kk;
      if (row >= t.col_limit) row = t.col_limit - 1;  // its mask bits are 0: any finite row
      dma16(t.u + row * t.ld + f4, lds_addr(&raw[slot][wave * 64]));
    }
    if (lane < 4) dma16(t.bmask + (int64_t)(b0 + jj) * TR + 16 * wave + lane * 4, lds_addr(&mring[slot][16 * wave]));
  };
  // this wave's DMAs of the tile issued D - 2 issues ago have landed
  auto wait_tile = [&]() {
    if (uw) wait_vm<2 * (D - 2)>();
    else wait_vm<D - 2>();
  };
  auto split = [&](const float4& x, int32_t j) {  // this lane's float4 of tile j -> buffer j % 2's images
    const int buf = j & 1;
    uint32_t h[4], m[4], l[4];
    split3(x.x, h[0], m[0], l[0]);
    split3(x.y, h[1], m[1], l[1]);
    split3(x.z, h[2], m[2], l[2]);
    split3(x.w, h[3], m[3], l[3]);
    const int o = img_row<NFB>(kk) + f4;
    *reinterpret_cast<uint2*>(&img[buf][0][o]) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    *reinterpret_cast<uint2*>(&img[buf][1][o]) = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
    *reinterpret_cast<uint2*>(&img[buf][2][o]) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
  };

  double acc[NFB][4];
  f32x4 cacc[NFB];
#pragma unroll
  for (int fb = 0; fb < NFB; ++fb) {
    cacc[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[fb][i] = 0.0;
  }
  int nacc = 0;
  const int trow = 8 * (lane >> 4) + ((lane & 15) >> 2);
  const int tcolo = 4 * (lane & 3);
  const int tr_lo = img_row<NFB>(trow) + tcolo, tr_hi = img_row<NFB>(trow + 4) + tcolo;
  const int mrow = 16 * wave + (lane & 15);
  const int mshift = 8 * (lane >> 4);
  uint32_t mwd;  // this lane's row mask of the next tile to multiply, and its A fragment
  bf16x8 a;
  auto fetch_a = [&](int32_t j) {
    mwd = mring[j % D][mrow];
    a = __builtin_bit_cast(bf16x8, lut[(mwd >> mshift) & 0xFFu]);
  };

  for (int32_t q = 0; q + 1 < D; ++q) issue(q);
  wait_tile();
  if (uw) split(raw[0][tid], 0);
  fetch_a(0);
  for (int32_t j = 0; j < n; ++j) {
    lds_barrier();  // tile j's images complete; ring slot (j - 1) % D free
    issue(j + D - 1);
    const bool any = __any(mwd != 0u);  // some row of the wave has an entry in tile j (wave-uniform)
    const int buf = j & 1;
    s16x4 bl[NFB][3], bh[NFB][3];
    if (any) {
#pragma unroll
      for (int fb = 0; fb < NFB; ++fb)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          bl[fb][p] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&img[buf][p][tr_lo + 16 * fb]));
          bh[fb][p] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(&img[buf][p][tr_hi + 16 * fb]));
        }
    }
    wait_tile();  // tile j + 1 landed (this wave's DMAs)
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    const bool more = j + 1 < n;
    if (uw && more) x = raw[(j + 1) % D][tid];
    const bf16x8 aj = a;
    if (more) fetch_a(j + 1);
    if (any) {
#pragma unroll
      for (int fb = 0; fb < NFB; ++fb)
#pragma unroll
        for (int p = 2; p >= 0; --p) {  // lo, mid, hi
          const s16x8 bv = {bl[fb][p][0], bl[fb][p][1], bl[fb][p][2], bl[fb][p][3],
                            bh[fb][p][0], bh[fb][p][1], bh[fb][p][2], bh[fb][p][3]};
          cacc[fb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aj, __builtin_bit_cast(bf16x8, bv), cacc[fb], 0, 0, 0);
        }
      if (++nacc == WG_TILES_FLUSH) {
#pragma unroll
        for (int fb = 0; fb < NFB; ++fb) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[fb][i] += (double)cacc[fb][i];
          cacc[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        nacc = 0;
      }
    }
    if (uw && more) split(x, j + 1);
  }
  wait_vm<0>();  // the dummy DMAs: nothing may land in LDS after the workgroup ends
  if (nacc > 0) {
#pragma unroll
    for (int fb = 0; fb < NFB; ++fb)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[fb][i] += (double)cacc[fb][i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = 16 * wave + 4 * (lane >> 4) + i;
    const int64_t row = rb * TR + rl;
    if (it.w < 0 && row >= t.n_plan) continue;
    double* dst = it.w < 0 ? t.part + row * t.ld : t.slots + ((int64_t)it.w * TR + rl) * W;
#pragma unroll
    for (int fb = 0; fb < NFB; ++fb) dst[16 * fb + (lane & 15)] = acc[fb][i];
  }
}

