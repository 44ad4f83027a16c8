// chain.hip -- the whole Chebyshev chain of a small graph in ONE launch
// (reference calibration/WATS.py:29-37 recurrence, heat sum :65-68 by
// Clenshaw's recurrence, row-L1 normalisation :71-72), F == 1 on unweighted
// graphs: SURVEY.md 7.5's "persistent kernel with a grid barrier for small
// graphs" (VERDICT r2 item 7).
//
// Why.  A PubMed-size chain (9.1 k active rows, 88.6 k nonzeros, K = 16) moves
// 1.2 MB per step; as K + 3 launches it is bound by the launch boundaries
// (~5 us each eagerly; a hipGraph replay of the same launches measured slower
// on this stack, +2.7 us per node: profiles/r03/s3_graph_probe.log).  Here P
// workgroups (one per CU, 1024 threads) run every step:
//
//  * each worker owns a contiguous, cost-balanced range of internal rows; its
//    rows' 16-bit column ids, row pointers, X0, dinv (sign = isolated flag) and
//    previous u stay in LDS for the whole chain;
//  * the gathered vector u = b * dinv (the value-free Clenshaw form of
//    DESIGN.md 4.1) of ALL active rows is staged in LDS; each step sums
//    u[col] over a row with a team of TS lanes (TS ~ row length / 4), float64;
//  * a worker publishes its rows' new u as data-tagged 8-byte granules {u,
//    tag = launch epoch * 64 + phase}, each ONE write-through (sc1) store; the
//    next phase re-stages u by loading every granule (sc1) until its tag is the
//    phase's -- no separate flag, counter or drain (MI355X_MICROARCH.md,
//    handoff-1to1).  Two granule buffers alternate by phase: a worker can only
//    write phase j+2's granules after every worker published phase j+1, i.e.
//    finished staging phase j.  One worker (small graphs, ids and both u
//    buffers in LDS) exchanges nothing: u alternates between two LDS buffers.
//    A wait gives up after ~0.5 s and raises an error flag (never a hang).
//
// Numbers (Clenshaw, b_K = c_K X0 implicit, as dist.hip's phase loop):
//   phase j = 1..K computes b_k, k = K - j:
//     b_k = ck X0 + cacc (L_hat b_{k+1}) - [j >= 3] b_{k+2},
//     cacc = j == 1 ? (k == 0 ? c_K : 2 c_K) : (k == 0 ? 1 : 2),  ck = c_k - [j == 2] c_K,
//   L_hat b = -dinv_i sum_j u_j (- b_i on isolated rows); k = 0 gives S.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "internal.h"

namespace wg {
namespace {

constexpr int kChainThreads = 1024;
constexpr int kChainWaves = kChainThreads / 64;
constexpr int kChainLds = 160 * 1024 - 64;  // dynamic LDS per worker

struct ChainArgs {
  int32_t n_act;
  int32_t K;
  int32_t P;
  int32_t stride;             // workgroup b is worker b / stride when b % stride == 0 (XCD placement)
  int32_t ustride;            // floats per exchange buffer
  const uint16_t* ids;        // [nnz_act] column ids (row order): the worker's local column ids (P > 1)
  const uint16_t* wcols;      // P > 1: each worker's gathered columns (ascending), concatenated
  const int32_t* wcol_off;    // [P + 1] their offsets
  const uint16_t* gids;       // [nnz_act] global column ids (direct mode)
  const uint16_t* bcols;      // direct mode: each worker's back-edge columns (build_chain_plan), concatenated
  const int32_t* bcol_off;    // [P + 1]
  int32_t direct;             // tuning key "chain_direct": gathers read the granules (no LDS staging)
  const int4* wdesc;          // [P] {row0, row1, e0, e1}
  const int32_t* wpass;       // [P][kChainWaves + 1] pass offsets of each worker's waves (into passes)
  const int2* passes;         // one wave pass: {first row, rows | log2 team size << 8}
  const int32_t* rowptr;      // internal row pointers
  const double* dinv;
  const uint8_t* iso;
  const int32_t* perm;
  const float* X0;            // the caller's signal: internal X0 = X0[perm[row]], u_0 = X0 * dinv on the fly
  int64_t n;                  // rows; [n_act, n) are the closed-form rows (S = coef * X0)
  double coef;
  uint64_t* gbuf;             // [2][ustride] tagged granules {float bits, tag << 32}
  int32_t* bar;               // [1] workers finished, [2] epoch + 1 of the last timed-out launch, [3] launch epoch
                              // (bumped by the launch's last worker to finish: every worker read it first)
  int32_t* host_flag;         // host-mapped: epoch + 1 of the last timed-out launch (read by the next API call)
  int64_t wait_ticks;         // a granule wait gives up after this many wall-clock ticks (~0.5 s)
  int32_t fault_phase;        // fault injection (tuning key "chain_fault", tests): worker 0 skips this phase's publish
  float* S;                   // caller order
  float* H;
#ifdef WG_DEBUG_BOUNDS
  int32_t dbg_lds;            // the launch's dynamic LDS bytes
#endif
  double c[kChainMaxK + 1];   // heat coefficients exp(-s k)
};

// LDS layout of one worker (byte offsets, 16-B aligned sections): u [, u2] (one worker: every
// active row, twice; else the nu columns the worker gathers), dinv (double) and its reciprocal, X0,
// previous u, current u of the own rows, row pointers, 16-bit ids, wave passes, the gathered
// columns' global ids
struct ChainLayout {
  int64_t u2, dv, x0o, pu, cu, lrp, id, pas, wc, bytes;
  __host__ __device__ ChainLayout(int64_t nu, int64_t nr, int64_t ne, int64_t npass, bool single) {
    auto al = [](int64_t x) { return (x + 15) & ~(int64_t)15; };
    const int64_t ub = al(4 * nu);
    u2 = ub;
    dv = single ? 2 * ub : ub;
    x0o = al(dv + 16 * nr);  // dinv and its reciprocal
    pu = al(x0o + 4 * nr);
    cu = al(pu + 4 * nr);
    lrp = al(cu + 4 * nr);
    id = al(lrp + 4 * (nr + 1));
    pas = al(id + 2 * ne);
    wc = al(pas + 8 * npass);
    bytes = al(wc + (single ? 0 : 2 * nu));
  }
};

__device__ __forceinline__ uint64_t ld_sc1_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// u[0, n) <- the granules of one phase (n <= kChainThreads * kStageMax): every element of the
// thread in flight at once (one memory round trip when the producers are done), re-polled with
// a short sleep until every tag is the phase's; false after wait_ticks of the constant-rate
// wall clock (a worker never published)
constexpr int kStageMax = 24;
#ifndef WG_CHAIN_SLEEP  // s_sleep units (64 cycles) between polls of granules not yet published
#define WG_CHAIN_SLEEP 1
#endif
__device__ __forceinline__ bool stage_tagged(float* u, const uint64_t* g, const uint16_t* cols, int n, uint32_t tag,
                                             int tid, int64_t wait_ticks) {
  uint32_t pending = 0;
  int src[kStageMax];  // the granule of local column tid + q * threads
#pragma unroll
  for (int q = 0; q < kStageMax; ++q) {
    const int i = tid + q * kChainThreads;
    src[q] = i < n ? (int)cols[i] : 0;
    if (i < n) pending |= 1u << q;
  }
  const uint64_t t0 = wall_clock64();
  while (pending) {
    uint64_t v[kStageMax];
#pragma unroll
    for (int q = 0; q < kStageMax; ++q) v[q] = (pending >> q) & 1 ? ld_sc1_u64(g + src[q]) : 0ull;
#pragma unroll
    for (int q = 0; q < kStageMax; ++q) {
      if (((pending >> q) & 1) && (uint32_t)(v[q] >> 32) == tag) {
        u[tid + q * kChainThreads] = __uint_as_float((uint32_t)v[q]);
        pending &= ~(1u << q);
      }
    }
    if (pending) {
      __builtin_amdgcn_s_sleep(WG_CHAIN_SLEEP);
      if ((int64_t)(wall_clock64() - t0) > wait_ticks) return false;
    }
  }
  return true;
}

// a granule wait that gave up: the launch's epoch recorded (once per worker) for the next API call
__device__ __forceinline__ void chain_fail(const ChainArgs& a, int* s_bad, uint32_t ep) {
  if (atomicExch(s_bad, 1) == 0) {
    // epoch + 1: a fresh plan's flag starts at 0 (nothing reported), so its first launch (epoch 0) counts too
    __hip_atomic_store(a.bar + 2, (int32_t)(ep + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.host_flag) __hip_atomic_store(a.host_flag, (int32_t)(ep + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// u_0 of internal row c: the caller's X0 row perm[c] times dinv (what the permute-in pass wrote)
__device__ __forceinline__ float chain_u0(const ChainArgs& a, int c) {
  return (float)((double)a.X0[a.perm[c]] * a.dinv[c]);
}

// direct mode: u of columns c[0 .. n) for phase j -- u_0 (from the caller's X0) in phase 1,
// else the previous phase's granules, all loads in flight at once, re-polled until every tag is
// `want`; false past the deadline (the values are then NaN)
__device__ __forceinline__ bool fetch_u(const ChainArgs& a, const uint64_t* gprev, int j, uint32_t want,
                                        const int (&c)[4], int n, float (&x)[4], uint64_t deadline) {
  if (j == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < n) x[i] = chain_u0(a, c[i]);
    return true;
  }
  uint64_t v[4];
  uint32_t pending = (1u << n) - 1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (i < n) v[i] = ld_sc1_u64(gprev + c[i]);
  for (;;) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (((pending >> i) & 1) && (uint32_t)(v[i] >> 32) == want) {
        x[i] = __uint_as_float((uint32_t)v[i]);
        pending &= ~(1u << i);
      }
    if (!pending) return true;
    if (wall_clock64() > deadline) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((pending >> i) & 1) x[i] = __int_as_float(0x7fc00000);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((pending >> i) & 1) v[i] = ld_sc1_u64(gprev + c[i]);
  }
}

__global__ __launch_bounds__(kChainThreads) void cheb_chain1_kernel(ChainArgs a) {
  if (blockIdx.x % a.stride) return;  // placement filler
  const int w = blockIdx.x / a.stride;
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x;
  const int4 d = a.wdesc[w];
  const int row0 = d.x, nr = d.y - d.x, e0 = d.z, ne = d.w - d.z;
  const int32_t* wp = a.wpass + w * (kChainWaves + 1);
  const int pass0 = wp[0], npass = wp[kChainWaves] - pass0;
  const int wc0 = a.P == 1 ? 0 : a.wcol_off[w];
  const int nu = a.P == 1 ? a.n_act : a.wcol_off[w + 1] - wc0;       // columns this worker gathers
  const ChainLayout lay(nu, nr, ne, npass, a.P == 1);
  WG_DCHECK(lay.bytes <= a.dbg_lds && row0 >= 0 && nr >= 0 && row0 + nr <= a.n_act && e0 >= 0 && ne >= 0 && nu >= 0 &&
                nu <= a.n_act,
            "worker %d: rows [%d, %d) entries %d+%d columns %d need %lld LDS bytes of %d", w, row0, row0 + nr, e0, ne, nu,
            (long long)lay.bytes, a.dbg_lds);
  float* u = reinterpret_cast<float*>(smem);                         // [nu] the gathered u (local ids)
  float* u2 = reinterpret_cast<float*>(smem + lay.u2);               // [n_act] one worker: the next u
  double* dv = reinterpret_cast<double*>(smem + lay.dv);             // [nr] dinv, negative = isolated row
  double* rdv = dv + nr;                                             // [nr] 1 / dinv
  float* x0o = reinterpret_cast<float*>(smem + lay.x0o);             // [nr]
  float* pu = reinterpret_cast<float*>(smem + lay.pu);               // [nr] previous u of own rows
  float* cu = reinterpret_cast<float*>(smem + lay.cu);               // [nr] current u of own rows
  int32_t* lrp = reinterpret_cast<int32_t*>(smem + lay.lrp);         // [nr + 1]
  uint16_t* id = reinterpret_cast<uint16_t*>(smem + lay.id);         // [ne]
  int2* pas = reinterpret_cast<int2*>(smem + lay.pas);               // [npass] the worker's wave passes
  uint16_t* wc = reinterpret_cast<uint16_t*>(smem + lay.wc);         // [nu] P > 1: global id of local column
  const uint32_t ep = (uint32_t)a.bar[3] & 0x3ffffffu;             // this launch's epoch (tags ep * 64 + j)
  // A granule wait that gave up leaves stale u in this worker's LDS: from then on the worker
  // publishes NaN for its rows and writes NaN S / H, so every result that depends on the
  // missing data is NaN (never silently wrong), and the launch's epoch is recorded in bar[2]
  // and in the host-mapped flag (wg_wavelet_features / wg_chain_status report it).
  __shared__ int s_bad;
  if (tid == 0) s_bad = 0;
  // ---- stage the worker's rows, its pass table and u_0
  for (int i = tid; i < nr; i += kChainThreads) {
    const double di = a.dinv[row0 + i];
    dv[i] = a.iso[row0 + i] ? -di : di;
    rdv[i] = 1.0 / di;
    const float x = a.X0[a.perm[row0 + i]];
    x0o[i] = x;
    cu[i] = (float)((double)x * di);
    lrp[i] = a.rowptr[row0 + i] - e0;
  }
  if (tid == 0) lrp[nr] = ne;
  for (int64_t i = (int64_t)a.n_act + (int64_t)w * kChainThreads + tid; i < a.n; i += (int64_t)a.P * kChainThreads) {
    const int32_t r = a.perm[i];  // the closed-form rows, dealt over the workers
    const double sv = a.coef * (double)a.X0[r];
    a.S[r] = (float)sv;
    a.H[r] = (float)(sv / (fabs(sv) + 1e-8));
  }
  const uint16_t* idsrc = a.direct ? a.gids : a.ids;
  for (int i = tid; i < ne; i += kChainThreads) {
    id[i] = idsrc[e0 + i];
    WG_DCHECK(id[i] < (a.direct ? a.n_act : nu), "worker %d entry %d: column id %d past %d", w, e0 + i, (int)id[i],
              a.direct ? a.n_act : nu);
  }
  for (int i = tid; i < npass; i += kChainThreads) pas[i] = a.passes[pass0 + i];
  if (a.direct) {
    // no LDS copy of u: the gathers read u_0 and then the granules themselves
  } else if (a.P == 1) {
    for (int i = tid; i < a.n_act; i += kChainThreads) u[i] = chain_u0(a, i);
  } else {
    for (int i = tid; i < nu; i += kChainThreads) {
      const int c = a.wcols[wc0 + i];
      WG_DCHECK(c < a.n_act, "worker %d: gathered column %d past %d active rows", w, c, a.n_act);
      wc[i] = (uint16_t)c;
      u[i] = chain_u0(a, c);
    }
  }
  __syncthreads();
#ifdef WG_CHAIN_TRACE  // timing build: worker 0 prints its phase timeline (s_memtime cycles)
  long long tr[2 * kChainMaxK + 4];
  int ntr = 0;
  tr[ntr++] = clock64();
#endif
  const int wave = tid >> 6, lane = tid & 63;
  const int pb = wp[wave] - pass0, pe = wp[wave + 1] - pass0;  // this wave's passes (no workgroup sync inside a phase)
  const int K = a.K;
  bool bad = false;  // uniform over the workgroup (read after a barrier)
  for (int j = 1; j <= K; ++j) {
    const int k = K - j;
    const double cacc = (j == 1) ? (k == 0 ? a.c[K] : 2.0 * a.c[K]) : (k == 0 ? 1.0 : 2.0);
    const double ck = a.c[k] - (j == 2 ? a.c[K] : 0.0);
    const bool prevs = j >= 3;
    const uint64_t tag = (uint64_t)((ep << 6) | (uint32_t)j) << 32;
    // staging: two granule buffers by phase; direct: four (a worker publishing phase j overwrites
    // phase j - 4, read by its readers in phase j - 3: every reader is also a producer of this
    // worker (symmetric graphs) or a back edge it polls, and its phase j - 2 granules, seen before
    // this worker's barrier of phase j - 1, prove it passed its own barrier after phase j - 3)
    uint64_t* gnext = a.gbuf + (size_t)(j & (a.direct ? 3 : 1)) * a.ustride;
    const uint64_t* gprev = a.gbuf + (size_t)((j - 1) & 3) * a.ustride;
    const uint32_t want = (ep << 6) | (uint32_t)(j - 1);
    const uint64_t deadline = wall_clock64() + (uint64_t)a.wait_ticks;
    if (a.direct && j >= 2) {  // back edges: one granule of every worker that reads this one's rows
      const int b0 = a.bcol_off[w], b1 = a.bcol_off[w + 1];
      for (int i = b0 + tid; i < b1; i += kChainThreads)
        while ((uint32_t)(ld_sc1_u64(gprev + a.bcols[i]) >> 32) != want) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() > deadline) {
            chain_fail(a, &s_bad, ep);
            break;
          }
        }
    }
    for (int pi = pb; pi < pe; ++pi) {
      const int2 P = pas[pi];
      const int lts = P.y >> 8;
      const int TS = 1 << lts;
      const int team = lane >> lts;
      const int tl = lane & (TS - 1);
      {
        const int row = P.x + team;
        const bool act = team < (P.y & 0xff);
        const int li = row - row0;
        double s = 0.0;
        if (act && a.direct) {  // the same four chains, each term a granule (or u_0) from memory
          const int b = lrp[li], e = lrp[li + 1];
          double s1 = 0.0, s2 = 0.0, s3 = 0.0;
          int q = b + tl;
          float x[4];
          for (; q + 3 * TS < e; q += 4 * TS) {
            const int c4[4] = {id[q], id[q + TS], id[q + 2 * TS], id[q + 3 * TS]};
            if (!fetch_u(a, gprev, j, want, c4, 4, x, deadline)) chain_fail(a, &s_bad, ep);
            s += (double)x[0];
            s1 += (double)x[1];
            s2 += (double)x[2];
            s3 += (double)x[3];
          }
          for (; q < e; q += TS) {
            const int c1[4] = {id[q], 0, 0, 0};
            if (!fetch_u(a, gprev, j, want, c1, 1, x, deadline)) chain_fail(a, &s_bad, ep);
            s += (double)x[0];
          }
          s = (s + s1) + (s2 + s3);
        } else if (act) {  // four independent LDS chains per lane (the phase is latency-bound)
          const int b = lrp[li], e = lrp[li + 1];
          double s1 = 0.0, s2 = 0.0, s3 = 0.0;
          int q = b + tl;
          for (; q + 3 * TS < e; q += 4 * TS) {
            const int i0 = id[q], i1 = id[q + TS], i2 = id[q + 2 * TS], i3 = id[q + 3 * TS];
            s += (double)u[i0];
            s1 += (double)u[i1];
            s2 += (double)u[i2];
            s3 += (double)u[i3];
          }
          for (; q < e; q += TS) s += (double)u[id[q]];
          s = (s + s1) + (s2 + s3);
        }
        for (int off = TS >> 1; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        if (act && tl == 0) {
          const double dsi = dv[li];
          const double di = fabs(dsi);
          const double rdi = rdv[li];  // 1 / dinv
          const float ui = cu[li];     // this row's u of the previous phase (b_{k+1} * dinv)
          double lb = -di * s;
          if (dsi < 0.0) lb -= (double)ui * rdi;  // isolated row: L_hat_ii = -1 (ui / di = b_i)
          const double t = ck * (double)x0o[li] + cacc * lb - (prevs ? (double)pu[li] * rdi : 0.0);
          if (k > 0) {
            pu[li] = ui;  // b_{k+1} (as u): the next phase's b_{k+2}
            const float un = bad ? __int_as_float(0x7fc00000) : (float)(t * di);
            cu[li] = un;
            if (a.P == 1) u2[row] = un;
            else if (!(j == a.fault_phase && w == 0))
              __hip_atomic_store(gnext + row, tag | __float_as_uint(un), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            const int32_t r = a.perm[row];
            const float nan = __int_as_float(0x7fc00000);
            a.S[r] = bad ? nan : (float)t;
            a.H[r] = bad ? nan : (float)(t / (fabs(t) + 1e-8));
          }
        }
      }
    }
#ifdef WG_CHAIN_TRACE
    __syncthreads();
    tr[ntr++] = clock64();
#endif
    if (k == 0) break;
    __syncthreads();  // every gather of this phase is done with u
    if (a.direct) {  // nothing to stage: the next phase's gathers read this phase's granules
      bad = s_bad != 0;
      continue;
    }
    if (a.P == 1) {
      float* t = u;
      u = u2;
      u2 = t;
    } else if (!stage_tagged(u, gnext, wc, nu, (uint32_t)(tag >> 32), tid, a.wait_ticks)) {
      if (atomicExch(&s_bad, 1) == 0) {  // one lane per worker records the failed launch
        __hip_atomic_store(a.bar + 2, (int32_t)(ep + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.host_flag) __hip_atomic_store(a.host_flag, (int32_t)(ep + 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
    bad = s_bad != 0;
#ifdef WG_CHAIN_TRACE
    tr[ntr++] = clock64();
#endif
  }
  if (tid == 0) {  // the last worker to finish moves the epoch on for the next launch
    const int32_t done = __hip_atomic_fetch_add(a.bar + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == a.P - 1) {
      __hip_atomic_store(a.bar + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.bar + 3, (int32_t)((ep + 1) & 0x3ffffffu), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#ifdef WG_CHAIN_TRACE
  if (w == 0 && tid == 0) {
    printf("chain1 trace P=%d n_act=%d rows=%d entries=%d passes(wave0)=%d: staged at %lld\n", a.P, a.n_act, nr, ne,
           pe - pb, tr[0]);
    for (int i = 1; i < ntr; ++i) printf("  +%lld", tr[i] - tr[i - 1]);
    printf("\n");
  }
#endif
}


// ---- solo: the whole chain in ONE workgroup, no exchange at all.  PubMed-size
// graphs do not fit one workgroup's LDS with their 16-bit ids (177 KB for 88.6 k entries), so the
// chain above runs 128 workers and pays two Infinity-Cache trips per phase.  Here the ids live in
// the 1024 threads' REGISTERS (E slots per lane, two 16-bit LDS byte offsets per VGPR) and LDS holds
// u twice (the gathered u_{k+1} and, in place, u_{k+2} -> u_k), X0 and dinv: 16 B per active row.
// Each wave runs a static list of passes (the plan): a pass gives 64 / TS rows of similar length a
// team of TS lanes each and lasts L slots (ceil(length / TS), the pass's longest row); a lane sums
// its slots' u in float32, flushed to float64 every 8 slots; at the pass's last slot (uniform: a
// scalar compare) the team's sums meet by shuffles and the row's epilogue writes u_k over u_{k+2}:
//   u_k = dinv (ck X0 - cacc dinv s) - u_{k+2} [- cacc u_{k+1} on isolated rows]
// (cheb_chain1_kernel's b_k = ck X0 + cacc L_hat b_{k+1} - b_{k+2} times dinv, no division; the
// last phase's u_0 = S dinv is divided out at the end).  One workgroup barrier per phase.  The kernel
// does its own prologue (internal X0, u_0, the closed-form rows).  The plan orders each team's entries slot by slot so that a read
// group's 32 lanes hit distinct LDS banks where they can.  No co-residency, no wait, no timeout.
constexpr int kSoloBlock = 16;  // loads issued per block before their sums
constexpr int64_t kSoloMaxNnz = 1 << 15;  // the auto plan's limit (build_chain_plan)
constexpr int kSoloSlots = 8;   // a pass's team size keeps ceil(length / TS) within this many slots

struct SoloArgs {
  int32_t n_act;
  int32_t K;
  int32_t off_ub, off_x0, off_dv, off_pt;  // LDS byte offsets (u buffer A at 0; off_pt: the pass table)
  int32_t n_pass;
  const uint32_t* ids;             // [E / 2][threads]: two 16-bit LDS byte offsets (column * 4) per word
  const int4* passes;              // {first row, rows | log2 TS << 8, L, 0}
  const int32_t* wpass;            // [waves + 1]: each wave's passes
  const int32_t* wslots;           // [waves]: slots each wave uses
  const double* dinv;
  const uint8_t* iso;
  const int32_t* perm;
  const float* X0;  // the caller's signal (the permute-in is done here)
  int64_t n;        // rows; [n_act, n) are the closed-form rows
  double coef;      // their S = coef * X0
  float* S;
  float* H;
  double c[kChainMaxK + 1];
};

template <int E>
__device__ __forceinline__ uint32_t solo_entry(const uint32_t (&w)[E / 2], int q) {
  return (q & 1) ? (w[q >> 1] >> 16) : (w[q >> 1] & 0xffffu);
}

template <int E>
__global__ __launch_bounds__(kChainThreads) void cheb_chain_solo_kernel(SoloArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int na = a.n_act;
  float* x0 = reinterpret_cast<float*>(smem + a.off_x0);  // [na]
  float* dv = reinterpret_cast<float*>(smem + a.off_dv);  // [na] dinv, negative: isolated row
  int4* pt = reinterpret_cast<int4*>(smem + a.off_pt);     // [n_pass] every wave's passes
  uint32_t idw[E / 2];
#pragma unroll
  for (int q = 0; q < E / 2; ++q) idw[q] = a.ids[q * kChainThreads + tid];
  {
    float* ua = reinterpret_cast<float*>(smem);
    float* ub = reinterpret_cast<float*>(smem + a.off_ub);
    for (int i = tid; i < na; i += kChainThreads) {  // the internal X0 and u_0
      const float x = a.X0[a.perm[i]];
      const double di = a.dinv[i];
      ua[i] = (float)((double)x * di);
      ub[i] = 0.0f;
      x0[i] = x;
      dv[i] = a.iso[i] ? -(float)di : (float)di;
    }
    for (int64_t i = na + tid; i < a.n; i += kChainThreads) {  // closed-form rows
      const int32_t r = a.perm[i];
      const double sv = a.coef * (double)a.X0[r];
      a.S[r] = (float)sv;
      a.H[r] = (float)(sv / (fabs(sv) + 1e-8));
    }
    if (tid == 0) ua[na] = ub[na] = 0.0f;  // the pad column
    for (int i = tid; i < a.n_pass; i += kChainThreads) pt[i] = a.passes[i];
  }
  // a pass descriptor as scalars (uniform over the wave)
  auto pass_at = [&](int i) -> int4 {
    const int4 v = pt[i];
    return int4{__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                __builtin_amdgcn_readfirstlane(v.z), 0};
  };
  const int p0 = a.wpass[wave], p1 = a.wpass[wave + 1];
  const int nslots = a.wslots[wave];
  __syncthreads();
  const int K = a.K;
  int cur = 0;  // the buffer of u_{k+1} (gathered); the other holds u_{k+2} and receives u_k
  for (int j = 1; j <= K; ++j) {
    const int k = K - j;  // cheb_chain1_kernel's phase coefficients
    const double cacc = (j == 1) ? (k == 0 ? a.c[K] : 2.0 * a.c[K]) : (k == 0 ? 1.0 : 2.0);
    const double ck = a.c[k] - (j == 2 ? a.c[K] : 0.0);
    const bool prevs = j >= 3;
    const unsigned char* ug = smem + (cur ? a.off_ub : 0);
    float* uo = reinterpret_cast<float*>(smem + (cur ? 0 : a.off_ub));
    const float* ugf = reinterpret_cast<const float*>(ug);
    // the decoded offsets must not be hoisted out of the phase loop (E more live registers)
#pragma unroll
    for (int q = 0; q < E / 2; ++q) asm volatile("" : "+v"(idw[q]));
    int pi = p0;
    int4 pd = pi < p1 ? pass_at(pi) : int4{0, 0, 0, 0};
    int4 pn = pi + 1 < p1 ? pass_at(pi + 1) : int4{0, 0, 0, 0};  // the next pass, read ahead
    int pend = pi < p1 ? pd.z - 1 : -1;  // the slot that ends the current pass
    float accf = 0.0f;
    double accd = 0.0;
    auto finish = [&]() {
      const int lts = pd.y >> 8;
      const int TS = 1 << lts;
      const int team = lane >> lts;
      double sum = accd + (double)accf;
      for (int off = TS >> 1; off >= 1; off >>= 1) sum += __shfl_xor(sum, off, 64);
      if ((lane & (TS - 1)) == 0 && team < (pd.y & 0xff)) {
        const int row = pd.x + team;
        const float dr = dv[row];
        const double di = fabs((double)dr);
        const double xr = (double)x0[row];
        const double u2 = prevs ? (double)uo[row] : 0.0;  // u_{k+2} (own row)
        const double u1 = dr < 0.0f ? (double)ugf[row] : 0.0;  // isolated row: L_hat_ii = -1
        // b_k * dinv; the last phase's (S * dinv) is divided out after the loop
        uo[row] = (float)(di * (ck * xr - cacc * di * sum) - u2 - cacc * u1);
      }
      accf = 0.0f;
      accd = 0.0;
      ++pi;
      if (pi < p1) {
        pd = pn;
        pend += pd.z;
        if (pi + 1 < p1) pn = pass_at(pi + 1);
      } else {
        pend = -1;
      }
    };
#pragma unroll
    for (int b = 0; b < E; b += kSoloBlock) {
      if (b >= nslots) break;  // uniform
      float x[kSoloBlock];
#pragma unroll
      for (int q = 0; q < kSoloBlock; ++q) x[q] = *reinterpret_cast<const float*>(ug + solo_entry<E>(idw, b + q));
#pragma unroll
      for (int q = 0; q < kSoloBlock; ++q) {
        accf += x[q];
        if ((q & 7) == 7) {
          accd += (double)accf;
          accf = 0.0f;
        }
        if (b + q == pend) finish();
      }
    }
    __syncthreads();  // u_k complete before the next phase gathers it
    cur ^= 1;
  }
  // S = (S * dinv) / dinv and H = S / (|S|_1 + 1e-8), to the caller's rows
  const float* us = reinterpret_cast<const float*>(smem + (cur ? a.off_ub : 0));
  for (int i = tid; i < na; i += kChainThreads) {
    const double t = (double)us[i] / fabs((double)dv[i]);
    const int32_t r = a.perm[i];
    a.S[r] = (float)t;
    a.H[r] = (float)(t / (fabs(t) + 1e-8));
  }
}

const void* solo_kernel(int E) {
  switch (E) {
    case 32: return (const void*)cheb_chain_solo_kernel<32>;
    case 64: return (const void*)cheb_chain_solo_kernel<64>;
    case 96: return (const void*)cheb_chain_solo_kernel<96>;
    case 128: return (const void*)cheb_chain_solo_kernel<128>;
    default: return nullptr;
  }
}

template <typename T>
int upload(T** d, const std::vector<T>& h) {
  if (int rc = dmalloc(d, h.size())) return rc;
  if (!h.empty()) WG_HIP_TRY(hipMemcpy(*d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return WG_OK;
}

// rows r0..r1 (descending length) as wave passes: runs of rows sharing a team size TS (~4
// entries per lane, at most 64 lanes), 64 / TS rows per pass
void make_passes(const std::vector<int32_t>& rp, int64_t r0, int64_t r1, std::vector<int2>& out,
                 std::vector<int64_t>& cost) {
  int64_t r = r0;
  while (r < r1) {
    const int64_t len = rp[r + 1] - rp[r];
    int lts = 0;
    while (lts < 6 && ((int64_t)4 << lts) < len) ++lts;
    const int64_t rows = std::min<int64_t>(64 >> lts, r1 - r);
    int64_t n = 0;
    while (n < rows) {  // the same team size for every row of the pass (lengths only decrease)
      const int64_t l = rp[r + n + 1] - rp[r + n];
      int t = 0;
      while (t < 6 && ((int64_t)4 << t) < l) ++t;
      if (t != lts) break;
      ++n;
    }
    out.push_back(int2{(int)r, (int)n | (lts << 8)});
    cost.push_back((len + (1 << lts) - 1) / (1 << lts) + 8);  // the longest lane's entries + an epilogue
    r += n;
  }
}


// The solo plan (cheb_chain_solo_kernel), or WG_ERR_UNSUPPORTED when the graph does not fit one
// workgroup (16 B of LDS per active row, <= 128 slots per lane).
// Passes: consecutive rows (descending length) sharing a team size TS, the smallest power of two
// with ceil(length / TS) <= kSoloSlots; 64 / TS rows per pass, L = the longest row's ceil(length /
// TS) slots.  Passes go to the 16 waves longest first onto the least loaded wave (L + an epilogue's
// worth of slots).  Slot by slot, each read group's 32 lanes take, fewest choices first, an entry of
// their row (a team's lanes share its row's entries) whose LDS bank (column mod 32) has the fewest
// distinct columns so far -- the same column is a broadcast, free (MI355X_MICROARCH.md, LDS:
// ds_read_b32 serves two groups of 32 lanes, one cycle per extra distinct address on a bank).
int build_solo_plan(wg_laplacian_s* L, ChainPlan* p, const std::vector<int32_t>& rp, const std::vector<uint16_t>& ids) {
  const int64_t na = L->n_active;
  const int T = kChainThreads;
  if (na < 1 || 4 * (na + 1) > 0xffff) return WG_ERR_UNSUPPORTED;  // 16-bit LDS byte offsets
  auto al = [](int64_t x) { return (x + 15) & ~(int64_t)15; };
  const int64_t off_ub = al(4 * (na + 1)), off_x0 = al(off_ub + 4 * (na + 1)), off_dv = al(off_x0 + 4 * na);
  if (al(off_dv + 4 * na) > kChainLds) return WG_ERR_UNSUPPORTED;
  struct Pass {
    int32_t row0, n, lts, L;
  };
  std::vector<Pass> passes;
  for (int64_t r = 0; r < na;) {
    auto ts_of = [&](int64_t len) {
      int l = 0;
      while (l < 6 && (len + (1 << l) - 1) / (1 << l) > kSoloSlots) ++l;
      return l;
    };
    const int64_t len0 = rp[r + 1] - rp[r];
    const int lts = ts_of(len0);
    int n = 0;
    int64_t L = 1;
    while (n < (64 >> lts) && r + n < na && ts_of(rp[r + n + 1] - rp[r + n]) == lts) {
      L = std::max<int64_t>(L, (rp[r + n + 1] - rp[r + n] + (1 << lts) - 1) >> lts);
      ++n;
    }
    passes.push_back(Pass{(int32_t)r, n, lts, (int32_t)L});
    r += n;
  }
  // passes onto waves: longest first onto the least loaded (slots + an epilogue's worth)
  constexpr int kEpiSlots = 6;
  std::vector<int> order(passes.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return passes[x].L > passes[y].L; });
  std::vector<int64_t> load(kChainWaves, 0), slots_w(kChainWaves, 0);
  std::vector<std::vector<int>> per(kChainWaves);
  for (int i : order) {
    const int v = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    load[v] += passes[i].L + kEpiSlots;
    slots_w[v] += passes[i].L;
    per[v].push_back(i);
  }
  const int64_t need = *std::max_element(slots_w.begin(), slots_w.end());
  int E = 0;
  for (int e : {32, 64, 96, 128})
    if (need <= e) {
      E = e;
      break;
    }
  if (!E) return WG_ERR_UNSUPPORTED;
  // slots: per lane, the byte offset (column * 4) of each slot's entry; pads read the zero column na
  const uint16_t pad = (uint16_t)(4 * na);
  std::vector<uint16_t> slot((size_t)T * E, pad);
  std::vector<int4> ptab;
  std::vector<int32_t> wpass(kChainWaves + 1, 0), wslots(kChainWaves, 0);
  int64_t cyc_plain = 0, cyc_sched = 0;  // pass-1 LDS cycles (sum over slots and read groups of the worst bank)
  for (int v = 0; v < kChainWaves; ++v) {
    wpass[v] = (int32_t)ptab.size();
    int q0 = 0;
    for (int i : per[v]) {
      const Pass& ps = passes[i];
      ptab.push_back(int4{ps.row0, ps.n | (ps.lts << 8), ps.L, 0});
      const int TS = 1 << ps.lts;
      std::vector<std::vector<uint16_t>> pool(64 >> ps.lts);  // each team's remaining columns
      for (int t = 0; t < ps.n; ++t)
        for (int32_t e = rp[ps.row0 + t]; e < rp[ps.row0 + t + 1]; ++e) pool[t].push_back(ids[e]);
      std::vector<std::vector<uint16_t>> plain(pool);  // the natural order, for the cycle count
      for (int q = 0; q < ps.L; ++q) {
        for (int g = 0; g < 2; ++g) {
          int load_s[32] = {0}, load_p[32] = {0};
          std::vector<uint16_t> seen_s, seen_p;
          std::vector<int> lanes;
          for (int l = 32 * g; l < 32 * g + 32; ++l) lanes.push_back(l);
          std::stable_sort(lanes.begin(), lanes.end(),
                           [&](int x, int y) { return pool[x >> ps.lts].size() < pool[y >> ps.lts].size(); });
          for (int l : lanes) {
            std::vector<uint16_t>& pl = pool[l >> ps.lts];
            uint16_t c = (uint16_t)na;
            if (!pl.empty()) {
              size_t best = 0;
              int bc = 1 << 30;
              for (size_t x = 0; x < pl.size(); ++x) {
                const int cost = std::find(seen_s.begin(), seen_s.end(), pl[x]) != seen_s.end() ? -1 : load_s[pl[x] & 31];
                if (cost < bc) {
                  bc = cost;
                  best = x;
                }
              }
              c = pl[best];
              pl[best] = pl.back();
              pl.pop_back();
            }
            slot[(size_t)(64 * v + l) * E + q0 + q] = (uint16_t)(4 * c);
            if (std::find(seen_s.begin(), seen_s.end(), c) == seen_s.end()) {
              seen_s.push_back(c);
              ++load_s[c & 31];
            }
            // the plain order: lane tl of a team takes entries tl, tl + TS, ...
            const int team = l >> ps.lts, tl = l & (TS - 1);
            const size_t e = (size_t)q * TS + tl;
            const uint16_t cp = (team < ps.n && e < plain[team].size()) ? plain[team][e] : (uint16_t)na;
            if (std::find(seen_p.begin(), seen_p.end(), cp) == seen_p.end()) {
              seen_p.push_back(cp);
              ++load_p[cp & 31];
            }
          }
          cyc_sched += *std::max_element(load_s, load_s + 32);
          cyc_plain += *std::max_element(load_p, load_p + 32);
        }
      }
      for (const auto& pl : pool)
        if (!pl.empty()) return fail(WG_ERR_INVALID, "solo plan: entries left over");
      q0 += ps.L;
    }
    wslots[v] = q0;
  }
  wpass[kChainWaves] = (int32_t)ptab.size();
  const int64_t lds = al(off_dv + 4 * na) + 16 * (int64_t)ptab.size();  // + the pass table
  if (lds > kChainLds) return WG_ERR_UNSUPPORTED;
  p->solo_npass = (int32_t)ptab.size();
  if (ptab.empty()) ptab.push_back(int4{0, 0, 0, 0});
  std::vector<uint32_t> w((size_t)(E / 2) * T);
  for (int t = 0; t < T; ++t)
    for (int q = 0; q < E / 2; ++q)
      w[(size_t)q * T + t] = (uint32_t)slot[(size_t)t * E + 2 * q] | ((uint32_t)slot[(size_t)t * E + 2 * q + 1] << 16);
  const void* kern = solo_kernel(E);
  if (!kern) return WG_ERR_UNSUPPORTED;
  if (int rc = ensure_dyn_lds(kern, kChainLds)) return rc;
  p->P = 1;
  p->n_act = (int32_t)na;
  p->lds_bytes = (int32_t)lds;
  p->solo_E = E;
  p->ustride = (int32_t)((na + 63) / 64 * 64);
  int rc = upload(&p->sids, w);
  if (!rc) rc = upload(&p->spass, ptab);
  if (!rc) rc = upload(&p->swpass, wpass);
  if (!rc) rc = upload(&p->swslots, wslots);
  if (!rc) rc = dmalloc(&p->bar, 4);
  if (rc) return rc;
  WG_HIP_TRY(hipMemset(p->bar, 0, 4 * sizeof(int32_t)));
  WG_HIP_TRY(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
  WG_HIP_TRY(hipHostMalloc((void**)&p->host_flag, sizeof(int32_t), hipHostMallocMapped));
  *p->host_flag = 0;
  WG_HIP_TRY(hipHostGetDevicePointer((void**)&p->d_host_flag, p->host_flag, 0));
  p->seen = 0;
  char buf[256];
  snprintf(buf, sizeof(buf), "chain1: one launch per chain, 1 workers x %d threads (solo: %d slots per lane in "
           "registers, %d passes, busiest wave %lld slots), %lld active rows, %lld nonzeros, LDS %d B; LDS read "
           "cycles per phase %lld (plain order %lld)\n",
           T, E, (int)passes.size(), (long long)need, (long long)na, (long long)rp[na], p->lds_bytes,
           (long long)cyc_sched, (long long)cyc_plain);
  p->text = buf;
  return WG_OK;
}

int build_chain_plan(wg_laplacian_s* L, ChainPlan* p) {
  const int64_t na = L->n_active;
  std::vector<int32_t> rp(na + 1);
  WG_HIP_TRY(hipMemcpy(rp.data(), L->rowptr, sizeof(int32_t) * (na + 1), hipMemcpyDeviceToHost));
  const int64_t nnz = rp[na];
  std::vector<int32_t> col(std::max<int64_t>(nnz, 1));
  if (nnz) WG_HIP_TRY(hipMemcpy(col.data(), L->col, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
  std::vector<uint16_t> ids(std::max<int64_t>(nnz, 1));
  for (int64_t e = 0; e < nnz; ++e) {
    if (col[e] < 0 || col[e] >= na) return fail(WG_ERR_INVALID, "chain plan: column %d outside the active rows", col[e]);
    ids[e] = (uint16_t)col[e];
  }
  // one workgroup, ids in registers: auto up to kSoloMaxNnz entries (Cora-size K = 8: 29.3 vs 49.8 us per
  // chain; PubMed-size K = 16: 217 vs 78.4 with 128 workers -- one CU's VALU and LDS, r05 s19-s20), or
  // wherever it fits with chain_solo = 2
  if (L->tune.chain_wg <= 0 && (L->tune.chain_solo == 2 || (L->tune.chain_solo == 1 && nnz <= kSoloMaxNnz))) {
    const int rc = build_solo_plan(L, p, rp, ids);
    if (rc != WG_ERR_UNSUPPORTED) return rc;
    p->release();
  }
  // workers: contiguous row ranges of equal cost (entries + an epilogue weight per row); per worker,
  // wave passes dealt to its 16 waves by longest-first greedy balance
  const int64_t kRowCost = 4;
  const int64_t total = nnz + kRowCost * na;
  // one worker when its ids, passes and both u buffers fit LDS (no exchange at all), else chain_wg
  int P = L->tune.chain_wg > 0 ? L->tune.chain_wg : 1;
  static_assert(24576 <= kChainThreads * kStageMax, "active rows per staging thread");
  std::vector<int4> wd;
  std::vector<int2> passes;
  std::vector<int32_t> wpass;
  std::vector<uint16_t> wcols, lids;  // P > 1: each worker's gathered columns; the entries' local ids
  std::vector<int32_t> wcol_off;
  std::vector<uint16_t> bcols;        // P > 1: each worker's back-edge columns (direct mode polls them)
  std::vector<int32_t> bcol_off;
  std::vector<int32_t> local(na, -1);
  size_t lds = 0;
  // auto: one worker if it fits, else 128 with direct gathers (73.8 vs 80.9 us per PubMed-size chain at
  // 64; staged: 64 workers 79.5, 128 77.9; r04 s43), doubled until a worker fits LDS
  const int p_auto = L->tune.chain_direct ? 128 : 64;
  for (;; P = (P == 1 && L->tune.chain_wg <= 0) ? p_auto : 2 * P) {
    if (P > 1024) return WG_ERR_UNSUPPORTED;  // (and never more than can be resident: below)
    wd.assign(P, int4{0, 0, 0, 0});
    passes.clear();
    wpass.assign((size_t)P * (kChainWaves + 1), 0);
    wcols.clear();
    wcol_off.assign(P + 1, 0);
    bcols.clear();
    bcol_off.assign(P + 1, 0);
    lids.assign(ids.begin(), ids.end());
    lds = 0;
    int64_t r = 0;
    bool fits = true;
    // every worker's rows first: a worker's staging list needs its consumers
    std::vector<int32_t> owner(na, 0);
    for (int w = 0; w < P; ++w) {
      const int64_t goal = total * (w + 1) / P;
      const int64_t r0 = r;
      while (r < na && (w == P - 1 || rp[r] + kRowCost * r < goal)) ++r;
      wd[w] = int4{(int)r0, (int)r, rp[r0], rp[r]};
      for (int64_t i = r0; i < r; ++i) owner[i] = w;
    }
    // refs[c * P + w]: worker w gathers a row of worker c.  A worker overwrites the granule
    // buffer of phase j with phase j + 2 once it has staged phase j + 1 from the workers it
    // reads; a worker c that reads w must have finished reading w's phase j by then, which it
    // has once it published phase j + 1 -- so w also stages one granule of every worker that
    // reads it but that it does not read (directed graphs; symmetric ones have none)
    std::vector<char> refs((size_t)P * P, 0);
    if (P > 1)
      for (int w = 0; w < P; ++w)
        for (int64_t e = wd[w].z; e < wd[w].w; ++e) refs[(size_t)owner[ids[e]] * P + w] = 1;
    for (int w = 0; w < P && fits; ++w) {
      const int64_t r0 = wd[w].x;
      r = wd[w].y;
      std::vector<int2> wps;
      std::vector<int64_t> cost;
      make_passes(rp, r0, r, wps, cost);
      std::vector<int> order(wps.size());
      for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
      std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return cost[x] > cost[y]; });
      std::vector<int64_t> load(kChainWaves, 0);
      std::vector<std::vector<int2>> per(kChainWaves);
      for (int i : order) {
        const int v = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        load[v] += cost[i];
        per[v].push_back(wps[i]);
      }
      for (int v = 0; v < kChainWaves; ++v) {
        wpass[(size_t)w * (kChainWaves + 1) + v] = (int32_t)passes.size();
        passes.insert(passes.end(), per[v].begin(), per[v].end());
      }
      wpass[(size_t)w * (kChainWaves + 1) + kChainWaves] = (int32_t)passes.size();
      int64_t nu = na;
      if (P > 1) {  // the columns this worker's rows gather, ascending, and their local ids
        std::vector<int32_t> cs(ids.begin() + rp[r0], ids.begin() + rp[r]);
        for (int c = 0; c < P; ++c)  // back edges: a granule of each reader this worker does not read
          if (c != w && refs[(size_t)w * P + c] && !refs[(size_t)c * P + w] && wd[c].y > wd[c].x) {
            cs.push_back(wd[c].x);
            bcols.push_back((uint16_t)wd[c].x);
          }
        bcol_off[w + 1] = (int32_t)bcols.size();
        std::sort(cs.begin(), cs.end());
        cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
        for (size_t i = 0; i < cs.size(); ++i) {
          local[cs[i]] = (int32_t)i;
          wcols.push_back((uint16_t)cs[i]);
        }
        for (int64_t e = rp[r0]; e < rp[r]; ++e) lids[e] = (uint16_t)local[ids[e]];
        wcol_off[w + 1] = (int32_t)wcols.size();
        nu = (int64_t)cs.size();
      }
      const ChainLayout lay(nu, r - r0, rp[r] - rp[r0], (int64_t)wps.size(), P == 1);
      lds = std::max(lds, (size_t)lay.bytes);
      if (lay.bytes > kChainLds) fits = false;
    }
    if (fits) break;
  }
  // every worker spins on other workers' granules, so all P (x the XCD stride) workgroups must be
  // resident at once: never more than one per CU, and no more than the occupancy query admits for
  // this LDS size (a plain launch does not check; a shared GPU is caught by the wait timeout)
  {
    int dev = 0, per_cu = 0;
    WG_HIP_TRY(hipGetDevice(&dev));
    if (int rc = ensure_dyn_lds((const void*)cheb_chain1_kernel, kChainLds)) return rc;
    WG_HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)cheb_chain1_kernel, kChainThreads,
                                                            (lds + 15) / 16 * 16));
    const int64_t stride = (L->tune.chain_xcd && P <= 32) ? 8 : 1;
    const int64_t resident = (int64_t)n_cus(dev) * std::min(per_cu, 1);
    if ((int64_t)P * stride > resident) return WG_ERR_UNSUPPORTED;
  }
  p->P = P;
  p->n_act = (int32_t)na;
  p->lds_bytes = (int32_t)((lds + 15) / 16 * 16);
  p->ustride = (int32_t)((na + 63) / 64 * 64);
  if (wcols.empty()) wcols.push_back(0);
  if (bcols.empty()) bcols.push_back(0);
  int rc = upload(&p->ids, P == 1 ? ids : lids);
  if (!rc) rc = upload(&p->wcols, wcols);
  if (!rc) rc = upload(&p->gids, ids);
  if (!rc) rc = upload(&p->bcols, bcols);
  if (!rc) rc = upload(&p->bcol_off, bcol_off);
  if (!rc) rc = upload(&p->wcol_off, wcol_off);
  if (!rc) rc = upload(&p->wdesc, wd);
  if (!rc) rc = upload(&p->wpass, wpass);
  if (!rc) rc = upload(&p->passes, passes);
  if (!rc) rc = dmalloc(&p->bar, 4);
  if (!rc) rc = dmalloc(&p->gbuf, (size_t)4 * p->ustride);
  if (rc) return rc;
  WG_HIP_TRY(hipEventCreateWithFlags(&p->done, hipEventDisableTiming));
  WG_HIP_TRY(hipHostMalloc((void**)&p->host_flag, sizeof(int32_t), hipHostMallocMapped));
  *p->host_flag = 0;
  WG_HIP_TRY(hipHostGetDevicePointer((void**)&p->d_host_flag, p->host_flag, 0));
  p->seen = 0;
  WG_HIP_TRY(hipMemset(p->bar, 0, 4 * sizeof(int32_t)));
  WG_HIP_TRY(hipMemset(p->gbuf, 0, 4 * p->ustride * sizeof(uint64_t)));  // tag 0: never a live phase's
  char buf[192];
  snprintf(buf, sizeof(buf), "chain1: one launch per chain, %d workers x %d threads, %lld active rows, %lld nonzeros, "
           "%d wave passes, LDS %d B per worker\n", P, kChainThreads, (long long)na, (long long)nnz,
           (int)passes.size(), p->lds_bytes);
  p->text = buf;
  return WG_OK;
}

}  // namespace

void ChainPlan::release() {
  for (void* q : {(void*)ids, (void*)wcols, (void*)wcol_off, (void*)gids, (void*)bcols, (void*)bcol_off, (void*)wdesc, (void*)wpass, (void*)passes, (void*)bar,
                  (void*)gbuf, (void*)u0, (void*)x0, (void*)sids, (void*)spass, (void*)swpass, (void*)swslots})
    (void)hipFree(q);
  if (host_flag) (void)hipHostFree(host_flag);
  if (done) (void)hipEventDestroy(done);
  *this = ChainPlan{};
}

void release_chain1(wg_laplacian_s* L) {
  if (L->chain1) {
    L->chain1->release();
    delete L->chain1;
    L->chain1 = nullptr;
  }
  L->chain1_failed = false;
  L->chain1_off = false;  // a tune gives the one-launch chain another chance
}

int get_chain1_plan(wg_laplacian_s* L, int64_t F, int32_t K, ChainPlan** out) {
  *out = nullptr;
  const int64_t na = L->n_active;
  // F = 1, unweighted (value-free u), relabelled (active rows first), u of every active row in
  // LDS with 16-bit ids, launch-bound sizes (auto: <= 2^18 nonzeros), K within the argument block
  if (F != 1 || K < 1 || K > kChainMaxK || !L->unit || !L->reordered || L->n_cols != L->n_rows || na < 1 ||
      na > 24576 || L->tune.chain == 0 || (L->tune.chain < 0 && L->nnz > ((int64_t)1 << 18)) ||
      L->tune.uscale == 0)
    return WG_OK;
  if (L->chain1_failed || L->chain1_off) return WG_OK;
  if (!L->chain1) {
    auto* p = new ChainPlan();
    const int rc = build_chain_plan(L, p);
    if (rc) {
      p->release();
      delete p;
      if (rc != WG_ERR_UNSUPPORTED) return rc;
      L->chain1_failed = true;
      return WG_OK;
    }
    L->chain1 = p;
  }
  *out = L->chain1;
  return WG_OK;
}

int launch_chain1(wg_laplacian_s* L, ChainPlan* p, const float* X0, int32_t K, double s, float* S, float* H,
                  hipStream_t stream) {
  const int64_t n = L->n_rows;
  double coef = 0.0;  // closed-form rows: S = X0 * sum_k (-1)^k c_k
  for (int32_t k = 0; k <= K; ++k) coef += ((k & 1) ? -1.0 : 1.0) * std::exp(-s * (double)k);
  if (p->solo_E) {  // one workgroup (cheb_chain_solo_kernel), its own prologue
    SoloArgs a{};
    a.n_act = p->n_act;
    a.K = K;
    auto al = [](int64_t x) { return (int32_t)((x + 15) & ~(int64_t)15); };
    const int64_t na = p->n_act;
    a.off_ub = al(4 * (na + 1));
    a.off_x0 = al(a.off_ub + 4 * (na + 1));
    a.off_dv = al(a.off_x0 + 4 * na);
    a.off_pt = al(a.off_dv + 4 * na);
    a.n_pass = p->solo_npass;
    a.ids = p->sids;
    a.passes = p->spass;
    a.wpass = p->swpass;
    a.wslots = p->swslots;
    a.dinv = L->dinv;
    a.iso = L->iso;
    a.perm = L->perm;
    a.X0 = X0;
    a.n = n;
    a.coef = coef;
    a.S = S;
    a.H = H;
    for (int32_t k = 0; k <= K; ++k) a.c[k] = std::exp(-s * (double)k);
    const void* kern = solo_kernel(p->solo_E);
    if (!kern) return fail(WG_ERR_INVALID, "chain solo: no kernel for %d slots", p->solo_E);
    if (int rc = prof_mark(L, stream, true)) return rc;
    void* args[] = {&a};
    WG_HIP_TRY(hipLaunchKernel(kern, dim3(1), dim3(kChainThreads), args, (size_t)p->lds_bytes, stream));
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    WG_HIP_TRY(hipStreamIsCapturing(stream, &cs));
    if (cs == hipStreamCaptureStatusNone) WG_HIP_TRY(hipEventRecord(p->done, stream));
    p->done_stale = cs != hipStreamCaptureStatusNone;
    return prof_mark(L, stream, false);
  }
  if (int rc = ensure_dyn_lds((const void*)cheb_chain1_kernel, kChainLds)) return rc;
  static int wall_khz[64] = {0};  // the wall clock's rate per device (constant)
  int dev = 0;
  WG_HIP_TRY(hipGetDevice(&dev));
  if (dev >= 0 && dev < 64 && !wall_khz[dev]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) != hipSuccess || v <= 0) v = 100000;
    wall_khz[dev] = v;
  }
  ChainArgs a{};
  a.n_act = p->n_act;
  a.K = K;
  a.P = p->P;
  // one XCD holds 32 workers (one per CU): more would wait for residency that never comes
  a.stride = (L->tune.chain_xcd && p->P <= 32) ? 8 : 1;
  a.ustride = p->ustride;
  a.ids = p->ids;
  a.wcols = p->wcols;
  a.wcol_off = p->wcol_off;
  a.gids = p->gids;
  a.bcols = p->bcols;
  a.bcol_off = p->bcol_off;
  a.direct = (L->tune.chain_direct && p->P > 1) ? 1 : 0;
  a.wdesc = p->wdesc;
  a.wpass = p->wpass;
  a.passes = p->passes;
  a.rowptr = L->rowptr;
  a.dinv = L->dinv;
  a.iso = L->iso;
  a.perm = L->perm;
  a.X0 = X0;
  a.n = n;
  a.coef = coef;
  a.gbuf = p->gbuf;
  a.bar = p->bar;
  a.host_flag = p->d_host_flag;
  a.wait_ticks = (int64_t)((dev >= 0 && dev < 64) ? wall_khz[dev] : 100000) * 500;  // 0.5 s
  a.fault_phase = L->tune.chain_fault;
  a.S = S;
  a.H = H;
#ifdef WG_DEBUG_BOUNDS
  a.dbg_lds = p->lds_bytes;
#endif
  for (int32_t k = 0; k <= K; ++k) a.c[k] = std::exp(-s * (double)k);
  if (int rc = prof_mark(L, stream, true)) return rc;
  hipLaunchKernelGGL(cheb_chain1_kernel, dim3((unsigned)(p->P * a.stride)), dim3(kChainThreads), (size_t)p->lds_bytes,
                     stream, a);
  WG_LAUNCH_CHECK();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  WG_HIP_TRY(hipStreamIsCapturing(stream, &cs));
  if (cs == hipStreamCaptureStatusNone) WG_HIP_TRY(hipEventRecord(p->done, stream));
  p->done_stale = cs != hipStreamCaptureStatusNone;
  return prof_mark(L, stream, false);
}

void chain1_turn_off(wg_laplacian_s* L) {
  if (!L->chain1_off) ++L->tune_gen;  // a captured chain holding the one-launch kernel is re-captured
  L->chain1_off = true;
}

int chain1_check(wg_laplacian_s* L) {
  // a previous launch of the one-launch chain that gave up a wait (its S / H are NaN): reported
  // by the next call instead of launching over it (the flag is host-mapped: no sync)
  ChainPlan* p = L->chain1;
  if (!p || !p->host_flag) return WG_OK;
  const int32_t failed = __atomic_load_n(p->host_flag, __ATOMIC_ACQUIRE);
  if (failed == p->seen) return WG_OK;
  p->seen = failed;
  chain1_turn_off(L);  // later calls take the multi-launch path
  ++L->chain1_timeouts;
  return fail(WG_ERR_TIMEOUT,
              "wg_wavelet_features: a previous one-launch chain (csrc/chain.hip) gave up waiting for a worker; its "
              "S / H were written as NaN (was the GPU shared with another kernel?)");
}

int chain1_status(wg_laplacian_s* L, int32_t* timed_out) {
  *timed_out = 0;
  if (!L->chain1) return WG_OK;
  ChainPlan* p = L->chain1;
  if (p->done_stale)  // the last launch sits in a graph the caller replays: no event of ours follows it
    WG_HIP_TRY(hipDeviceSynchronize());
  else  // the handle's last one-launch chain only (eager, or replayed from the handle's own graph)
    WG_HIP_TRY(hipEventSynchronize(p->done));
  const int32_t failed = __atomic_load_n(p->host_flag, __ATOMIC_ACQUIRE);
  *timed_out = failed != p->seen ? 1 : 0;  // since the last report (here or by wg_wavelet_features)
  if (*timed_out) {  // later calls take the multi-launch path
    chain1_turn_off(L);
    ++L->chain1_timeouts;
  }
  p->seen = failed;
  return WG_OK;
}

}  // namespace wg
