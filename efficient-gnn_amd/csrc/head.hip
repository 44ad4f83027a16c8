// head.hip -- SURVEY section 8(f)-3: the WATS temperature head fused on the
// device (reference calibration/WATS.py:101-105 net, :124-130 forward):
//     t  = W2 relu(W1 h_i + b1) + b2          (Linear(F,16) - ReLU - Linear(16,1))
//     T  = log(exp(t) + 1.1)
//     out_i = log_softmax(logits_i / T)
// forward and backward (the gradients calib_train needs, WATS.py:145-151).
// One wave per row; the hidden units live on lanes 0..HID-1; the classes on
// all lanes.  The backward's parameter gradients are per-block float64
// partials reduced in block order by a second kernel (deterministic).
#include <algorithm>
#include <cmath>

#include "internal.h"

namespace wg {
namespace {

constexpr int kHeadBlocks = 1024;

struct HeadArgs {
  int64_t n, F, C;
  int32_t hid;
  const float* H;
  const float* logits;
  const float* W1;  // [hid][F]
  const float* b1;  // [hid]
  const float* W2;  // [hid]
  const float* b2;  // [1]
};

// lanes < hid: pre-activation of hidden unit `lane`; returns t (wave-uniform)
__device__ __forceinline__ float head_mlp(const HeadArgs& a, int64_t row, int lane, float& pre) {
  pre = 0.0f;
  float contrib = 0.0f;
  if (lane < a.hid) {
    float acc = a.b1[lane];
    const float* h = a.H + row * a.F;
    const float* w = a.W1 + (int64_t)lane * a.F;
    for (int64_t f = 0; f < a.F; ++f) acc = fmaf(w[f], h[f], acc);
    pre = acc;
    contrib = a.W2[lane] * fmaxf(acc, 0.0f);
  }
  for (int off = 32; off >= 1; off >>= 1) contrib += __shfl_xor(contrib, off, 64);  // same sum on every lane
  return contrib + a.b2[0];
}

__device__ __forceinline__ float wave_max(float v) {
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__global__ __launch_bounds__(kBlock) void head_forward_kernel(HeadArgs a, float* __restrict__ out,
                                                              float* __restrict__ t_save) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < a.n; row += waves) {
    float pre;
    const float t = head_mlp(a, row, lane, pre);
    const float T = logf(expf(t) + 1.1f);  // WATS.py:125
    if (lane == 0 && t_save) t_save[row] = t;
    const float* lg = a.logits + row * a.C;
    float m = -INFINITY;
    for (int64_t c = lane; c < a.C; c += 64) m = fmaxf(m, lg[c] / T);
    m = wave_max(m);
    float s = 0.0f;
    for (int64_t c = lane; c < a.C; c += 64) s += expf(lg[c] / T - m);
    s = wave_sum(s);
    const float ls = logf(s);
    for (int64_t c = lane; c < a.C; c += 64) out[row * a.C + c] = lg[c] / T - m - ls;  // WATS.py:128-130
  }
}

// partial layout per block: gW1 [hid*F], gb1 [hid], gW2 [hid], gb2 [1]
__global__ __launch_bounds__(kBlock) void head_backward_kernel(HeadArgs a, const float* __restrict__ out,
                                                               const float* __restrict__ t_save,
                                                               const float* __restrict__ gout,
                                                               float* __restrict__ glogits,
                                                               double* __restrict__ partial) {
  extern __shared__ double g_head_red[];  // [4 waves][P]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t P = (int64_t)a.hid * a.F + 2 * a.hid + 1;
  double* mine = g_head_red + wave * P;
  for (int64_t i = lane; i < P; i += 64) mine[i] = 0.0;
  const int64_t waves = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < a.n; row += waves) {
    float pre;
    const float t = t_save ? t_save[row] : head_mlp(a, row, lane, pre);
    if (t_save) (void)head_mlp(a, row, lane, pre);  // hidden pre-activations again (cheap)
    const float et = expf(t);
    const float T = logf(et + 1.1f);
    const float* lg = a.logits + row * a.C;
    const float* go = gout + row * a.C;
    const float* lp = out + row * a.C;
    // d log_softmax: dcal_c = g_c - p_c * sum_c g_c ; cal = logits / T
    float gs = 0.0f;
    for (int64_t c = lane; c < a.C; c += 64) gs += go[c];
    gs = wave_sum(gs);
    float dTs = 0.0f;  // sum_c dcal_c * logits_c
    for (int64_t c = lane; c < a.C; c += 64) {
      const float dcal = go[c] - expf(lp[c]) * gs;
      if (glogits) glogits[row * a.C + c] = dcal / T;
      dTs += dcal * lg[c];
    }
    dTs = wave_sum(dTs);
    const double dT = -(double)dTs / ((double)T * (double)T);
    const double dt = dT * (double)et / ((double)et + 1.1);  // d log(e^t + 1.1) / dt
    if (lane < a.hid) {
      const float z = fmaxf(pre, 0.0f);
      mine[(int64_t)a.hid * a.F + a.hid + lane] += dt * (double)z;        // gW2
      const double dz = (pre > 0.0f) ? dt * (double)a.W2[lane] : 0.0;
      mine[(int64_t)a.hid * a.F + lane] += dz;                             // gb1
      const float* h = a.H + row * a.F;
      for (int64_t f = 0; f < a.F; ++f) mine[(int64_t)lane * a.F + f] += dz * (double)h[f];  // gW1
    }
    if (lane == 0) mine[P - 1] += dt;  // gb2
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < P; i += kBlock) {
    double s = 0.0;
    for (int w = 0; w < 4; ++w) s += g_head_red[w * P + i];  // wave order
    partial[(int64_t)blockIdx.x * P + i] = s;
  }
}

__global__ void head_reduce_kernel(int64_t P, int nblocks, const double* __restrict__ partial, int32_t hid, int64_t F,
                                   float* __restrict__ gW1, float* __restrict__ gb1, float* __restrict__ gW2,
                                   float* __restrict__ gb2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  double s = 0.0;
  for (int b = 0; b < nblocks; ++b) s += partial[(int64_t)b * P + i];  // block order
  const int64_t nw1 = (int64_t)hid * F;
  if (i < nw1) gW1[i] = (float)s;
  else if (i < nw1 + hid) gb1[i - nw1] = (float)s;
  else if (i < nw1 + 2 * hid) gW2[i - nw1 - hid] = (float)s;
  else gb2[0] = (float)s;
}

int head_args(int64_t n, int64_t F, int64_t C, int32_t hid, const float* H, const float* logits, const float* W1,
              const float* b1, const float* W2, const float* b2, HeadArgs* a) {
  if (n < 0 || F < 1 || C < 1 || hid < 1 || hid > 64 || (n > 0 && (!H || !logits)) || !W1 || !b1 || !W2 || !b2)
    return fail(WG_ERR_INVALID, "wats_head: bad arguments (n=%lld F=%lld C=%lld hid=%d)", (long long)n, (long long)F,
                (long long)C, hid);
  *a = HeadArgs{n, F, C, hid, H, logits, W1, b1, W2, b2};
  return WG_OK;
}

int head_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(kHeadBlocks, ceil_div(n, 4))); }

}  // namespace
}  // namespace wg

using namespace wg;

extern "C" {

int wg_wats_head_forward(int64_t n, int64_t F, int64_t C, int32_t hid, const float* H, const float* logits,
                         const float* W1, const float* b1, const float* W2, const float* b2, float* out, float* t_save,
                         void* stream_) {
  HeadArgs a;
  if (int rc = head_args(n, F, C, hid, H, logits, W1, b1, W2, b2, &a)) return rc;
  if (n > 0 && !out) return fail(WG_ERR_INVALID, "wats_head_forward: out is NULL");
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(head_forward_kernel, dim3(head_blocks(n)), dim3(kBlock), 0, as_stream(stream_), a, out, t_save);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int wg_wats_head_workspace(int64_t n, int64_t F, int32_t hid, int64_t* bytes) {
  if (!bytes || n < 0 || F < 1 || hid < 1) return fail(WG_ERR_INVALID, "wats_head_workspace: bad arguments");
  *bytes = (int64_t)head_blocks(n) * ((int64_t)hid * F + 2 * hid + 1) * (int64_t)sizeof(double);
  return WG_OK;
}

int wg_wats_head_backward(int64_t n, int64_t F, int64_t C, int32_t hid, const float* H, const float* logits,
                          const float* W1, const float* b1, const float* W2, const float* b2, const float* out,
                          const float* t_save, const float* grad_out, float* grad_logits, float* gW1, float* gb1,
                          float* gW2, float* gb2, void* workspace, void* stream_) {
  HeadArgs a;
  if (int rc = head_args(n, F, C, hid, H, logits, W1, b1, W2, b2, &a)) return rc;
  if (!gW1 || !gb1 || !gW2 || !gb2 || !workspace || (n > 0 && (!out || !grad_out)))
    return fail(WG_ERR_INVALID, "wats_head_backward: NULL argument");
  hipStream_t stream = as_stream(stream_);
  const int64_t P = (int64_t)hid * F + 2 * hid + 1;
  const size_t lds = (size_t)4 * P * sizeof(double);
  if (lds > 64 * 1024) return fail(WG_ERR_UNSUPPORTED, "wats_head_backward: hid*F too large (%lld)", (long long)P);
  const int nb = head_blocks(n);
  if (n > 0) {
    hipLaunchKernelGGL(head_backward_kernel, dim3(nb), dim3(kBlock), lds, stream, a, out, t_save, grad_out,
                       grad_logits, static_cast<double*>(workspace));
    WG_LAUNCH_CHECK();
  } else {
    WG_HIP_TRY(hipMemsetAsync(workspace, 0, (size_t)nb * P * sizeof(double), stream));
  }
  hipLaunchKernelGGL(head_reduce_kernel, dim3((unsigned)ceil_div(P, 256)), dim3(256), 0, stream, P, nb,
                     static_cast<const double*>(workspace), hid, F, gW1, gb1, gW2, gb2);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // extern "C"
