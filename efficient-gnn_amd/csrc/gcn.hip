// gcn.hip -- SURVEY section 8(f)-2: the propagation of the base model WATS
// wraps, CompatibleGCN.forward (reference src/gnn/model.py:43-52):
//     deg = adj.sum(dim=1); deg[deg == 0] = 1; adj_norm = adj / deg
//     x -> adj_norm @ x           (twice per forward)
// as a CSR SpMM on the Chebyshev step kernel (a k = 1 step of an operator
// whose entries are adj_norm's: every entry kept, self loops included, no
// isolated diagonal).  The transpose operator (for the backward,
// d(adj_norm @ x)/dx^T g = adj_norm^T g) is built on the device by a stable
// radix sort of the entries by column.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "internal.h"

namespace wg {
namespace {

// deg_i = sum_j a_ij (float64 sum, float32 result), 0 -> 1 (model.py:43-44)
__global__ __launch_bounds__(kBlock) void gcn_degree_kernel(int64_t n, const int64_t* __restrict__ indptr,
                                                            const float* __restrict__ values, float* __restrict__ deg) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  double s = 0.0;
  for (int64_t e = indptr[row] + lane; e < indptr[row + 1]; e += 64) s += values ? (double)values[e] : 1.0;
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_down(s, off, 64);
  if (lane == 0) {
    const float d = (float)s;
    deg[row] = (d == 0.0f) ? 1.0f : d;
  }
}

// adj_norm entries a_ij / deg_i (float32 IEEE division, as torch's adj / deg), and each entry's row
__global__ __launch_bounds__(kBlock) void gcn_norm_kernel(int64_t n, const int64_t* __restrict__ indptr,
                                                          const float* __restrict__ values,
                                                          const float* __restrict__ deg, float* __restrict__ out,
                                                          int32_t* __restrict__ row_of) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const float d = deg[row];
  for (int64_t e = indptr[row] + lane; e < indptr[row + 1]; e += 64) {
    out[e] = (values ? values[e] : 1.0f) / d;
    row_of[e] = (int32_t)row;
  }
}

__global__ void gcn_iota_kernel(int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)i;
}

__global__ void gcn_count_kernel(int64_t nnz, const int32_t* __restrict__ keys, int64_t* __restrict__ cnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) atomicAdd(reinterpret_cast<unsigned long long*>(cnt + keys[e]), 1ull);
}

// transposed entry t (sorted by column, stable): column = original row, value = original value
__global__ void gcn_gather_t_kernel(int64_t nnz, const int32_t* __restrict__ order, const int32_t* __restrict__ row_of,
                                    const float* __restrict__ val, int32_t* __restrict__ idx_t,
                                    float* __restrict__ val_t) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nnz) return;
  const int32_t e = order[t];
  idx_t[t] = row_of[e];
  val_t[t] = val[e];
}

template <typename F_>
int cub_run(hipStream_t stream, F_&& fn) {
  size_t bytes = 0;
  WG_HIP_TRY(fn(nullptr, bytes));
  void* tmp = nullptr;
  WG_HIP_TRY(hipMalloc(&tmp, std::max<size_t>(bytes, 1)));
  hipError_t e = fn(tmp, bytes);
  hipError_t e2 = hipStreamSynchronize(stream);
  (void)hipFree(tmp);
  WG_HIP_TRY(e);
  WG_HIP_TRY(e2);
  return WG_OK;
}

struct Bufs {
  std::vector<void*> p;
  template <typename T>
  int alloc(T** out, size_t n) {
    int rc = dmalloc(out, n);
    if (!rc) p.push_back(*out);
    return rc;
  }
  ~Bufs() {
    for (void* q : p) (void)hipFree(q);
  }
};

}  // namespace
}  // namespace wg

using namespace wg;

extern "C" {

int wg_rownorm_create(int64_t n, int64_t nnz, const int64_t* indptr, const int32_t* indices, const float* values,
                      uint32_t flags, void* stream_, wg_laplacian_t* out) {
  if (!out) return fail(WG_ERR_INVALID, "wg_rownorm_create: out is NULL");
  *out = nullptr;
  if (n < 0 || nnz < 0 || !indptr || (nnz > 0 && !indices))
    return fail(WG_ERR_INVALID, "wg_rownorm_create: bad shape (n=%lld nnz=%lld)", (long long)n, (long long)nnz);
  if (nnz > INT32_MAX || n > INT32_MAX) return fail(WG_ERR_UNSUPPORTED, "wg_rownorm_create: nnz/n exceed int32");
  hipStream_t stream = as_stream(stream_);
  Bufs tmp;
  float *deg, *vnorm;
  int32_t* row_of;
  int rc = 0;
  if ((rc = tmp.alloc(&deg, n)) || (rc = tmp.alloc(&vnorm, nnz)) || (rc = tmp.alloc(&row_of, nnz))) return rc;
  if (n > 0) {
    hipLaunchKernelGGL(gcn_degree_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(kBlock), 0, stream, n, indptr, values,
                       deg);
    WG_LAUNCH_CHECK();
    hipLaunchKernelGGL(gcn_norm_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(kBlock), 0, stream, n, indptr, values, deg,
                       vnorm, row_of);
    WG_LAUNCH_CHECK();
  }
  const int64_t* op_indptr = indptr;
  const int32_t* op_indices = indices;
  const float* op_values = vnorm;
  int64_t* indptr_t = nullptr;
  int32_t* idx_t = nullptr;
  float* val_t = nullptr;
  if (flags & WG_FLAG_TRANSPOSE) {
    // stable radix sort of the entry ids by column -> CSR of adj_norm^T
    int32_t *ids, *order, *keys_sorted;
    if ((rc = tmp.alloc(&ids, nnz)) || (rc = tmp.alloc(&order, nnz)) || (rc = tmp.alloc(&keys_sorted, nnz)) ||
        (rc = tmp.alloc(&indptr_t, n + 1)) || (rc = tmp.alloc(&idx_t, nnz)) || (rc = tmp.alloc(&val_t, nnz)))
      return rc;
    WG_HIP_TRY(hipMemsetAsync(indptr_t, 0, sizeof(int64_t) * (n + 1), stream));
    if (nnz > 0) {
      hipLaunchKernelGGL(gcn_iota_kernel, dim3((unsigned)ceil_div(nnz, 256)), dim3(256), 0, stream, nnz, ids);
      WG_LAUNCH_CHECK();
      int end_bit = 1;
      while (end_bit < 32 && (1ll << end_bit) < n) ++end_bit;
      rc = cub_run(stream, [&](void* t, size_t& b) {
        return hipcub::DeviceRadixSort::SortPairs(t, b, indices, keys_sorted, ids, order, (int)nnz, 0, end_bit, stream);
      });
      if (rc) return rc;
      hipLaunchKernelGGL(gcn_count_kernel, dim3((unsigned)ceil_div(nnz, 256)), dim3(256), 0, stream, nnz, indices,
                         indptr_t + 1);
      WG_LAUNCH_CHECK();
      rc = cub_run(stream, [&](void* t, size_t& b) {
        return hipcub::DeviceScan::InclusiveSum(t, b, indptr_t + 1, indptr_t + 1, (int)n, stream);
      });
      if (rc) return rc;
      hipLaunchKernelGGL(gcn_gather_t_kernel, dim3((unsigned)ceil_div(nnz, 256)), dim3(256), 0, stream, nnz, order,
                         row_of, vnorm, idx_t, val_t);
      WG_LAUNCH_CHECK();
    }
    op_indptr = indptr_t;
    op_indices = idx_t;
    op_values = val_t;
  }
  auto* L = new wg_laplacian_s();
  if (hipGetDevice(&L->device) != hipSuccess) {
    delete L;
    return fail(WG_ERR_HIP, "wg_rownorm_create: no HIP device");
  }
  L->n_rows = n;
  L->n_cols = n;
  L->nnz_input = nnz;
  L->reordered = !(flags & WG_FLAG_NO_REORDER);
  rc = build_operator(L, op_indptr, op_indices, op_values, nullptr, /*raw=*/true, stream);
  if (rc == WG_OK && !(flags & WG_FLAG_KEEP_COLUMN_ORDER)) rc = sort_row_columns(L, stream);
  if (rc == WG_OK && hipStreamSynchronize(stream) != hipSuccess) rc = fail(WG_ERR_HIP, "wg_rownorm_create: sync");
  if (rc != WG_OK) {
    (void)hipStreamSynchronize(stream);
    delete L;
    return rc;
  }
  *out = L;
  return WG_OK;
}

int wg_spmm(wg_laplacian_t P, int64_t F, const float* x, float* y, void* stream_) {
  if (!P || F < 1 || (P->n_rows && (!x || !y))) return fail(WG_ERR_INVALID, "wg_spmm: bad arguments");
  if (P->n_cols != P->n_rows) return fail(WG_ERR_INVALID, "wg_spmm: sharded handle");
  hipStream_t stream = as_stream(stream_);
  const int64_t n = P->n_rows;
  if (n == 0) return WG_OK;
  if (!P->reordered) return launch_step(P, 1, F, x, nullptr, y, nullptr, nullptr, 1.0, 0.0, stream);
  // internal (degree-sorted) order: permute in, one k = 1 step, permute out
  const size_t stride = ((size_t)n * F + 63) / 64 * 64;
  if (P->ws_floats < 2 * stride) {
    WG_HIP_TRY(hipStreamSynchronize(stream));
    (void)hipFree(P->ws);
    P->ws = nullptr;
    P->ws_floats = 0;
    WG_HIP_TRY(hipMalloc(&P->ws, 2 * stride * sizeof(float)));
    P->ws_floats = 2 * stride;
  }
  float* xi = P->ws;
  float* yi = P->ws + stride;
  int rc = launch_permute(P, 0, F, x, xi, stream);
  if (!rc) rc = launch_step(P, 1, F, xi, nullptr, yi, nullptr, nullptr, 1.0, 0.0, stream);
  if (!rc) rc = launch_permute(P, 1, F, yi, y, stream);
  return rc;
}

}  // extern "C"
