// prologue.hip -- building L_hat on the device (reference a1 + a2 + a3):
//   compute_normalized_laplacian  calibration/WATS.py:24-27
//     = scipy.sparse.csgraph.laplacian(adj, normed=True), _laplacian.py:467-475
//   rescale  (2/2.0)*L - identity(N)  calibration/WATS.py:55
//   X0 = log1p(adj.sum(axis=1))      calibration/WATS.py:58-59
// plus the dense-adjacency ingestion that replaces csr_matrix(adj.cpu().numpy())
// (WATS.py:99) and the shard degree helper.
//
// Exactness: scipy computes w = A.sum(axis=0) - A.diagonal() in float32.  Its
// column sum is `ones(1,M) @ A`, i.e. a CSC mat-vec that adds each column's
// entries sequentially in ascending row order, in float32.  For unweighted
// graphs (values == NULL) the sum is an integer, so a float64 atomic sum is
// exact.  For weighted graphs the prologue reproduces the sequential order:
// entries are stably sorted by column (CSR order is row-major, so each
// column's entries stay in ascending row order) and summed by one thread per
// column in float32.  The values are then -((a_ij / sw_i) / sw_j) with IEEE
// division and sqrt (no fast-math), i.e. bit-identical to scipy.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <vector>

#include "internal.h"

namespace wg {
namespace {

// Wave per row: off-diagonal count, row sum incl. diagonal (float64), diagonal
// value, optional float64 column sums (unweighted path).
__global__ __launch_bounds__(kBlock) void row_info_kernel(
    int64_t n_rows, const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices,
    const float* __restrict__ values, int32_t* __restrict__ offdiag_len, double* __restrict__ rowsum,
    float* __restrict__ diag, double* __restrict__ colsum, int32_t* __restrict__ colcnt, int32_t* __restrict__ nonunit,
    int raw) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int64_t e0 = indptr[row], e1 = indptr[row + 1];
  int cnt = 0;
  double rs = 0.0;
  float dg = 0.0f;
  for (int64_t e = e0 + lane; e < e1; e += 64) {
    const int32_t c = indices[e];
    const float v = values ? values[e] : 1.0f;
    rs += (double)v;
    if (c == row && !raw) {
      dg += v;
    } else {
      ++cnt;
      atomicAdd(colcnt + c, 1);
      if (v != 1.0f) *nonunit = 1;  // weighted off-diagonal entry
    }
    if (colsum) atomicAdd(colsum + c, (double)v);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    cnt += __shfl_down(cnt, off, 64);
    rs += __shfl_down(rs, off, 64);
    dg += __shfl_down(dg, off, 64);
  }
  if (lane == 0) {
    offdiag_len[row] = cnt;
    rowsum[row] = rs;
    diag[row] = dg;
  }
}

__global__ void f64_to_f32_kernel(int64_t n, const double* __restrict__ in, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (float)in[i];
}

// column entry counts (for the weighted path's column pointers)
__global__ void col_count_kernel(int64_t nnz, const int32_t* __restrict__ indices, int32_t* __restrict__ cnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < nnz) atomicAdd(cnt + indices[e], 1);
}

// scipy's float32 sequential column sum over entries sorted by (column, row)
__global__ void col_seq_sum_kernel(int64_t n_cols, const int32_t* __restrict__ colptr,
                                   const float* __restrict__ sorted_vals, float* __restrict__ colsum) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_cols) return;
  float s = 0.0f;
  for (int32_t e = colptr[c]; e < colptr[c + 1]; ++e) s += sorted_vals[e];
  colsum[c] = s;
}

// w_j = colsum_j - diag_j (float32, scipy), sw_j = w_j == 0 ? 1 : sqrt(w_j), iso_j = (w_j == 0)
__global__ void degree_kernel(int64_t n_cols, int64_t n_rows, const float* __restrict__ colsum,
                              const float* __restrict__ diag, const float* __restrict__ w_cols,
                              float* __restrict__ sw, uint8_t* __restrict__ iso_col) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_cols) return;
  const float w = w_cols ? w_cols[j] : colsum[j] - (j < n_rows ? diag[j] : 0.0f);
  const bool iso = (w == 0.0f);
  sw[j] = iso ? 1.0f : sqrtf(w);
  iso_col[j] = iso ? 1 : 0;
}

// dinv in the internal column order: 1 / sw (float64), sw as scipy's float32
__global__ void dinv_kernel(int64_t n_cols, int64_t n_rows, const int32_t* __restrict__ perm, const float* __restrict__ sw,
                            double* __restrict__ dinv) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_cols) return;
  const int64_t src = (j < n_rows) ? perm[j] : j;
  dinv[j] = 1.0 / (double)sw[src];
}

// Sort key: off-diagonal length, then "needed in the chain" (0 for purely
// isolated rows: w_i == 0, no off-diagonal entries in row i or column i --
// T_k,i = (-1)^k X0_i in closed form and no other row gathers it).
__global__ void sort_key_kernel(int64_t n, const int32_t* __restrict__ len, const int32_t* __restrict__ colcnt,
                                const uint8_t* __restrict__ iso_col, int allow_closed, unsigned long long* __restrict__ key) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool pure = allow_closed && iso_col[i] && len[i] == 0 && colcnt[i] == 0;
  key[i] = ((unsigned long long)len[i] << 1) | (pure ? 0ull : 1ull);
}

__global__ void count_pure_kernel(int64_t n, const unsigned long long* __restrict__ key, unsigned int* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && key[i] == 0ull) atomicAdd(cnt, 1u);
}

__global__ void iota_kernel(int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)i;
}

__global__ void invert_perm_kernel(int64_t n, const int32_t* __restrict__ perm, int32_t* __restrict__ iperm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) iperm[perm[i]] = (int32_t)i;
}

__global__ void gather_len_kernel(int64_t n, const int32_t* __restrict__ perm, const int32_t* __restrict__ len,
                                  int32_t* __restrict__ out, const uint8_t* __restrict__ iso_col,
                                  uint8_t* __restrict__ iso_row) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int32_t r = perm[i];
    out[i] = len[r];
    iso_row[i] = iso_col[r];
  }
}

// Wave per internal row: the original row's off-diagonal entries (column order
// preserved), relabelled columns, scipy-exact L_hat value.
__global__ __launch_bounds__(kBlock) void fill_lhat_kernel(
    int64_t n_rows, const int32_t* __restrict__ perm, const int32_t* __restrict__ iperm,
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, const float* __restrict__ values,
    const float* __restrict__ sw, const int32_t* __restrict__ rowptr, int32_t* __restrict__ col,
    float* __restrict__ val, int raw) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n_rows) return;
  const int32_t r = perm[i];
  const float swr = sw[r];
  const int64_t e0 = indptr[r], e1 = indptr[r + 1];
  int32_t pos = rowptr[i];
  for (int64_t base = e0; base < e1; base += 64) {
    const int64_t e = base + lane;
    int32_t c = 0;
    bool keep = false;
    if (e < e1) {
      c = indices[e];
      keep = raw || (c != r);
    }
    const unsigned long long m = __ballot(keep);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (keep) {
      const float a = values ? values[e] : 1.0f;
      // scipy _laplacian.py:472-474: data /= w[row]; data /= w[col]; data *= -1
      col[pos + before] = (c < n_rows) ? iperm[c] : c;
      val[pos + before] = raw ? a : -((a / swr) / sw[c]);
    }
    pos += __popcll(m);
  }
}

__global__ void bucket_hist_kernel(int64_t n, const int32_t* __restrict__ len, unsigned int* __restrict__ hist) {
  __shared__ unsigned int h[kBuckets];
  if (threadIdx.x < kBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = len[i];
    const int b = (l > 1) ? 32 - __clz(l - 1) : 0;  // ceil(log2 l)
    atomicAdd(h + b, 1u);
  }
  __syncthreads();
  if (threadIdx.x < kBuckets && h[threadIdx.x]) atomicAdd(hist + threadIdx.x, h[threadIdx.x]);
}

__global__ __launch_bounds__(kBlock) void dense_count_kernel(int64_t n_rows, int64_t n_cols, int64_t ld,
                                                             const float* __restrict__ adj,
                                                             int64_t* __restrict__ counts) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const float* p = adj + row * ld;
  int64_t cnt = 0;
  for (int64_t c = lane; c < n_cols; c += 64) cnt += (p[c] != 0.0f);
  for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_down(cnt, off, 64);
  if (lane == 0) counts[row] = cnt;
}

__global__ __launch_bounds__(kBlock) void dense_fill_kernel(int64_t n_rows, int64_t n_cols, int64_t ld,
                                                            const float* __restrict__ adj,
                                                            const int64_t* __restrict__ indptr,
                                                            int32_t* __restrict__ indices, float* __restrict__ values) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const float* p = adj + row * ld;
  int64_t pos = indptr[row];
  for (int64_t base = 0; base < n_cols; base += 64) {
    const int64_t c = base + lane;
    const float v = (c < n_cols) ? p[c] : 0.0f;
    const bool nz = (v != 0.0f);
    const unsigned long long m = __ballot(nz);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (nz) {
      indices[pos + before] = (int32_t)c;
      values[pos + before] = v;
    }
    pos += __popcll(m);
  }
}

__global__ __launch_bounds__(kBlock) void column_degree_kernel(int64_t n_rows, int64_t row_offset,
                                                               const int64_t* __restrict__ indptr,
                                                               const int32_t* __restrict__ indices,
                                                               const float* __restrict__ values,
                                                               double* __restrict__ colsum,
                                                               double* __restrict__ diag) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int64_t grow = row + row_offset;
  for (int64_t e = indptr[row] + lane; e < indptr[row + 1]; e += 64) {
    const int32_t c = indices[e];
    const double v = values ? (double)values[e] : 1.0;
    atomicAdd(colsum + c, v);
    if (c == grow) atomicAdd(diag + grow, v);
  }
}

__global__ void export_len_kernel(int64_t n, const int32_t* __restrict__ iperm, const int32_t* __restrict__ rowptr,
                                  int64_t* __restrict__ lens) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const int32_t i = iperm[r];
  lens[r] = rowptr[i + 1] - rowptr[i];
}

__global__ void export_fill_kernel(int64_t n_rows, const int32_t* __restrict__ perm, const int32_t* __restrict__ iperm,
                                   const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                   const float* __restrict__ val, const int64_t* __restrict__ out_ptr,
                                   int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rows) return;
  const int32_t i = iperm[r];
  int64_t o = out_ptr[r];
  for (int32_t e = rowptr[i]; e < rowptr[i + 1]; ++e, ++o) {
    const int32_t c = col[e];
    out_idx[o] = (c < n_rows) ? perm[c] : c;
    out_val[o] = val[e];
  }
}

__global__ void export_iso_kernel(int64_t n, const int32_t* __restrict__ iperm, const uint8_t* __restrict__ iso,
                                  uint8_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n) out[r] = iso[iperm[r]];
}

__global__ void log1p_degree_kernel(int64_t n, const float* __restrict__ rowsum, float* __restrict__ x0) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x0[i] = (float)log1p((double)rowsum[i]);
}

template <typename F_>
int cub_call(hipStream_t stream, F_&& fn) {
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

// RAII list of temporary device buffers
struct Scratch {
  std::vector<void*> bufs;
  template <typename T>
  int alloc(T** p, size_t n) {
    int rc = dmalloc(p, n);
    if (!rc) bufs.push_back(*p);
    return rc;
  }
  ~Scratch() {
    for (void* p : bufs) (void)hipFree(p);
  }
};

}  // namespace

// raw = false: L_hat of the adjacency (the Laplacian prologue).  raw = true: a
// general CSR operator -- every entry kept with its given value, no isolated
// diagonal, no closed-form rows (the row-normalised GCN adjacency, gcn.hip).
int build_operator(wg_laplacian_s* L, const int64_t* indptr, const int32_t* indices, const float* values,
                   const float* w_cols, bool raw, hipStream_t stream) {
  const int64_t n_rows = L->n_rows, n_cols = L->n_cols, nnz = L->nnz_input;
  const int64_t nb_rows = std::max<int64_t>(1, ceil_div(n_rows, 256));
  const int64_t nb_cols = std::max<int64_t>(1, ceil_div(n_cols, 256));
  Scratch tmp;
  int32_t *len, *len_sorted, *ids;
  double* rowsum64;
  float *diag, *colsum32, *sw;
  double* colsum64 = nullptr;
  uint8_t* iso_col;
  unsigned int* hist;
  int rc = 0;
  int32_t* colcnt;
  unsigned long long *key, *key_sorted;
  unsigned int* npure_d;
  int32_t* nonunit_d;
  if ((rc = tmp.alloc(&colcnt, n_cols)) || (rc = tmp.alloc(&key, n_rows)) || (rc = tmp.alloc(&key_sorted, n_rows)) ||
      (rc = tmp.alloc(&npure_d, 1)) || (rc = tmp.alloc(&nonunit_d, 1)))
    return rc;
  WG_HIP_TRY(hipMemsetAsync(nonunit_d, 0, sizeof(int32_t), stream));
  WG_HIP_TRY(hipMemsetAsync(colcnt, 0, sizeof(int32_t) * std::max<int64_t>(1, n_cols), stream));
  if ((rc = tmp.alloc(&len, n_rows)) || (rc = tmp.alloc(&len_sorted, n_rows)) || (rc = tmp.alloc(&ids, n_rows)) ||
      (rc = tmp.alloc(&rowsum64, n_rows)) || (rc = tmp.alloc(&diag, n_rows)) || (rc = tmp.alloc(&colsum32, n_cols)) ||
      (rc = tmp.alloc(&sw, n_cols)) || (rc = tmp.alloc(&iso_col, n_cols)) || (rc = tmp.alloc(&hist, kBuckets)))
    return rc;
  if ((rc = dmalloc(&L->rowptr, n_rows + 1)) || (rc = dmalloc(&L->iso, n_rows)) || (rc = dmalloc(&L->perm, n_rows)) ||
      (rc = dmalloc(&L->iperm, n_rows)) || (rc = dmalloc(&L->rowsum, n_rows)) || (rc = dmalloc(&L->dinv, n_cols)))
    return rc;
  const bool unweighted_colsum = (w_cols == nullptr) && (values == nullptr);
  if (unweighted_colsum) {
    if ((rc = tmp.alloc(&colsum64, n_cols))) return rc;
    WG_HIP_TRY(hipMemsetAsync(colsum64, 0, sizeof(double) * std::max<int64_t>(1, n_cols), stream));
  }
  if (n_rows > 0) {
    hipLaunchKernelGGL(row_info_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, stream, n_rows, indptr, indices,
                       values, len, rowsum64, diag, colsum64, colcnt, nonunit_d, raw ? 1 : 0);
    WG_LAUNCH_CHECK();
  }
  if (w_cols == nullptr && n_cols > 0) {
    if (unweighted_colsum) {
      hipLaunchKernelGGL(f64_to_f32_kernel, dim3(nb_cols), dim3(256), 0, stream, n_cols, colsum64, colsum32);
      WG_LAUNCH_CHECK();
    } else if (nnz == 0) {
      WG_HIP_TRY(hipMemsetAsync(colsum32, 0, sizeof(float) * n_cols, stream));
    } else {
      // scipy order: stable sort by column, sequential float32 sum per column
      int32_t *keys_out, *colptr;
      float* vals_out;
      if ((rc = tmp.alloc(&keys_out, nnz)) || (rc = tmp.alloc(&vals_out, nnz)) || (rc = tmp.alloc(&colptr, n_cols + 1)))
        return rc;
      int end_bit = 1;
      while (end_bit < 32 && (1ll << end_bit) < n_cols) ++end_bit;
      rc = cub_call(stream, [&](void* t, size_t& b) {
        return hipcub::DeviceRadixSort::SortPairs(t, b, indices, keys_out, values, vals_out, (int)nnz, 0, end_bit,
                                                  stream);
      });
      if (rc) return rc;
      WG_HIP_TRY(hipMemsetAsync(colptr, 0, sizeof(int32_t) * (n_cols + 1), stream));
      hipLaunchKernelGGL(col_count_kernel, dim3(ceil_div(nnz, 256)), dim3(256), 0, stream, nnz, indices, colptr + 1);
      WG_LAUNCH_CHECK();
      rc = cub_call(stream, [&](void* t, size_t& b) {
        return hipcub::DeviceScan::InclusiveSum(t, b, colptr + 1, colptr + 1, (int)n_cols, stream);
      });
      if (rc) return rc;
      hipLaunchKernelGGL(col_seq_sum_kernel, dim3(nb_cols), dim3(256), 0, stream, n_cols, colptr, vals_out, colsum32);
      WG_LAUNCH_CHECK();
    }
  }
  if (n_cols > 0) {
    hipLaunchKernelGGL(degree_kernel, dim3(nb_cols), dim3(256), 0, stream, n_cols, n_rows, colsum32, diag, w_cols, sw,
                       iso_col);
    WG_LAUNCH_CHECK();
    if (raw) WG_HIP_TRY(hipMemsetAsync(iso_col, 0, n_cols, stream));  // no diagonal term
  }
  if (n_rows == 0) {
    WG_HIP_TRY(hipMemsetAsync(L->rowptr, 0, sizeof(int32_t), stream));
    WG_HIP_TRY(hipStreamSynchronize(stream));
    return WG_OK;
  }
  L->n_active = n_rows;
  // relabelling by descending off-diagonal length (stable: ties keep caller order)
  hipLaunchKernelGGL(iota_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, ids);
  WG_LAUNCH_CHECK();
  if (L->reordered) {
    // closed-form rows: purely isolated rows (w_i == 0, no entries in row or column i).  On a row
    // shard w is the GLOBAL column degree (w_cols, wats_hip.dist's all-reduce): on an unweighted
    // graph w_i == 0 means no shard's row has an entry in column i, so such an own row is never
    // a halo row elsewhere and can be finished in closed form too; with
    // values a zero sum need not mean no entries, so weighted shards keep every row
    const int allow_closed = (!raw && (w_cols == nullptr || values == nullptr)) ? 1 : 0;
    hipLaunchKernelGGL(sort_key_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, len, colcnt, iso_col, allow_closed,
                       key);
    WG_LAUNCH_CHECK();
    rc = cub_call(stream, [&](void* t, size_t& b) {
      return hipcub::DeviceRadixSort::SortPairsDescending(t, b, key, key_sorted, ids, L->perm, (int)n_rows, 0, 33,
                                                          stream);
    });
    if (rc) return rc;
    WG_HIP_TRY(hipMemsetAsync(npure_d, 0, sizeof(unsigned int), stream));
    hipLaunchKernelGGL(count_pure_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, key, npure_d);
    WG_LAUNCH_CHECK();
    unsigned int npure = 0;
    WG_HIP_TRY(hipMemcpyAsync(&npure, npure_d, sizeof(unsigned int), hipMemcpyDeviceToHost, stream));
    WG_HIP_TRY(hipStreamSynchronize(stream));
    L->n_active = n_rows - (int64_t)npure;
  } else {
    WG_HIP_TRY(hipMemcpyAsync(L->perm, ids, sizeof(int32_t) * n_rows, hipMemcpyDeviceToDevice, stream));
  }
  hipLaunchKernelGGL(invert_perm_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, L->perm, L->iperm);
  WG_LAUNCH_CHECK();
  hipLaunchKernelGGL(dinv_kernel, dim3(nb_cols), dim3(256), 0, stream, n_cols, n_rows, L->perm, sw, L->dinv);
  WG_LAUNCH_CHECK();
  hipLaunchKernelGGL(gather_len_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, L->perm, len, len_sorted, iso_col,
                     L->iso);
  WG_LAUNCH_CHECK();
  WG_HIP_TRY(hipMemsetAsync(L->rowptr, 0, sizeof(int32_t), stream));
  rc = cub_call(stream, [&](void* t, size_t& b) {
    return hipcub::DeviceScan::InclusiveSum(t, b, len_sorted, L->rowptr + 1, (int)n_rows, stream);
  });
  if (rc) return rc;
  int32_t total = 0;
  WG_HIP_TRY(hipMemcpyAsync(&total, L->rowptr + n_rows, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
  WG_HIP_TRY(hipStreamSynchronize(stream));
  L->nnz = total;
  // +4 padding: the F == 1 vectorised index loads read whole aligned 4-groups
  if ((rc = dmalloc(&L->col, L->nnz + 4)) || (rc = dmalloc(&L->val, L->nnz + 4))) return rc;
  WG_HIP_TRY(hipMemsetAsync(L->col + L->nnz, 0, 4 * sizeof(int32_t), stream));
  WG_HIP_TRY(hipMemsetAsync(L->val + L->nnz, 0, 4 * sizeof(float), stream));
  hipLaunchKernelGGL(fill_lhat_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, stream, n_rows, L->perm, L->iperm,
                     indptr, indices, values, sw, L->rowptr, L->col, L->val, raw ? 1 : 0);
  WG_LAUNCH_CHECK();
  WG_HIP_TRY(hipMemsetAsync(hist, 0, sizeof(unsigned int) * kBuckets, stream));
  hipLaunchKernelGGL(bucket_hist_kernel, dim3(std::min<int64_t>(nb_rows, 1024)), dim3(256), 0, stream, n_rows,
                     len_sorted, hist);
  WG_LAUNCH_CHECK();
  WG_HIP_TRY(hipMemcpyAsync(L->bucket, hist, sizeof(unsigned int) * kBuckets, hipMemcpyDeviceToHost, stream));
  hipLaunchKernelGGL(f64_to_f32_kernel, dim3(nb_rows), dim3(256), 0, stream, n_rows, rowsum64, L->rowsum);
  WG_LAUNCH_CHECK();
  std::vector<uint8_t> isoh(n_rows);
  WG_HIP_TRY(hipMemcpyAsync(isoh.data(), L->iso, n_rows, hipMemcpyDeviceToHost, stream));
  int32_t max_len = 0;
  if (L->reordered) {
    WG_HIP_TRY(hipMemcpyAsync(&max_len, len_sorted, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    WG_HIP_TRY(hipStreamSynchronize(stream));
  } else {
    std::vector<int32_t> lh(n_rows);
    WG_HIP_TRY(hipMemcpyAsync(lh.data(), len_sorted, sizeof(int32_t) * n_rows, hipMemcpyDeviceToHost, stream));
    WG_HIP_TRY(hipStreamSynchronize(stream));
    max_len = *std::max_element(lh.begin(), lh.end());
  }
  int32_t nonunit = 0;
  WG_HIP_TRY(hipMemcpy(&nonunit, nonunit_d, sizeof(int32_t), hipMemcpyDeviceToHost));
  L->unit = (nonunit == 0) && !raw;
  int64_t niso = 0;
  for (auto v : isoh) niso += v;
  L->n_iso = niso;
  L->max_row = max_len;
  L->avg_len = L->nnz / n_rows;
  L->n_closed = n_rows - L->n_active;
  return WG_OK;
}

}  // namespace wg

namespace wg {
// Each row's entries in ascending internal column id (values follow): rows of
// a power-law graph then start with their hub columns, so neighbouring lanes
// and iterations of the step kernel share cache lines.  Synchronous.
int sort_row_columns(wg_laplacian_s* L, hipStream_t stream) {
  const int64_t n = L->n_rows, nnz = L->nnz;
  if (n == 0 || nnz == 0 || L->cols_sorted) {
    L->cols_sorted = true;
    return WG_OK;
  }
  int32_t* col2 = nullptr;
  float* val2 = nullptr;
  int rc = 0;
  if ((rc = dmalloc(&col2, nnz + 4)) || (rc = dmalloc(&val2, nnz + 4))) {
    (void)hipFree(col2);
    return rc;
  }
  WG_HIP_TRY(hipMemsetAsync(col2 + nnz, 0, 4 * sizeof(int32_t), stream));
  WG_HIP_TRY(hipMemsetAsync(val2 + nnz, 0, 4 * sizeof(float), stream));
  int end_bit = 1;
  while (end_bit < 32 && (1ll << end_bit) < L->n_cols) ++end_bit;
  rc = cub_call(stream, [&](void* t, size_t& b) {
    return hipcub::DeviceSegmentedRadixSort::SortPairs(t, b, L->col, col2, L->val, val2, (int)nnz, (int)n, L->rowptr,
                                                       L->rowptr + 1, 0, end_bit, stream);
  });
  if (rc) {
    (void)hipFree(col2);
    (void)hipFree(val2);
    return rc;
  }
  (void)hipFree(L->col);
  (void)hipFree(L->val);
  L->col = col2;
  L->val = val2;
  L->cols_sorted = true;
  return WG_OK;
}
}  // namespace wg

using namespace wg;

wg_laplacian_s::~wg_laplacian_s() {
  chain.release();
  wg::release_chain1(this);
  for (hipEvent_t e : ev) (void)hipEventDestroy(e);
  for (auto& kv : plans) kv.second.release();
  wg::release_lds1(this);
  for (void* p : {(void*)rowptr, (void*)col, (void*)val, (void*)iso, (void*)perm, (void*)iperm, (void*)rowsum,
                  (void*)ws, (void*)dinv, (void*)prp, (void*)pcol, (void*)trace_buf, (void*)tsum})
    (void)hipFree(p);
  if (side_fork) (void)hipEventDestroy(side_fork);
  if (side_join) (void)hipEventDestroy(side_join);
  if (side) (void)hipStreamDestroy(side);
}

extern "C" {

int wg_dense_to_csr_count(const float* adj, int64_t n_rows, int64_t n_cols, int64_t ld, int64_t* indptr,
                          int64_t* nnz_host, void* stream_) {
  if (n_rows < 0 || n_cols < 0 || ld < n_cols || !indptr || !nnz_host || (n_rows > 0 && n_cols > 0 && !adj))
    return fail(WG_ERR_INVALID, "wg_dense_to_csr_count: bad arguments");
  if (n_cols > INT32_MAX) return fail(WG_ERR_INVALID, "wg_dense_to_csr_count: n_cols exceeds int32");
  hipStream_t stream = as_stream(stream_);
  WG_HIP_TRY(hipMemsetAsync(indptr, 0, sizeof(int64_t), stream));
  if (n_rows > 0) {
    hipLaunchKernelGGL(dense_count_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, stream, n_rows, n_cols, ld, adj,
                       indptr + 1);
    WG_LAUNCH_CHECK();
    int rc = cub_call(stream, [&](void* tmp, size_t& bytes) {
      return hipcub::DeviceScan::InclusiveSum(tmp, bytes, indptr + 1, indptr + 1, (int)n_rows, stream);
    });
    if (rc) return rc;
  }
  WG_HIP_TRY(hipMemcpyAsync(nnz_host, indptr + n_rows, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
  WG_HIP_TRY(hipStreamSynchronize(stream));
  return WG_OK;
}

int wg_dense_to_csr_fill(const float* adj, int64_t n_rows, int64_t n_cols, int64_t ld, const int64_t* indptr,
                         int32_t* indices, float* values, void* stream_) {
  if (n_rows < 0 || n_cols < 0 || ld < n_cols || !indptr) return fail(WG_ERR_INVALID, "wg_dense_to_csr_fill: bad arguments");
  if (n_rows == 0 || n_cols == 0) return WG_OK;
  hipLaunchKernelGGL(dense_fill_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, as_stream(stream_), n_rows, n_cols,
                     ld, adj, indptr, indices, values);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int wg_column_degree(int64_t n_rows, int64_t row_offset, const int64_t* indptr, const int32_t* indices,
                     const float* values, double* colsum_f64, double* diag_f64, void* stream_) {
  if (n_rows < 0 || !indptr || !colsum_f64 || !diag_f64) return fail(WG_ERR_INVALID, "wg_column_degree: bad arguments");
  if (n_rows == 0) return WG_OK;
  hipLaunchKernelGGL(column_degree_kernel, dim3(ceil_div(n_rows, 4)), dim3(kBlock), 0, as_stream(stream_), n_rows,
                     row_offset, indptr, indices, values, colsum_f64, diag_f64);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

int wg_laplacian_create(int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t* indptr, const int32_t* indices,
                        const float* values, const float* w_cols, uint32_t flags, void* stream_, wg_laplacian_t* out) {
  if (!out) return fail(WG_ERR_INVALID, "wg_laplacian_create: out is NULL");
  *out = nullptr;
  if (n_rows < 0 || n_cols < n_rows || nnz < 0 || !indptr || (nnz > 0 && !indices))
    return fail(WG_ERR_INVALID, "wg_laplacian_create: bad shape (n_rows=%lld n_cols=%lld nnz=%lld)", (long long)n_rows,
                (long long)n_cols, (long long)nnz);
  if (nnz > INT32_MAX || n_cols > INT32_MAX)
    return fail(WG_ERR_UNSUPPORTED, "wg_laplacian_create: nnz/n_cols exceed int32 (shard the graph)");
  if (n_cols > n_rows && !w_cols) return fail(WG_ERR_INVALID, "wg_laplacian_create: halo columns need w_cols");
  auto* L = new wg_laplacian_s();
  if (hipGetDevice(&L->device) != hipSuccess) {
    delete L;
    return fail(WG_ERR_HIP, "wg_laplacian_create: no HIP device");
  }
  L->n_rows = n_rows;
  L->n_cols = n_cols;
  L->nnz_input = nnz;
  L->reordered = !(flags & WG_FLAG_NO_REORDER);
  L->values_null = (values == nullptr);
  int rc = build_operator(L, indptr, indices, values, w_cols, /*raw=*/false, as_stream(stream_));
  if (rc == WG_OK && !(flags & WG_FLAG_KEEP_COLUMN_ORDER)) rc = sort_row_columns(L, as_stream(stream_));
  if (rc != WG_OK) {
    (void)hipStreamSynchronize(as_stream(stream_));
    delete L;
    return rc;
  }
  *out = L;
  return WG_OK;
}

// A literal operator (every stored entry kept with its value, diagonal included,
// nothing normalised): what chebyshev_polynomials(L, k, X0) applies when the
// caller hands it an explicit matrix (reference calibration/WATS.py:29-37 is
// called with L_rescaled, a float64 scipy CSR, at WATS.py:62).
int wg_operator_create(int64_t n, int64_t nnz, const int64_t* indptr, const int32_t* indices, const float* values,
                       uint32_t flags, void* stream_, wg_laplacian_t* out) {
  if (!out) return fail(WG_ERR_INVALID, "wg_operator_create: out is NULL");
  *out = nullptr;
  if (n < 0 || nnz < 0 || !indptr || (nnz > 0 && (!indices || !values)))
    return fail(WG_ERR_INVALID, "wg_operator_create: bad shape (n=%lld nnz=%lld)", (long long)n, (long long)nnz);
  if (nnz > INT32_MAX || n > INT32_MAX) return fail(WG_ERR_UNSUPPORTED, "wg_operator_create: nnz/n exceed int32");
  auto* L = new wg_laplacian_s();
  if (hipGetDevice(&L->device) != hipSuccess) {
    delete L;
    return fail(WG_ERR_HIP, "wg_operator_create: no HIP device");
  }
  L->n_rows = n;
  L->n_cols = n;
  L->nnz_input = nnz;
  L->reordered = !(flags & WG_FLAG_NO_REORDER);
  int rc = build_operator(L, indptr, indices, values, nullptr, /*raw=*/true, as_stream(stream_));
  if (rc == WG_OK && !(flags & WG_FLAG_KEEP_COLUMN_ORDER)) rc = sort_row_columns(L, as_stream(stream_));
  if (rc == WG_OK && hipStreamSynchronize(as_stream(stream_)) != hipSuccess)
    rc = fail(WG_ERR_HIP, "wg_operator_create: sync");
  if (rc != WG_OK) {
    (void)hipStreamSynchronize(as_stream(stream_));
    delete L;
    return rc;
  }
  *out = L;
  return WG_OK;
}

int wg_laplacian_destroy(wg_laplacian_t L) {
  if (!L) return WG_OK;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(L->device);
  (void)hipDeviceSynchronize();
  delete L;
  (void)hipSetDevice(cur);
  return WG_OK;
}

int wg_laplacian_export(wg_laplacian_t L, int64_t* indptr, int32_t* indices, float* values, uint8_t* iso,
                        void* stream_) {
  if (!L || !indptr) return fail(WG_ERR_INVALID, "wg_laplacian_export: NULL argument");
  hipStream_t stream = as_stream(stream_);
  const int64_t n = L->n_rows;
  WG_HIP_TRY(hipMemsetAsync(indptr, 0, sizeof(int64_t), stream));
  if (n == 0) return WG_OK;
  hipLaunchKernelGGL(export_len_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, n, L->iperm, L->rowptr,
                     indptr + 1);
  WG_LAUNCH_CHECK();
  int rc = cub_call(stream, [&](void* tmp, size_t& bytes) {
    return hipcub::DeviceScan::InclusiveSum(tmp, bytes, indptr + 1, indptr + 1, (int)n, stream);
  });
  if (rc) return rc;
  hipLaunchKernelGGL(export_fill_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, n, L->perm, L->iperm, L->rowptr,
                     L->col, L->val, indptr, indices, values);
  WG_LAUNCH_CHECK();
  if (L->cols_sorted && L->nnz > 0) {
    // rows were sorted by internal column: back to ascending caller column
    int32_t* idx2 = nullptr;
    float* val2 = nullptr;
    if ((rc = dmalloc(&idx2, L->nnz)) || (rc = dmalloc(&val2, L->nnz))) {
      (void)hipFree(idx2);
      return rc;
    }
    int end_bit = 1;
    while (end_bit < 32 && (1ll << end_bit) < L->n_cols) ++end_bit;
    rc = cub_call(stream, [&](void* t, size_t& b) {
      return hipcub::DeviceSegmentedRadixSort::SortPairs(t, b, indices, idx2, values, val2, (int)L->nnz, (int)n,
                                                         indptr, indptr + 1, 0, end_bit, stream);
    });
    if (!rc) {
      (void)hipMemcpyAsync(indices, idx2, sizeof(int32_t) * L->nnz, hipMemcpyDeviceToDevice, stream);
      (void)hipMemcpyAsync(values, val2, sizeof(float) * L->nnz, hipMemcpyDeviceToDevice, stream);
      rc = hipStreamSynchronize(stream) == hipSuccess ? WG_OK : fail(WG_ERR_HIP, "export: sync");
    }
    (void)hipFree(idx2);
    (void)hipFree(val2);
    if (rc) return rc;
  }
  if (iso) {
    hipLaunchKernelGGL(export_iso_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, n, L->iperm, L->iso, iso);
    WG_LAUNCH_CHECK();
  }
  return WG_OK;
}

int wg_log1p_degree(wg_laplacian_t L, float* x0, void* stream_) {
  if (!L || (!x0 && L->n_rows)) return fail(WG_ERR_INVALID, "wg_log1p_degree: NULL argument");
  if (L->n_rows == 0) return WG_OK;
  hipLaunchKernelGGL(log1p_degree_kernel, dim3(ceil_div(L->n_rows, 256)), dim3(256), 0, as_stream(stream_), L->n_rows,
                     L->rowsum, x0);
  WG_LAUNCH_CHECK();
  return WG_OK;
}

}  // extern "C"
