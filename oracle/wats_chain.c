/*
 * wats_chain.c -- CPU oracle, TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference graph-wavelet path
 * (CaptainCuong/Efficient-GNN calibration/WATS.py:24-74) for the full-size
 * parity checks (Reddit-size, 8M R-MAT), where the numpy/scipy restatement
 * (oracle/wats_oracle.py) takes minutes.  Only tests/, __graft_entry__.smoke()
 * and bench.py's checks load it (through oracle/wats_oracle_c.py), as the
 * checker; the product path (efficient-gnn_amd/wats_hip) never does.
 *
 * Same arithmetic, same order as the reference's scipy calls:
 *   - w = colsum(A) - diag(A): scipy _laplacian.py:467 sums a float32 CSR's
 *     columns as a CSC mat-vec, i.e. sequentially per column in ascending row
 *     order, in float32; then the float32 subtraction;
 *   - iso = (w == 0), sw = iso ? 1 : sqrtf(w)              (_laplacian.py:470-471);
 *   - L_hat_ij = -((a_ij / sw_i) / sw_j) in float32, i != j  (:472-474);
 *     L_hat_ii = -iso_i  (setdiag(1 - iso) at :475, then "- identity(N)" at
 *     WATS.py:55); entries in ascending column order (scipy's canonical CSR
 *     after the subtraction), upcast to float64;
 *   - T_0 = X0, T_1 = L_hat X0, T_i = 2 L_hat T_{i-1} - T_{i-2} (WATS.py:29-37):
 *     each row's sum sequential over its entries in float64 (sparsetools
 *     csr_matvec(s)); (2 L_hat) x equals 2 (L_hat x) exactly;
 *   - S = sum_i alpha_i T_i, left to right from 0 (alpha_i = np.exp(-s i), WATS.py:65-68);
 *   - H = S / (sum_f |S_if| + 1e-8)                            (WATS.py:71-72).
 * Rows are independent, so the OpenMP row loop gives the same bits for any
 * thread count.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no FMA
 * contraction, like scipy's baseline x86-64 wheels).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Off-diagonal L_hat in ascending column order per row (+ the iso flags).
 * Returns 0, or -1 on allocation failure.  *out_* are malloc'ed. */
static int rescaled_laplacian(int64_t n, const int64_t* indptr, const int32_t* indices, const float* values,
                              int64_t** out_ptr, int32_t** out_col, double** out_val, uint8_t** out_iso) {
  float* colsum = (float*)calloc((size_t)(n > 0 ? n : 1), sizeof(float));
  float* diag = (float*)calloc((size_t)(n > 0 ? n : 1), sizeof(float));
  float* sw = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
  uint8_t* iso = (uint8_t*)malloc((size_t)(n > 0 ? n : 1));
  int64_t* ptr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
  if (!colsum || !diag || !sw || !iso || !ptr) return -1;
  /* sequential float32 column sums in ascending row order; duplicates summed as stored */
  for (int64_t i = 0; i < n; ++i)
    for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) {
      const float a = values ? values[e] : 1.0f;
      colsum[indices[e]] += a;
      if (indices[e] == i) diag[i] += a;
    }
  for (int64_t j = 0; j < n; ++j) {
    const float w = colsum[j] - diag[j];
    iso[j] = (w == 0.0f);
    sw[j] = iso[j] ? 1.0f : sqrtf(w);
  }
  free(colsum);
  free(diag);
  /* count off-diagonal entries per row (duplicates of a column are summed first, as
   * scipy's canonical format does; the inputs here are canonical CSR) */
  ptr[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t c = 0;
    for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) c += (indices[e] != i);
    ptr[i + 1] = ptr[i] + c;
  }
  int32_t* col = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ptr[n] > 0 ? ptr[n] : 1));
  double* val = (double*)malloc(sizeof(double) * (size_t)(ptr[n] > 0 ? ptr[n] : 1));
  if (!col || !val) return -1;
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t i = 0; i < n; ++i) {
    int64_t o = ptr[i];
    for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) {
      const int32_t j = indices[e];
      if (j == i) continue;
      const float a = values ? values[e] : 1.0f;
      const float v = -((a / sw[i]) / sw[j]);
      col[o] = j;
      val[o] = (double)v;
      ++o;
    }
    /* ascending column order (input rows are canonical; keep a stable insertion sort for safety) */
    for (int64_t p = ptr[i] + 1; p < ptr[i + 1]; ++p) {
      const int32_t cj = col[p];
      const double cv = val[p];
      int64_t q = p - 1;
      while (q >= ptr[i] && col[q] > cj) {
        col[q + 1] = col[q];
        val[q + 1] = val[q];
        --q;
      }
      col[q + 1] = cj;
      val[q + 1] = cv;
    }
  }
  free(sw);
  *out_ptr = ptr;
  *out_col = col;
  *out_val = val;
  *out_iso = iso;
  return 0;
}

/* y = L_hat x (+ the isolated diagonal), row i's sum in ascending column order with the
 * diagonal term at its column position, float64; scale 2 for k >= 2; minus xm2. */
static void cheb_apply(int64_t n, int64_t F, const int64_t* ptr, const int32_t* col, const double* val,
                       const uint8_t* iso, const double* x, const double* xm2, double* y) {
#pragma omp parallel
  {
    double* acc = (double*)malloc(sizeof(double) * (size_t)F);
#pragma omp for schedule(dynamic, 256)
    for (int64_t i = 0; i < n; ++i) {
      for (int64_t f = 0; f < F; ++f) acc[f] = 0.0;
      int diag_done = !iso[i];
      for (int64_t e = ptr[i]; e < ptr[i + 1]; ++e) {
        const int32_t j = col[e];
        if (!diag_done && j > i) {
          for (int64_t f = 0; f < F; ++f) acc[f] += -1.0 * x[i * F + f];
          diag_done = 1;
        }
        const double v = val[e];
        for (int64_t f = 0; f < F; ++f) acc[f] += v * x[(int64_t)j * F + f];
      }
      if (!diag_done)
        for (int64_t f = 0; f < F; ++f) acc[f] += -1.0 * x[i * F + f];
      for (int64_t f = 0; f < F; ++f) y[i * F + f] = xm2 ? (2.0 * acc[f]) - xm2[i * F + f] : acc[f];
    }
    free(acc);
  }
}

/* graph_wavelet_features for an F-column float32 signal X0 (n x F, row-major):
 * S (n x F float64) and optionally H.  K >= 0; alpha[0..K] = the heat
 * coefficients exp(-s i) as the caller's numpy computes them (WATS.py:65:
 * np.exp, whose last bit may differ from libm's).  threads <= 0: OpenMP
 * default.  Returns 0 or -1 (allocation). */
int wo_wavelet_features(int64_t n, const int64_t* indptr, const int32_t* indices, const float* values,
                        const float* X0, int64_t F, int32_t K, const double* alpha, double* S, double* H,
                        int32_t threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
  int64_t* ptr = NULL;
  int32_t* col = NULL;
  double* val = NULL;
  uint8_t* iso = NULL;
  if (rescaled_laplacian(n, indptr, indices, values, &ptr, &col, &val, &iso)) return -1;
  const size_t m = (size_t)(n * F > 0 ? n * F : 1);
  double* b[3];
  for (int q = 0; q < 3; ++q) b[q] = (double*)malloc(sizeof(double) * m);
  if (!b[0] || !b[1] || !b[2]) return -1;
  /* S = 0 + alpha_0 T_0 (T_0 = X0 upcast) */
  for (size_t i = 0; i < (size_t)(n * F); ++i) {
    b[0][i] = (double)X0[i];
    S[i] = alpha[0] * b[0][i];
  }
  double *tm2 = NULL, *tm1 = b[0];
  for (int32_t k = 1; k <= K; ++k) {
    double* out = (tm1 == b[0]) ? b[1] : (tm1 == b[1] ? b[2] : b[0]);
    if (out == tm2) out = (b[0] != tm1 && b[0] != tm2) ? b[0] : (b[1] != tm1 && b[1] != tm2) ? b[1] : b[2];
    cheb_apply(n, F, ptr, col, val, iso, tm1, k >= 2 ? tm2 : NULL, out);
    const double a = alpha[k];
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n * F; ++i) S[i] = S[i] + a * out[i];
    tm2 = tm1;
    tm1 = out;
  }
  if (H) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      double t = 0.0;
      for (int64_t f = 0; f < F; ++f) t += fabs(S[i * F + f]);
      const double den = t + 1e-8;
      for (int64_t f = 0; f < F; ++f) H[i * F + f] = S[i * F + f] / den;
    }
  }
  for (int q = 0; q < 3; ++q) free(b[q]);
  free(ptr);
  free(col);
  free(val);
  free(iso);
  return 0;
}

int wo_abi_version(void) { return 1; }
