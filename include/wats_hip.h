/*
 * wats_hip.h -- C ABI of the MI355X (gfx950) graph-wavelet feature extractor.
 *
 * Drop-in boundary for the hot path of CaptainCuong/Efficient-GNN
 * `calibration/WATS.py` (the reference is pure Python over scipy.sparse; this
 * header lists the entry points a ctypes / cffi binding of that path binds).
 * Each entry cites the reference function it replaces.
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer (hipMalloc / torch CUDA tensor
 *     storage) unless its name ends in `_host`.  Buffers are caller-owned,
 *     row-major, contiguous, F (signal columns) innermost.
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *     All work is enqueued on it; no entry point synchronises the device
 *     except the ones documented as "synchronous" (graph creation / dense
 *     ingestion, which size device allocations from device-computed counts).
 *   - Return value: WG_OK (0) or a negative WG_ERR_* code; the message of the
 *     last failure on the calling host thread is wg_last_error().  No entry
 *     point aborts the process.
 *   - A wg_laplacian_t is not thread-safe: one host thread per handle.
 *     Multi-GPU = one process per GPU, one handle per process (row shard).
 */
#ifndef WATS_HIP_H
#define WATS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WG_ABI_VERSION 1

enum wg_status {
  WG_OK = 0,
  WG_ERR_INVALID = -1,   /* bad argument (shape, null pointer, range) */
  WG_ERR_HIP = -2,       /* a HIP runtime call failed */
  WG_ERR_OOM = -3,       /* device allocation failed */
  WG_ERR_UNSUPPORTED = -4,
  WG_ERR_TIMEOUT = -5    /* an in-kernel wait gave up (the one-launch chain): that launch's outputs are NaN */
};

/* creation flags */
#define WG_FLAG_NONE 0u
#define WG_FLAG_NO_REORDER 1u   /* keep the caller's row order (no degree relabelling) */
#define WG_FLAG_TRANSPOSE 2u    /* wg_rownorm_create: build adj_norm^T instead of adj_norm */
#define WG_FLAG_KEEP_COLUMN_ORDER 4u /* keep each row's input entry order (default: ascending
                                        internal column, which shares cache lines between
                                        neighbouring gathers on power-law graphs) */

typedef struct wg_laplacian_s* wg_laplacian_t;

typedef struct wg_laplacian_info {
  int64_t n_rows;        /* rows owned by this handle (all N on one GPU) */
  int64_t n_cols;        /* column space = n_rows + halo rows (== n_rows on one GPU) */
  int64_t nnz_input;     /* stored entries of the input adjacency rows */
  int64_t nnz;           /* off-diagonal entries of L_hat (self loops removed) */
  int64_t n_isolated;    /* rows with w_i == 0 (L_hat_ii = -1) */
  int64_t max_row_nnz;   /* longest L_hat row */
  int32_t n_segments;    /* row-length bins of the step kernel */
  int32_t reordered;     /* 1 if rows are relabelled by descending degree */
  int64_t n_closed_form; /* purely isolated rows (w_i = 0, empty row and column):
                            T_k = (-1)^k X0 exactly, kept out of the step kernel
                            by wg_wavelet_features */
} wg_laplacian_info;

/* -------------------------------------------------------------------------
 * Library
 * ---------------------------------------------------------------------- */
const char* wg_last_error(void);
int wg_abi_version(void);

/* -------------------------------------------------------------------------
 * a8 / section 8(f)-1: dense adjacency ingestion.
 * Replaces `csr_matrix(adj.cpu().numpy())` (calibration/WATS.py:99) with an
 * on-device compaction.  Two calls: count (writes indptr[n+1], returns nnz in
 * *nnz_host; synchronous), then fill (indices/values sized nnz; async).
 * Entries != 0.0f are kept, in column order, exactly like scipy.
 * ---------------------------------------------------------------------- */
int wg_dense_to_csr_count(const float* adj, int64_t n_rows, int64_t n_cols, int64_t ld,
                          int64_t* indptr, int64_t* nnz_host, void* stream);
int wg_dense_to_csr_fill(const float* adj, int64_t n_rows, int64_t n_cols, int64_t ld,
                         const int64_t* indptr, int32_t* indices, float* values, void* stream);

/* -------------------------------------------------------------------------
 * Degree helpers (used for row shards, where the Laplacian's column degree
 * w_j = colsum_j(A) - A_jj spans every shard and is summed across ranks).
 * wg_column_degree ACCUMULATES (+=) this shard's column sums into
 * colsum_f64[n_cols_global] and its diagonal into diag_f64 (indexed by the
 * global column id `row_offset + i` of local row i).  Column ids are global.
 * scipy semantics: `_laplacian.py:467` (w = m.sum(axis=0) - m.diagonal()).
 * ---------------------------------------------------------------------- */
int wg_column_degree(int64_t n_rows, int64_t row_offset, const int64_t* indptr,
                     const int32_t* indices, const float* values /* NULL = 1 */,
                     double* colsum_f64, double* diag_f64, void* stream);

/* -------------------------------------------------------------------------
 * a1 + a2: compute_normalized_laplacian + rescale.
 * Replaces `csgraph.laplacian(adj, normed=True)` (calibration/WATS.py:24-27,
 * scipy _laplacian.py:467-475) followed by `(2/2.0)*L - identity(N)`
 * (calibration/WATS.py:55).  Builds on the device:
 *     L_hat_ij = -((a_ij / sqrt(w_i)) / sqrt(w_j))   (float32, scipy op order)
 *     for i != j, with w = column sums minus diagonal and sqrt(w)=1 where w==0;
 *     L_hat_ii = -1 for isolated rows (w_i == 0), 0 (dropped) otherwise.
 * Inputs: CSR rows of A (int64 indptr[n_rows+1], int32 indices, float32
 * values or NULL for an unweighted graph); column ids in [0, n_cols) where
 * column i (< n_rows) is local row i (i.e. owned rows first, then halo rows).
 * w_cols (float32[n_cols], nullable): precomputed column degree
 * (colsum - diag) per column id; NULL = compute from this CSR (single GPU).
 * Synchronous.  The handle owns its device copy of L_hat and workspaces.
 * ---------------------------------------------------------------------- */
int wg_laplacian_create(int64_t n_rows, int64_t n_cols, int64_t nnz,
                        const int64_t* indptr, const int32_t* indices, const float* values,
                        const float* w_cols, uint32_t flags, void* stream,
                        wg_laplacian_t* out);
int wg_laplacian_destroy(wg_laplacian_t L);
int wg_laplacian_get_info(wg_laplacian_t L, wg_laplacian_info* info_host);

/* Export L_hat in the CALLER's row/column numbering: the off-diagonal
 * entries as CSR (int64 indptr[n_rows+1], int32 indices / float32 values
 * sized info.nnz; each row in ascending column order, or in the input's
 * order under WG_FLAG_KEEP_COLUMN_ORDER) plus iso[n_rows] (1 where
 * L_hat_ii = -1; nullable).  For bit-exact parity tests against scipy.  Async. */
int wg_laplacian_export(wg_laplacian_t L, int64_t* indptr, int32_t* indices,
                        float* values, uint8_t* iso, void* stream);

/* A literal CSR operator for chebyshev_polynomials(L, k, X0)
 * (calibration/WATS.py:29-37) called with an explicit matrix -- the reference
 * passes `L_rescaled = (2/2.0)*L - identity(N)`, a float64 scipy CSR
 * (WATS.py:55,62).  Every stored entry is kept with its value (float32),
 * diagonal entries included; nothing is normalised and no row is isolated.
 * Square n x n; the handle is a wg_laplacian_t of the same step kernel
 * (wg_cheb_step / wg_permute_rows; freed by wg_laplacian_destroy).
 * Synchronous. */
int wg_operator_create(int64_t n, int64_t nnz, const int64_t* indptr, const int32_t* indices,
                       const float* values, uint32_t flags, void* stream, wg_laplacian_t* out);

/* -------------------------------------------------------------------------
 * a3: input signal.  Replaces `X0 = log1p(adj.sum(axis=1))`
 * (calibration/WATS.py:58-59): row sums INCLUDING self loops, float32 (N,1),
 * in the caller's row order.
 * ---------------------------------------------------------------------- */
int wg_log1p_degree(wg_laplacian_t L, float* x0, void* stream);

/* -------------------------------------------------------------------------
 * a4 (+a5): one Chebyshev step of `chebyshev_polynomials`
 * (calibration/WATS.py:29-37), in the handle's INTERNAL row order (see
 * wg_permute_rows).  k == 1:  T_1 = L_hat T_0;  k >= 2:  T_k = 2 L_hat T_{k-1}
 * - T_{k-2}.  t_km1 has n_cols rows (owned + halo), t_km2 / t_k n_rows rows,
 * all with row stride F.  t_k may alias t_km2 (in-place).  If S != NULL the
 * heat-kernel sum of calibration/WATS.py:65-68 is fused:
 *   k == 1:  S = alpha0 * T_0 + alpha_k * T_1;    k >= 2:  S += alpha_k * T_k.
 * If H != NULL (last step) the row-L1 normalisation of WATS.py:71-72 is fused:
 *   H = S / (sum_f |S| + 1e-8).  Row sums accumulate in float64.
 * ---------------------------------------------------------------------- */
int wg_cheb_step(wg_laplacian_t L, int32_t k, int64_t F, const float* t_km1,
                 const float* t_km2, float* t_k, float* S, float* H,
                 double alpha0, double alpha_k, void* stream);

/* F == 1 on an unweighted graph: the column-blocked LDS step kernel
 * (csrc/lds1.hip) gathers u_{k-1} = T_{k-1} * dinv instead of T_{k-1}
 * (dinv_j = 1 / sqrt(w_j), w_j = 0 -> 1), so a row-sharded caller exchanges
 * halo rows of u.  Same recurrence as wg_cheb_step (calibration/WATS.py:32-36,
 * heat sum WATS.py:65-68), internal row order.
 * wg_cheb_u_len: *len = floats a u buffer must hold (n_cols rounded up to whole
 *   column blocks; entries past n_cols are never used), or 0 when this kernel
 *   does not apply (weighted graph, too many column blocks, "lds" tuned off).
 *   Builds the plan (synchronous, once).
 * wg_scale_dinv: u[i] = x[i] * dinv[i] for the handle's own rows i < n_rows.
 * wg_cheb_step_u: u_km1 has wg_cheb_u_len floats (own rows then halo rows,
 *   as t_km1 of wg_cheb_step); t_km1 / t_km2 / t_k are own rows only; u_k
 *   (nullable) receives u_k for the own rows.  WG_ERR_UNSUPPORTED when
 *   wg_cheb_u_len is 0. */
int wg_cheb_u_len(wg_laplacian_t L, int64_t* len_host);
/* Shape of the LDS kernel's plan (for byte accounting), or all zeros when it
 * does not apply: out[0] mode (1 row teams, 2 chunk windows), [1] column
 * blocks, [2] rows, [3] columns, [4] nonzeros, [5] non-empty (row, block)
 * segments, [6] 16-B chunks (padded ids), [7] workgroups.  active_only = 1:
 * the plan wg_wavelet_features uses (rows that enter the chain). */
int wg_lds_plan_info(wg_laplacian_t L, int32_t active_only, int64_t* out8_host);
int wg_scale_dinv(wg_laplacian_t L, const float* x, float* u, void* stream);
int wg_cheb_step_u(wg_laplacian_t L, int32_t k, const float* u_km1, const float* t_km1,
                   const float* t_km2, float* t_k, float* u_k, float* S, double alpha0,
                   double alpha_k, void* stream);

/* One step of the heat sum by Clenshaw's recurrence (WATS.py:32-36 with the
 * sum of :65-68), the step wg_wavelet_features (F > 1) and the row-sharded
 * chain run, on internal rows:
 *   out = ck * x0 + cacc * (L_hat b1) - b2        (b2 NULL = 0)
 * flags: WG_CLEN_UIN  b1 holds u = b * dinv (unweighted handles: the gathers
 *                     read no values; own + halo rows, like t_km1 of wg_cheb_step)
 *        WG_CLEN_UPREV b2 holds u;  WG_CLEN_UOUT out receives u (not with FINAL)
 *        WG_CLEN_FINAL out is the finished sum S
 *        WG_CLEN_ACTIVE only the rows that enter wg_wavelet_features' chain.
 * With WG_CLEN_UIN on a large unweighted graph and F a multiple of 16 (<= 64)
 * this is the hybrid step (dense blocks on the matrix cores). */
#define WG_CLEN_UIN 1
#define WG_CLEN_UPREV 2
#define WG_CLEN_UOUT 4
#define WG_CLEN_FINAL 8
#define WG_CLEN_ACTIVE 16
int wg_clenshaw_step(wg_laplacian_t L, int64_t F, const float* b1, const float* b2, const float* x0,
                     float* out, double ck, double cacc, int32_t flags, void* stream);

/* Row permutation between the caller's order and the internal order:
 * direction 0: dst[i_internal] = src[perm[i]]  (caller -> internal)
 * direction 1: dst[perm[i]] = src[i_internal]  (internal -> caller). */
int wg_permute_rows(wg_laplacian_t L, int32_t direction, int64_t F, const float* src,
                    float* dst, void* stream);

/* -------------------------------------------------------------------------
 * a7: graph_wavelet_features (calibration/WATS.py:39-74), fused:
 *   T_0 = X0 (N,F) -> K Chebyshev steps -> S = sum_k exp(-s k) T_k ->
 *   H = S / (||S||_1,row + 1e-8).
 * F > 1 or weighted: the sum is evaluated by Clenshaw's recurrence (K SpMM
 * steps, no S stream; tuning key "clenshaw" 0 = forward recurrence).
 * X0, S, H in the caller's row order, row stride F.  S and H nullable (at
 * least one non-NULL).  K >= 0.  Uses the handle's workspace.
 * The FIRST call with a given F (after creation or a wg_laplacian_tune) builds
 * the kernel plans and grows the workspace SYNCHRONOUSLY (host copies, device
 * allocation): on a stream that is being captured it returns
 * WG_ERR_UNSUPPORTED -- call it once uncaptured first; later calls are plain
 * asynchronous launches and may be captured.
 * A chain can be replayed as a hipGraph of the handle's own once the same
 * arguments (pointers, F, K, s) were seen on two calls in a row
 * (tuning key "graph": 0 off = default, the replay measured slower than eager
 * launches on ROCm 7.2; 1 on; -1 only when active nnz x width <= 2^22).
 * ---------------------------------------------------------------------- */
int wg_wavelet_features(wg_laplacian_t L, const float* X0, int64_t F, int32_t K, double s,
                        float* S, float* H, void* stream);
/* F == 1 on a small unweighted graph (<= 2^18 nonzeros, <= 24576 active rows;
 * tuning key "chain": -1 auto, 0 off, 1 on, "chain_wg" workers) with S and H
 * given, wg_wavelet_features runs the whole chain in ONE launch of P
 * cooperating workgroups that hand each step's vector over as tagged granules
 * (csrc/chain.hip).  A wait gives up after 0.5 s instead of
 * hanging; that launch then writes NaN for every S / H row that depends on the
 * missing data and records the failure in host-mapped memory, and the NEXT
 * wg_wavelet_features call on the handle returns WG_ERR_TIMEOUT without
 * launching.  wg_chain_status waits for the handle's last one-launch chain
 * (an event recorded after it, also after a replay of the handle's own
 * captured chain; no device-wide sync -- except after a chain captured into a
 * graph the CALLER replays, which records no event of the handle's, where it
 * synchronises the device) and reports a failure since the last report
 * in *timed_out_host (1 = a chain's results are invalid; tuning key
 * "chain_fault" = j injects one: worker 0 skips publishing phase j).  Either
 * report switches the handle to the multi-launch path (until the next tune)
 * and drops a chain the handle captured with the one-launch kernel, so calling
 * again recomputes the features there (the Python
 * graph_wavelet_features does so by itself).  The plan never asks for more
 * workers than the occupancy query lets be resident (one per CU at most);
 * when the graph would need more, the multi-launch path runs. */
int wg_chain_status(wg_laplacian_t L, int32_t* timed_out_host);

/* Tuning: key "iter" (team-mode nonzeros per lane sub-group; default by
 * shape), "chunk_iter" (chunk-mode nonzeros per sub-group),
 * "clenshaw" (wavelet_features' heat sum, default 1), "tiles" (the hybrid
 * step, DESIGN.md 4.6: -1 auto, 0 off, 1 whenever it applies; with "tile_th",
 * "tile_rows", "tile_max", "tile_rg", "tile_mfma"), "nt" (store hints), and the keys listed in
 * efficient-gnn_amd/csrc/internal.h (struct Tuning).  Plan-shaping keys are
 * synchronous (they drop cached plans); launch-time keys are not.  Timing
 * probes whose results are wrong on purpose ("seg_mask", "probe",
 * "probe_tailwin", "xdelay") exist only in a build
 * with -DWG_TIMING_PROBES; this library rejects them as unknown keys. */
int wg_laplacian_tune(wg_laplacian_t L, const char* key, int64_t value);
/* Row shards: the halo columns [n_rows + offsets[q], n_rows + offsets[q+1])
 * come from peer q (q < n_groups; offsets[0] = 0, offsets[n_groups] = halo
 * size), each group in descending degree.  Lets the F = 1 hub kernel stage
 * the top columns of the own range and of every group in LDS.
 * wg_dist_create sets it from the receive counts; synchronous; drops the F = 1
 * plans built so far.  n_groups = 0 clears it. */
int wg_laplacian_set_halo_groups(wg_laplacian_t L, int32_t n_groups, const int64_t* offsets_host);
/* Human-readable launch plan of the step kernel for an F-column signal
 * (thread-local string, valid until the next call on this thread). */
const char* wg_laplacian_describe(wg_laplacian_t L, int64_t F);

/* Live kernel timing for benchmarks: while enabled, wg_wavelet_features
 * records a HIP event pair on `stream` around every Chebyshev-step launch.
 * wg_profile_collect waits for the recorded events (synchronous), returns
 * the summed step-kernel time (ms), the number of step launches and the
 * longest one since the last collect, and resets the pool. */
int wg_profile_enable(wg_laplacian_t L, int32_t enable);
int wg_profile_collect(wg_laplacian_t L, double* sum_ms_host, int64_t* launches_host,
                       double* max_ms_host);
/* The same events, one duration per launch in launch order (ms_host[i], i < min(cap, *n_host);
 * *n_host = launches recorded): e.g. a folded chain's first launch apart from its K - 1 plain step
 * launches.  Synchronous; resets the record like wg_profile_collect. */
int wg_profile_durations(wg_laplacian_t L, double* ms_host, int64_t cap, int64_t* n_host);

/* a6 standalone: H = S / (||S||_1,row + 1e-8) (calibration/WATS.py:71-72). */
int wg_row_l1_normalize(const float* S, float* H, int64_t n_rows, int64_t F, void* stream);

/* Row-id mapping between the caller's numbering and the internal one:
 * direction 0: out[i] = internal id of caller row rows[i]; 1: the inverse. */
int wg_laplacian_map_rows(wg_laplacian_t L, int32_t direction, const int32_t* rows, int64_t n,
                          int32_t* out, void* stream);

/* Multi-GPU halo pack: dst[i] = src[rows[i]] for i < n (row stride F). */
int wg_gather_rows(const float* src, const int32_t* rows, int64_t n, int64_t F, float* dst,
                   void* stream);

/* -------------------------------------------------------------------------
 * Section 8(e): the row-sharded chain with its halo exchange in native code.
 * One process per GPU.  `L` is this rank's shard (n_rows own rows; columns
 * [own | halo], the halo grouped by owner rank, as wats_hip/dist.py plans
 * it).  Per Chebyshev step (reference calibration/WATS.py:35-36) the own rows
 * peers asked for are packed (send_rows: internal ids, grouped by peer,
 * send_counts[q] for peer q) and exchanged with grouped ncclSend / ncclRecv
 * (RCCL over xGMI) into the halo rows (recv_counts[q] from peer q), then the
 * step kernel runs.  The chain is captured into a hipGraph on its second call
 * with the same arguments and replayed from then on (wg_dist_set_graph(D, 0)
 * keeps it eager; profiling via wg_profile_enable(L) also runs eagerly).
 * Each step exchanges, then computes (the overlap variants measured in round
 * 2 -- two-phase steps, two halo tiers, streamed row blocks -- were slower
 * and are removed).
 * wg_dist_unique_id fills NCCL_UNIQUE_ID_BYTES (128) bytes on one rank; every
 * rank passes the same bytes to wg_dist_create (collective: blocks until all
 * ranks joined); unique_id NULL = no RCCL communicator (IPC exchange below).  X0, S, H: own rows (n_rows, F) in the caller's order.
 * ---------------------------------------------------------------------- */
typedef struct wg_dist_s* wg_dist_t;
int wg_dist_unique_id(void* id_out /* 128 bytes, host */);
int wg_dist_create(wg_laplacian_t L, const void* unique_id, int32_t rank, int32_t world,
                   const int32_t* send_rows, const int64_t* send_counts_host,
                   const int64_t* recv_counts_host, wg_dist_t* out);
int wg_dist_destroy(wg_dist_t D);
int wg_dist_set_graph(wg_dist_t D, int32_t enable);
int wg_dist_wavelet_features(wg_dist_t D, const float* X0, int64_t F, int32_t K, double s, float* S,
                             float* H, void* stream);
/* State of the sharded chain, out8_host: [0] 0 (exchange, then the step),
 * [1] own rows, [2] halo rows, [3] rows sent, [4] world, [5] exchange (1 IPC,
 * 2 RCCL, 0 none), [6] 1 if a captured hipGraph exists, [7] 1 (halo tiers). */
int wg_dist_info(wg_dist_t D, int64_t* out8_host);
/* Total time (ms) and count of the halo exchanges (pack + RCCL, or the IPC
 * pull) recorded while profiling was enabled on the shard's handle; resets. */
int wg_dist_profile_collect(wg_dist_t D, double* exchange_ms_host, int64_t* count_host);

/* One-sided exchange over IPC-mapped peer memory, instead of RCCL (create
 * with unique_id = NULL).  wg_dist_ipc_local allocates this rank's shared
 * region (two slots of the extended vector at up to F_max columns, or of the
 * F = 1 LDS kernel's u, plus `world` int64 phase flags) and writes a 128-byte
 * blob (IPC handle + layout); every rank gathers all blobs (rank order) and
 * calls wg_dist_ipc_connect, with halo_src[h] = the owner's internal row id
 * of halo row h (device int32, n_halo entries).  Per phase a rank waits until
 * every peer completed as many phases as itself (flags written by the peers
 * with system-scope stores), pulls its halo rows with system-scope loads
 * from the owners' slots, runs the step and signals its peers.  A wait gives
 * up after 60 s and sets a flag that wg_dist_status reports (it synchronises
 * the device). */
int wg_dist_ipc_local(wg_dist_t D, int64_t F_max, void* blob_out /* 128 bytes, host */);
int wg_dist_ipc_connect(wg_dist_t D, const void* blobs_host /* world x 128 bytes */,
                        const int32_t* halo_src);
/* Exchange mode "sdma" (after wg_dist_ipc_connect): every phase the owner packs the rows each
 * peer asked for into one of two send buffers in its IPC region (in the peer's halo order) and
 * signals the phase; the receiver waits for the signals on a copy stream and copies each
 * owner's block into its halo rows with hipMemcpyAsync (peer DMA: the transfer takes no CU time
 * on a multi-GPU node), the step waiting on the copies.  peer_send_off[q] = the row of rank q's
 * send buffer where q packed this rank's block (q's send offset for this rank; collective setup,
 * wats_hip.dist).  Replaces the pull exchange of the same handle.
 * (reference: the halo exchange of the row-sharded Chebyshev step, WATS.py:35-36 sharded per
 * SURVEY.md 8(e); no reference interface -- the reference has no multi-GPU path) */
int wg_dist_ipc_sdma(wg_dist_t D, const int64_t* peer_send_off /* world, host */);
int wg_dist_status(wg_dist_t D, int32_t* timed_out_host);

/* -------------------------------------------------------------------------
 * Section 8(f)-2: the base model's propagation.  CompatibleGCN.forward
 * (reference src/gnn/model.py:43-52) computes deg = adj.sum(dim=1),
 * deg[deg == 0] = 1, adj_norm = adj / deg and twice x -> adj_norm @ x with a
 * dense (N,N) torch.mm.  wg_rownorm_create builds adj_norm (every stored
 * entry, self loops included, value a_ij / deg_i in float32) from the CSR
 * rows of adj (square, n x n; values NULL = all ones) as a handle of the same
 * step kernel; WG_FLAG_TRANSPOSE builds adj_norm^T (the backward operator).
 * wg_spmm: y = op @ x for x, y (n, F) row-major in the caller's order, sums in
 * float64.  Handles are freed with wg_laplacian_destroy.  Create is synchronous.
 * ---------------------------------------------------------------------- */
int wg_rownorm_create(int64_t n, int64_t nnz, const int64_t* indptr, const int32_t* indices,
                      const float* values, uint32_t flags, void* stream, wg_laplacian_t* out);
int wg_spmm(wg_laplacian_t op, int64_t F, const float* x, float* y, void* stream);

/* -------------------------------------------------------------------------
 * Section 8(f)-3: the WATS temperature head, fused.  Reference
 * calibration/WATS.py:101-105 (net = Linear(F,16) - ReLU - Linear(16,1)) and
 * :124-130 (T = log(exp(net(H)) + 1.1); out = log_softmax(logits / T)).
 * H (n,F), logits (n,C), out (n,C) row-major; W1 [hid][F], b1 [hid], W2 [hid]
 * (Linear(hid,1).weight), b2 [1] (torch nn.Linear layout); hid <= 64.
 * forward: out, and t_save[n] = net(H) (nullable; speeds up the backward).
 * backward: from grad_out (n,C): grad_logits (nullable) and the parameter
 * gradients gW1 [hid][F], gb1, gW2, gb2 (overwritten, not accumulated), float64
 * sums in a fixed order; `workspace` holds wg_wats_head_workspace bytes.
 * ---------------------------------------------------------------------- */
int wg_wats_head_forward(int64_t n, int64_t F, int64_t C, int32_t hid, const float* H,
                         const float* logits, const float* W1, const float* b1, const float* W2,
                         const float* b2, float* out, float* t_save, void* stream);
int wg_wats_head_workspace(int64_t n, int64_t F, int32_t hid, int64_t* bytes_host);
int wg_wats_head_backward(int64_t n, int64_t F, int64_t C, int32_t hid, const float* H,
                          const float* logits, const float* W1, const float* b1, const float* W2,
                          const float* b2, const float* out, const float* t_save,
                          const float* grad_out, float* grad_logits, float* gW1, float* gb1,
                          float* gW2, float* gb2, void* workspace, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WATS_HIP_H */
