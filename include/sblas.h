/*
 * sblas.h -- C-ABI of the MI355X-native sparse-BLAS hot path (libsblas.so).
 *
 * Plain C: pointers, sizes and an int status.  No torch / HIP types appear in
 * signatures (streams are passed as `void *` holding a hipStream_t; NULL is
 * the device's null stream).  Every entry point returns SBLAS_OK (0) or a
 * positive sblas_status; nothing calls exit().
 *
 * Two layers:
 *  1. Reference operator API (drop-in, HOST pointers, ngpu devices, nothing
 *     persists across calls) -- sblas_spMV_mgpu_*, sblas_csrmm_mgpu,
 *     sblas_sptrsv_syncfree.  The exact C++-linkage names of the reference
 *     (spMV_mgpu_baseline, ..., cusparse_mgpu_csrmm, sptrsv_syncfree_cuda) are
 *     declared in sblas_refapi.h and forward here.
 *  2. Persistent device API (DEVICE pointers, one device per object) used by
 *     the benchmarks and by multi-process runs: upload once, run many times.
 */
#ifndef SBLAS_H
#define SBLAS_H

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    SBLAS_OK = 0,
    SBLAS_ERR_INVALID = 1,     /* bad argument / shape */
    SBLAS_ERR_HIP = 2,         /* HIP runtime failure (message: sblas_last_error) */
    SBLAS_ERR_NOMEM = 3,       /* footprint > 0.8 x free device memory */
    SBLAS_ERR_NODEV = 4,       /* no usable GPU */
    SBLAS_ERR_UNSUPPORTED = 5, /* e.g. local nnz >= 2^31 */
    SBLAS_ERR_RCCL = 6,
    SBLAS_ERR_IO = 7           /* file could not be read / parsed */
} sblas_status;

/* Kernel selector; numbering follows test_spmv's `kernel` argument
 * (spmv/test/dspmv_test.cu:80): 1 = csrmv (row split), 2 = csrmv_mp
 * (nnz-balanced), 3 = CSR5 (disabled in the reference, enabled here). */
typedef enum {
    SBLAS_SPMV_AUTO = 0,     /* chosen per handle by sblas_csr_pick (below) */
    SBLAS_SPMV_ROWSPLIT = 1, /* CSR-adaptive row blocks, wave64, LDS stream */
    SBLAS_SPMV_CSR5 = 2,     /* wave64 CSR5-style tiles, segmented sum */
    SBLAS_SPMV_CSR5_ALT = 3, /* same kernel as 2 */
    SBLAS_SPMV_PANEL = 4,    /* XCD-affine column panels of the row-split kernel */
    SBLAS_SPMV_XSORT = 5     /* column-sorted XCD groups, LDS row accumulators
                                (within the fp64 bound, not bitwise repeatable) */
} sblas_spmv_algo;

const char *sblas_status_string(int status);
const char *sblas_last_error(void);
int sblas_version(void);
int sblas_device_count(int *count);

/* ------------------------------------------------------------------------ */
/* 1. Reference operator API (host pointers).  Cites: spmv/include/
 *    spmv_kernel.h:11-36, spmm/include/spmm_kernel.h:6-31,
 *    sptrsv/sptrsv_v1/src/sptrsv_syncfree_cuda.h:287-300.  Devices are
 *    ordinals 0..ngpu-1; if fewer physical GPUs exist the ordinals wrap
 *    (d % count) so multi-partition logic can run on one GPU. Return: 0 ok,
 *    -1 footprint > 0.8 x free memory (reference behaviour), >0 sblas_status. */
int sblas_spMV_mgpu_baseline(int m, int n, long long nnz, double *alpha,
                             double *csrVal, long long *csrRowPtr,
                             int *csrColIndex, double *x, double *beta,
                             double *y, int ngpu);
int sblas_spMV_mgpu_v1(int m, int n, long long nnz, double *alpha,
                       double *csrVal, long long *csrRowPtr, int *csrColIndex,
                       double *x, double *beta, double *y, int ngpu,
                       int kernel);
int sblas_spMV_mgpu_v2(int m, int n, long long nnz, double *alpha,
                       double *csrVal, long long *csrRowPtr, int *csrColIndex,
                       double *x, double *beta, double *y, int ngpu,
                       int kernel, long long nb, int copy_of_workspace);
/* spmv_helper.cu:16-39 (fixed: last row r with rowptr[r] <= idx, Q5) */
int sblas_get_row_from_index(int n, long long *a, long long idx);
double sblas_get_time(void);                 /* spmv_helper.cu:41-48 */
double sblas_get_gpu_availble_mem(int ngpu); /* spmv_helper.cu:51-76, GB */

/* C = alpha*A*B + beta*C; A m x k CSR (int32); B k x n column-major (ld=k);
 * C m x n column-major (ld=m).  Row-partitioned across ngpu devices. */
int sblas_csrmm_mgpu(int m, int n, int k, const double *alpha, int nnz_A,
                     int *csrRowPtr_A, int *csrColIndex_A, double *csrVal_A,
                     const double *beta, double *B_dense, double *C_dense,
                     int ngpu);

/* Same operation with the reference's own partition (dspmm_mgpu_baseline.cu
 * :147-150): A replicated, B and C split by columns, device d owning columns
 * [floor(d*n/ngpu), floor((d+1)*n/ngpu)).  Comparison mode; no exchange. */
int sblas_csrmm_mgpu_colsplit(int m, int n, int k, const double *alpha, int nnz_A,
                              int *csrRowPtr_A, int *csrColIndex_A, double *csrVal_A,
                              const double *beta, double *B_dense, double *C_dense,
                              int ngpu);

/* Sync-free triangular solve, CSC input, x output; validates against x_ref
 * when x_ref != NULL (rel-L1, prints like the reference) and reports gflops.
 * substitution 0 forward (lower), 1 backward (upper). rhs must be 1. */
int sblas_sptrsv_syncfree(const int *cscColPtr, const int *cscRowIdx,
                          const double *cscVal, int m, int n, int nnz,
                          int substitution, int rhs, int opt, double *x,
                          const double *b, const double *x_ref, double *gflops,
                          int ngpu);

/* sptrsv_v3's overload (sptrsv/sptrsv_v3/src/sptrsv_syncfree_cuda.h:227-241):
 * the columns are cut into ngpu*task equal-count tasks, task d runs on device
 * d % ngpu (round robin, :276-400).  One process drives all devices (the
 * reference: one MPI rank per PE over NVSHMEM); tasks run as concurrent
 * blocks of the multi-device pull executor.  Prints v3's lines. */
int sblas_sptrsv_syncfree_v3(const int *cscColPtr, const int *cscRowIdx,
                             const double *cscVal, int m, int n, int nnz,
                             int substitution, int rhs, int opt, double *x,
                             const double *b, const double *x_ref, double *gflops,
                             int ngpu, int task);

/* ------------------------------------------------------------------------ */
/* 2. Persistent device API. */
typedef struct sblas_csr_s *sblas_csr;

/* Upload rows [row_begin, row_end) of a HOST global CSR (int64 rowptr) whose
 * element range is [idx_begin, idx_end) -- i.e. a spMV_mgpu_v1 slice: first
 * and last rows may be partial (dspmv_mgpu_v1.cu:125-133).  The device copy
 * uses an int32 local rowptr. */
int sblas_csr_upload_slice(sblas_csr *out, int device, int n,
                           const long long *rowptr, const int *col,
                           const double *val, int row_begin, int row_end,
                           long long idx_begin, long long idx_end,
                           void *stream);
/* Wrap DEVICE arrays (int32 rowptr[m+1], col[nnz], val[nnz]); the arrays are
 * copied into padded storage owned by the handle. */
int sblas_csr_from_device(sblas_csr *out, int device, int m, int n, int nnz,
                          const int *d_rowptr, const int *d_col,
                          const double *d_val, void *stream);
int sblas_csr_destroy(sblas_csr A);
int sblas_csr_info(sblas_csr A, int *m, int *n, long long *nnz);
/* Build the analysis for an algorithm (row blocks / CSR5 tiles); run once. */
int sblas_csr_analyse(sblas_csr A, int algo, void *stream);
/* y = alpha*A*x + beta*y on the handle's device; x, y DEVICE pointers.
 * Concurrency: the analysis keeps per-launch scratch on the device (XSORT:
 * work-queue claim heads that each launch re-arms for the next one, and the
 * wide-range partial sums; PANEL: the panel partials; ROWSPLIT: long-row
 * partials; CSR5: tile carries).  A handle therefore allows ONE launch in
 * flight at a time: issue its launches on one stream (they are then
 * ordered), or synchronise between launches on different streams.  Two
 * overlapping launches of one handle give wrong y in both.  Distinct handles
 * (even of the same matrix) are independent. */
int sblas_spmv(sblas_csr A, int algo, double alpha, const double *d_x,
               double beta, double *d_y, void *stream);
/* sblas_spmv that also measures the call's device span: ms = time from the
 * first kernel's start to the last kernel's end (events stamped by the
 * runtime at the kernels themselves, hipExtLaunchKernelGGL), excluding the
 * host's launch latency and event-record gaps.  Waits for the call. */
int sblas_spmv_timed(sblas_csr A, int algo, double alpha, const double *d_x,
                     double beta, double *d_y, void *stream, float *ms);
/* The algorithm SBLAS_SPMV_AUTO runs for this handle (decided once, cached;
 * analyse / spmv / spmv_timed with SBLAS_SPMV_AUTO resolve through it).  A
 * device probe measures column locality: over up to 65,536 sampled rows, the
 * share of entries whose column is within 16 columns (one 128-B line of x)
 * of the previous entry's (the previous row's last, for a row's first), and
 * how widely the columns spread.  The checks run in this order:
 *   1. XSORT when the handle holds >= 2M nonzeros, n*8 <= 120 MiB (its
 *      column groups) and the columns are spread (any adjacency: banded and
 *      stencil matrices included);
 *   2. else ROWSPLIT when the adjacency is >= 1/2 (e.g. the reference
 *      generator's contiguous columns, banded or blocked rows) or the columns
 *      are crowded into a narrow range, whose gathers then coalesce;
 *   3. else PANEL.
 * XSORT accumulates in LDS with fp64 atomics: its y is within the fp64 bound
 * but NOT bitwise repeatable run to run, so AUTO may pick a non-deterministic
 * kernel (ROWSPLIT, CSR5 and PANEL are deterministic).  If the XSORT analysis
 * is unsupported for the matrix, sblas_csr_analyse falls back to PANEL and the
 * choice becomes PANEL.  SBLAS_AUTO=<1..5> overrides the choice. */
int sblas_csr_pick(sblas_csr A, void *stream, int *algo);
/* Bitwise-repeatable SpMV on this handle (on != 0).  ROWSPLIT, CSR5 and
 * PANEL always are (each row's sum in a fixed order); XSORT then runs its
 * ordered form (a stream's chunks added in chunk order, the narrow group
 * walk fixed per range): the same y bit for bit on every call, within the
 * same fp64 bound, at some cost (bench.py `deterministic_beside`).  AUTO's
 * choice is unchanged.  New handles take SBLAS_DETERMINISTIC (=1: on; read
 * once per process); the reference's cusparseDcsrmv
 * (dspmv_mgpu_baseline.cu:163-167) is repeatable the same way. */
int sblas_csr_set_deterministic(sblas_csr A, int on);
/* The XSORT plan's shape (8 values): ready, row ranges, wide ranges, work
 * items, grid (persistent workgroups), solo (power-law layout), 256-entry
 * chunks, most chunks of one item.  For tools and tests. */
int sblas_csr_xsort_info(sblas_csr A, long long *info);
int sblas_csr_get_deterministic(sblas_csr A, int *on);
/* XCD column panels the analysed plan of `algo` runs over (0: the plain
 * layout / not analysed).  ROWSPLIT and CSR5 build per-panel plans (P = 4
 * on config 2) on large scattered-column matrices (x > 8 MiB, nnz >= 2M, most
 * sampled rows span > n/4 of the columns; test hooks "rs_panel" /
 * "csr5_panel" force either form); PANEL always does (unless only one panel
 * holds entries). */
int sblas_csr_panels(sblas_csr A, int algo, int *panels);
/* Device bytes held by the analysis of `algo` (free memory before - after
 * sblas_csr_analyse; 0 if not analysed): the layout's cost beside the CSR. */
long long sblas_csr_plan_bytes(sblas_csr A, int algo);
/* bytes the algorithm must move per call (DESIGN.md "Algorithmic bytes"). */
long long sblas_spmv_algorithmic_bytes(sblas_csr A, int beta_nonzero);

/* SpMM on a device handle: C(m x n, ldc) = alpha*A*B(k x n, ldb) + beta*C.
 * b_layout 0 = column-major B (ld=ldb >= k), 1 = row-major B (ld >= n).
 * Concurrency: the handle owns the SpMM scratch (the row-major B panel and
 * the split-row partials), so ONE sblas_spmm per handle may be in flight:
 * issue a handle's calls on one stream, or synchronise between calls on
 * different streams or threads.  Distinct handles are independent.
 * The plan is built on the first call and tuned to that call's width n (the
 * C-tile form sizes its slab sets so that XCDs x sets x row blocks x 16-column
 * groups of n fill the CUs about once): later calls with another n are
 * correct but keep the first call's grid and partial slots; for a different
 * width at full speed, use a second handle. */
int sblas_spmm(sblas_csr A, int n, double alpha, const double *d_B, int ldb,
               int b_layout, double beta, double *d_C, int ldc, void *stream);

/* Device CSR -> CSC transpose of a handle; outputs DEVICE arrays sized
 * colptr[n+1], rowidx[nnz], cval[nnz]; row indices ascend within columns
 * (bit-exact with tranpose.h:6-43).  A stable sort of the entries by column:
 * MSD partition passes + one pass per final bucket of columns (n > 512), or
 * LSD radix passes (n <= 512, or SBLAS_TRANSPOSE_ALGO=lsd). */
int sblas_csr_transpose(sblas_csr A, int *d_colptr, int *d_rowidx,
                        double *d_cval, void *stream);

/* Triangular solve handle over a DEVICE lower/upper CSC matrix with the
 * diagonal stored first (lower) / last (upper) in each column. */
typedef struct sblas_trsv_s *sblas_trsv;
int sblas_trsv_create(sblas_trsv *out, int device, int n, int nnz,
                      const int *d_colptr, const int *d_rowidx,
                      const double *d_val, int substitution, void *stream);
/* algo 0 = sync-free CSC push (reference algorithm), 1 = CSR pull with ready
 * flags (deterministic sums), 2 = level-set (rows grouped by level,
 * findlevel.h:71-147; one synchronisation per level; built on the first
 * algo-2 solve; x bit-identical to algo 1), 3 = the pull executor with its
 * tickets in level order (same analysis; x bit-identical to algo 1),
 * 4 = AUTO: the pull executor in level order when at least a quarter of the
 * rows depend on a row of their own 64-row wave (stencil / FEM triangles),
 * else in natural order (decided once per handle by a device probe). */
int sblas_trsv_solve(sblas_trsv T, int algo, const double *d_b, double *d_x,
                     void *stream);
/* algo 4's choice for this handle (1 or 3), probing on first use. */
int sblas_trsv_pick(sblas_trsv T, void *stream, int *algo);
int sblas_trsv_levels(sblas_trsv T, int *nlevel);
int sblas_trsv_destroy(sblas_trsv T);
/* SpTRSM, rhs right-hand sides (sptrsm_syncfree_cuda_executor,
 * sptrsv_v1/src/sptrsv_syncfree_cuda.h:170-282): d_b, d_x device n x rhs
 * row-major.  Pull executor; rhs == 1 is sblas_trsv_solve(T, 1, ...). */
int sblas_trsv_solve_rhs(sblas_trsv T, int rhs, const double *d_b, double *d_x, void *stream);
/* SpTRSM with the executor chosen: algo 1 = the pull executor above (opt
 * ignored); algo 3 = the pull executor with tickets in level order, 4 = 1 or
 * 3 as sblas_trsv_pick chooses (opt ignored; 2 is invalid); algo 0 = the reference's push dataflow (CSC scatter of left sums
 * with fp64 atomics, sptrsv_syncfree_cuda.h:170-282) with its lane mapping
 * opt: 1 OPT_WARP_NNZ (lanes over a column's entries), 2 OPT_WARP_RHS (lanes
 * over the right-hand sides), 3 OPT_WARP_AUTO (per column: rhs mapping when
 * (len <= rhs || rhs > 16) && len < 2048).  rhs >= 1.  Push sums land in
 * arrival order: within the fp64 bound, not bitwise repeatable. */
int sblas_trsv_solve_rhs_opt(sblas_trsv T, int algo, int opt, int rhs, const double *d_b,
                             double *d_x, void *stream);
/* Out-of-core SpMV (the task pool + streams of spMV_mgpu_v2,
 * dspmv_mgpu_v2.cu:33-441).  HOST CSR (int64 rowptr), x and y: the matrix is
 * streamed through ngpu devices in nnz-balanced chunks of chunk_nnz, over
 * nstreams streams per device (H2D of one chunk overlaps the kernel of the
 * previous), so it may exceed the aggregate HBM.  y = alpha*A*x + beta*y.
 * stats (optional, 6 doubles): total seconds, H2D GB/s of the streaming
 * phase, chunks, devices, seconds pinning the caller's col/val, seconds
 * (re)allocating the per-device pool (0 once warm). */
int sblas_spmv_ooc(int m, int n, long long nnz, double alpha, const long long *rowptr,
                   const int *col, const double *val, const double *x, double beta, double *y,
                   int ngpu, long long chunk_nnz, int nstreams, double *stats);
/* Multi-GPU CSR -> CSC transpose (replaces kernal_sptrans,
 * sptrans/sptrans_v1/src/sptrans_kernal.h:80-555).  HOST arrays in and out
 * (int32 rowptr as the reference).  nnz-balanced whole-row blocks, block d
 * transposed on device d % count, pieces composed on device 0; the result is
 * the stable global transpose (rows ascending within a column), bit-exact.
 * ms_transpose / ms_compose (optional): wall times of the two phases. */
int sblas_csr2csc_mgpu(int m, int n, int nnz, int ngpu, const int *rowptr, const int *col,
                       const double *val, int *colptr, int *rowidx, double *cval,
                       double *ms_transpose, double *ms_compose);
/* sptrans driver (cuda_sptrans / kernal_sptrans): transposes on ngpu devices,
 * prints the reference's timing lines and its value/pointer checks against
 * the *_ref arrays (when given), plus a row-index check. */
int sblas_sptrans(int m, int n, int nnz, int ngpu, const int *csrRowPtr, const int *csrColIdx,
                  const double *csrVal, int *cscRowIdx, int *cscColPtr, double *cscVal,
                  const int *cscRowIdx_ref, const int *cscColPtr_ref, const double *cscVal_ref);
/* Multi-GPU sync-free solve (replaces sptrsv_v3's NVSHMEM):
 * HOST CSC in, x out.  nnz-balanced blocks of the solve order, one per device
 * ordinal (d % count); full-length x per device in fine-grained memory;
 * producers push x_i to every later block over xGMI; consumers poll local
 * memory.  Blocks that wrap onto one GPU run concurrently (own streams).  b, x: n x rhs row-major (x[i*rhs+k], the reference's layout).
 * solve_ms (optional) = wall time of the kernels. */
int sblas_trsv_mgpu_solve(const int *colptr, const int *rowidx, const double *val,
                          int n, int substitution, int rhs, const double *b, double *x,
                          int ngpu, double *solve_ms);
/* Same executor over ngpu*tasks blocks, block d on device d % ngpu (wrapping
 * onto the visible GPUs); balance 0 = nnz-balanced blocks, 1 = equal row
 * counts (sptrsv_v3's split).  All blocks are launched on their own streams
 * before any is waited for, so blocks sharing a GPU run concurrently (each
 * with that GPU's workgroup budget divided by its block count). */
int sblas_trsv_mgpu_solve_tasks(const int *colptr, const int *rowidx, const double *val,
                                int n, int substitution, int rhs, const double *b, double *x,
                                int ngpu, int tasks, int balance, double *solve_ms);

/* Persistent form of the multi-GPU solve: create builds the blocks once
 * (CSC -> CSR of L on the host, ngpu*tasks blocks of the solve order, block d
 * on device d % ngpu, its rows and a fine-grained x uploaded); run uploads b
 * (HOST n x rhs row-major), resets x and the control words, solves and copies
 * x back (solve_ms: wall time of the kernels); repeated runs redo no O(nnz)
 * host work.  The one-shot sblas_trsv_mgpu_solve* above are create + run +
 * destroy. */
typedef struct sblas_trsv_mgpu_s *sblas_trsv_mgpu;
int sblas_trsv_mgpu_create(sblas_trsv_mgpu *out, const int *colptr, const int *rowidx,
                           const double *val, int n, int substitution, int rhs, int ngpu,
                           int tasks, int balance);
int sblas_trsv_mgpu_run(sblas_trsv_mgpu h, const double *b, double *x, double *solve_ms);
/* Where the blocks run: block d's physical device and row count (arrays of
 * *nblocks entries; any may be NULL). */
int sblas_trsv_mgpu_info(sblas_trsv_mgpu h, int *nblocks, int *block_device, int *block_rows);
int sblas_trsv_mgpu_destroy(sblas_trsv_mgpu h);
/* create fails with SBLAS_ERR_UNSUPPORTED (or SBLAS_ERR_HIP) before anything
 * is launched when two of its devices have no peer access (producers store
 * x_i into later blocks' memory; sptrsv_v3 needs NVSHMEM the same way,
 * sptrsv_v3/src/sptrsv_syncfree_cuda.h:245-249), so no block ever waits on a
 * store that cannot arrive; fine-grained allocation failures return the same
 * way.  Peer links are reference-counted per process: destroying one handle
 * or context never takes a link away from another live one. */

/* Multi-partition y assembly after an allgather of padded slices: partition
 * r's slice starts at d_gathered + r*stride; d_meta (DEVICE, 3*g ints) holds
 * {row0, nrows, cont} per partition; cont = first row continues partition
 * r-1 (its entry is added, in partition order).  If d_y_local != NULL it
 * is partition `self`'s slice and is prepared as the next call's y input
 * (continuation entry zeroed, last entry refreshed when the next partition
 * continues that row). */
int sblas_assemble_slices(const double *d_gathered, int g, long long stride,
                          const int *d_meta, double *d_y, int self,
                          double *d_y_local, void *stream);

/* y assembly for the cyclic row-chunk distribution (whole rows, no split
 * rows): chunk j = rows [j*chunk_rows, ...) is held by partition j % g at its
 * local rows (j / g)*chunk_rows + ..., partition r's slice starting at
 * d_gathered + r*stride.  Writes all m rows of d_y.  Replaces the
 * reference's host-side y copy-back (dspmv_mgpu_v1.cu:224-248) when the rows
 * are dealt cyclically; stride must hold ceil(ceil(m/chunk_rows)/g) chunks. */
int sblas_assemble_cyclic(const double *d_gathered, int g, long long stride,
                          long long chunk_rows, long long m, double *d_y, void *stream);

/* ------------------------------------------------------------------------ */
/* 3. Multi-GPU context (single process, RCCL over xGMI).  Replaces the
 *    reference's host-driven multi-GPU SpMV (spmv/src/dspmv_mgpu_v1.cu:16-280)
 *    for callers that keep the matrix: the slices stay resident per device,
 *    x is replicated with ncclBroadcast, and the y slices are exchanged on the
 *    devices (one ncclAllGather + placement, or the literal ncclAllReduce of
 *    the zero-padded y of BASELINE configs[2]), so every device holds the full
 *    y.  Devices must be distinct (no wrapping: one RCCL rank per GPU).
 *    Hardware status: on the 1-GPU pool this runs with g = 1 only; g > 1
 *    (ncclCommInitAll over distinct devices, split-row carries, cyclic
 *    placement across devices) is covered by CPU tests of the partition and
 *    placement logic and is unverified on multi-GPU hardware. */
typedef struct sblas_ctx_s *sblas_ctx;
typedef enum {
    SBLAS_CTX_ALLGATHER = 0, /* equal padded slices all-gathered, placed on device */
    SBLAS_CTX_ALLREDUCE = 1  /* zero-padded full y summed (nnz partition only;
                                dspmv_mgpu_v1.cu:235-248's merge as a collective) */
} sblas_ctx_exchange;
/* ncclCommInitAll over devlist[0..ngpu) (NULL: 0..ngpu-1). */
int sblas_ctx_create(sblas_ctx *out, int ngpu, const int *devlist);
int sblas_ctx_destroy(sblas_ctx ctx);
int sblas_ctx_ngpu(sblas_ctx ctx, int *ngpu);
/* The communicator as RCCL reports it: *nranks = ncclCommCount of device 0's
 * communicator (0 for a loopback context, which has none), and per context
 * device d its ordinal (ncclCommCuDevice; the wrapped ordinal in loopback). */
int sblas_ctx_comm_info(sblas_ctx ctx, int *nranks, int *devices);
/* HOST CSR (int64 rowptr) distributed over the devices and analysed for
 * `algo` (sblas_spmv_algo).  partition 0 = cyclic row chunks (chunk j of
 * ceil(m/(8g)) rows on device j % g; whole rows), 1 = spMV_mgpu_v1's
 * nnz-balanced split with split rows merged on the device, 2 = the
 * cost-weighted whole-row split (sblas_partition_cost, w =
 * 3, the cost of a row end in CSR5 entries).  Exchange SBLAS_CTX_ALLGATHER. */
int sblas_ctx_matrix_upload(sblas_ctx ctx, int m, int n, const long long *rowptr,
                            const int *col, const double *val, int algo, int partition);
/* Same with the exchange chosen (sblas_ctx_exchange); SBLAS_CTX_ALLREDUCE
 * needs a contiguous-range partition, 1 or 2 (SBLAS_ERR_INVALID otherwise). */
int sblas_ctx_matrix_upload_ex(sblas_ctx ctx, int m, int n, const long long *rowptr,
                               const int *col, const double *val, int algo, int partition,
                               int exchange);
/* Cyclic partition + all-gather with the exchange overlapped (replaces the
 * per-task copy/compute overlap of spMV_mgpu_v2, dspmv_mgpu_v2.cu:128-170):
 * each device's local chunks are cut into `parts` consecutive groups (at most
 * one per chunk; parts = 1 is sblas_ctx_matrix_upload(..., 0)), each group
 * its own handle running the whole slice's algorithm (AUTO resolved on the
 * whole slice).  A step runs part p's kernel on the device's main stream and
 * part p's all-gather + placement on a second (comm) stream while part
 * p + 1's kernel runs; the main stream then joins.  Stats: kernel = start ..
 * last part kernel, exchange = the tail after it, step = start .. join. */
int sblas_ctx_matrix_upload_parts(sblas_ctx ctx, int m, int n, const long long *rowptr,
                                  const int *col, const double *val, int algo, int parts);
/* The parts the loaded matrix runs in (1: not overlapped; 0: nothing loaded). */
int sblas_ctx_parts(sblas_ctx ctx, int *parts);
/* Device d's share: rows, entries, and the algorithmic bytes of its SpMV
 * launch with beta != 0 (sblas_spmv_algorithmic_bytes).  Any may be NULL. */
int sblas_ctx_slice_info(sblas_ctx ctx, int d, long long *rows, long long *nnz,
                         long long *alg_bytes_beta);
/* The SpMV algorithm device d's slice runs (its own sblas_csr_pick when the
 * context was loaded with SBLAS_SPMV_AUTO). */
int sblas_ctx_slice_algo(sblas_ctx ctx, int d, int *algo);
int sblas_ctx_set_x(sblas_ctx ctx, const double *x); /* host x -> every device */
int sblas_ctx_set_y(sblas_ctx ctx, const double *y); /* host y (beta input) */
/* y = alpha*A*x + beta*y on every device; afterwards each device holds the
 * full y, which is also the next call's y input.  stats (optional, 3
 * doubles, ms, max over devices): kernel, exchange (collective + placement),
 * whole step.  A one-device context (not overlapped) has nothing to
 * exchange: its kernel writes the full y in place (exchange ~0). */
int sblas_ctx_spmv(sblas_ctx ctx, double alpha, double beta, double *stats);
/* sblas_ctx_spmv for timing.  delay_us > 0: every device's stream first
 * waits delay_us on the device (the host enqueues the whole step meanwhile)
 * and then joins a one-word all-reduce that lines the devices up; each
 * device's span then runs from its start event to the end of its exchange,
 * without the host's launch latency.  wait = 0 returns once the step is
 * enqueued (sblas_ctx_sync waits).  stats (3 + 3g doubles, ms): max over
 * devices of kernel / exchange / step, then kernel / exchange / step of
 * device 0, 1, ... */
int sblas_ctx_spmv_ex(sblas_ctx ctx, double alpha, double beta, double delay_us, int wait,
                      double *stats);
/* Waits for the last step and returns its stats (3 + 3g doubles, as above). */
int sblas_ctx_sync(sblas_ctx ctx, double *stats);
int sblas_ctx_get_y(sblas_ctx ctx, int device_index, double *y); /* -> host */
/* Bind (or unbind with NULL) a context for the reference API: while bound,
 * sblas_spMV_mgpu_v1 / spMV_mgpu_v1 with ngpu == the context's size run on
 * it (RCCL exchange) instead of the host merge.  Binding LENDS the context:
 * each such call uploads and analyses its matrix into the context (nnz
 * partition, all-gather), replacing whatever matrix the caller had resident
 * there, and that matrix stays allocated after the call. */
int sblas_ctx_bind(sblas_ctx ctx);
/* The cyclic distribution's plan: chunk_rows = ceil(m/(g*chunks_per_rank)),
 * stride = rows of one device's padded slice.  No GPU needed. */
int sblas_cyclic_plan(long long m, int g, int chunks_per_rank, long long *chunk_rows,
                      long long *stride);
/* Local CSR of partition d under it: chunks d, d+g, ... concatenated (host
 * arrays; call with lrowptr/lcol/lval NULL to size).  No GPU needed. */
int sblas_cyclic_local_csr(int m, const long long *rowptr, const int *col, const double *val,
                           int g, long long chunk_rows, int d, long long *local_m,
                           long long *local_nnz, long long *lrowptr, int *lcol, double *lval);

/* ------------------------------------------------------------------------ */
/* Host utilities (no GPU needed). */
/* Matrix-Market: mode 0 = full mmio_data semantics (symmetric expansion,
 * pattern -> 1.0); mode 1 = test_spmv 'f' loader (file order, Q1/Q2);
 * mode 2 = test_spmv 'b' (values 1e-5); mode 3 = test_spmm's loader
 * (dspmm_baseline_test.cu:420-455: "%d %d %lg" entries, no symmetric
 * expansion) bucketed by row stably, file order within a row (feed it to
 * sblas_coo_sortbyrow for the reference's (row, col) order).  Call with
 * rowptr==NULL to size. */
int sblas_mm_read(const char *path, int mode, int *m, int *n, long long *nnz,
                  long long *rowptr, int *col, double *val);
/* Binary CSR cache.  sblas_mm_read keeps one automatically
 * when SBLAS_MM_CACHE is set ("1": <file>.m<mode>.csrbin beside the .mtx;
 * otherwise a directory), keyed by the source's size and mtime.  These two
 * write/read a standalone .csrbin (two-call protocol as sblas_mm_read). */
int sblas_csrbin_write(const char *path, int m, int n, long long nnz, const long long *rowptr,
                       const int *col, const double *val);
int sblas_csrbin_read(const char *path, int *m, int *n, long long *nnz, long long *rowptr,
                      int *col, double *val);

/* sortbyrow + COO -> CSR of test_spmm (spmm/test/dspmm_baseline_test.cu:
 * 41-55, 461-493): row/col/val (nnz entries) sorted in place by (row, col),
 * rowptr[m+1] filled from the row counts.  Duplicates keep their input order
 * (the reference's qsort leaves it unspecified). */
int sblas_coo_sortbyrow(int m, long long nnz, int *row, int *col, double *val, int *rowptr);

/* nnz-balanced partition of spMV_mgpu_v1 (dspmv_mgpu_v1.cu:60-94, Q5 fixed).
 * Arrays of g entries. */
int sblas_partition_nnz(int m, long long nnz, const long long *rowptr, int g,
                        long long *start_idx, long long *end_idx,
                        int *start_row, int *end_row, int *start_flag);
/* Cost-weighted whole-row split: contiguous row ranges balancing
 * sum_r (nnz_r + w), no split rows (start_flag all 0); same outputs as
 * sblas_partition_nnz.  w = 0 balances entries with rows kept whole. */
int sblas_partition_cost(int m, const long long *rowptr, int g, double w,
                         long long *start_idx, long long *end_idx,
                         int *start_row, int *end_row, int *start_flag);
/* row-block partition (dspmv_mgpu_baseline.cu:64-65); g+1 entries. */
int sblas_partition_rowblock(int m, int g, int *row_start);

/* Scaled synthetic of DESIGN.md: rows < n/8 have `heavy` nnz, others
 * `light`; distinct uniform-random (or prefix) sorted columns; values U[0,1).
 * Generates rows [row_begin,row_end) into caller arrays (rowptr is global,
 * int64, all n+1 entries filled by sblas_gen_synth_rowptr). */
int sblas_gen_synth_rowptr(int n, int heavy, int light, long long *rowptr);
int sblas_gen_synth_rows(int n, int heavy, int light, int prefix_cols,
                         unsigned long long seed, const long long *rowptr,
                         int row_begin, int row_end, int *col, double *val);
int sblas_gen_vector(int n, unsigned long long seed, double *v);
/* 3-D stencil (points = 7 or 27) on an nx*ny*nz grid, natural ordering: the
 * structured SuiteSparse kind.  Off-diagonals -U[0,1), diagonal 1 + sum|off|.
 * rowptr int64 (n+1); col == NULL: rowptr only. */
int sblas_gen_stencil3d(int nx, int ny, int nz, int points, unsigned long long seed,
                        long long *rowptr, int *col, double *val);
/* R-MAT power-law graph (a,b,c = 0.57,0.19,0.19), 2^scale vertices,
 * edge_factor*2^scale draws, labels permuted, duplicates merged, values U[0,1).
 * col/val hold cap >= edge_factor*2^scale entries; nnz = rowptr[2^scale]. */
int sblas_gen_rmat(int scale, int edge_factor, unsigned long long seed, long long *rowptr,
                   int *col, double *val, long long cap);
/* Unit-lower-triangular CSC (diagonal first) for SpTRSV benchmarks:
 * `offd` distinct rows per column within (j, j+band], values
 * (1 + r%10)/(20*row_len).  rowidx == NULL: colptr only. */
int sblas_gen_lower_banded(int n, int offd, int band, unsigned long long seed,
                           int *colptr, int *rowidx, double *val);

/* Measured memory ceiling (bench.py's `measured_peak`):
 * hand-written HBM stream probes on the current device, enqueued on
 * `stream`.  mode 0 = read `bytes` of src (16-B loads, 8 in flight per lane,
 * grid-stride; dst = an 8-byte sink that is never written in practice),
 * 1 = the same with non-temporal loads, 2 = copy src -> dst, 3 / 4 = modes
 * 0 / 1 with each workgroup streaming one contiguous span.  `bytes` a multiple of 16;
 * wg_per_cu 256-thread workgroups per CU (1..32).  Not part of the reference
 * API: the probes price the SpMV kernels against what this GPU streams. */
int sblas_hbm_probe(int mode, const void *src, void *dst, long long bytes, int wg_per_cu,
                    void *stream);
/* The same, waiting for it and returning its device span in *ms (events the
 * runtime stamps at the kernel's start and end, as sblas_spmv_timed). */
int sblas_hbm_probe_timed(int mode, const void *src, void *dst, long long bytes, int wg_per_cu,
                          void *stream, float *ms);

/* Test hooks (not part of the reference API). */
/* on != 0: every peer link the library asks for is refused, and a
 * multi-block trsv_mgpu treats blocks sharing a GPU as distinct devices, so
 * the refusal path runs on a one-GPU box.  Process-wide. */
int sblas_test_deny_peer_access(int on);
/* References the library holds on the a -> b peer link (0: none). */
int sblas_peer_refs(int a, int b);
/* Planner override for tests (set = 0 clears it), read when a plan is built:
 * "xs_cap" (xsort work per item: small values give many items, exercising the
 * dynamic claims on small matrices), "xs_allwide" (0/1), "xs_solo" (0/1),
 * "spmm_ctile" (0/1: C-tile form), "spmm_mfma_fill" (MFMA tile threshold),
 * "rs_panel" / "csr5_panel" (0/1: XCD-panel forms), "panels" (panel count).
 * Process-wide; production code never sets them. */
int sblas_test_set_option(const char *name, double value, int set);

#ifdef __cplusplus
}
#endif
#endif
