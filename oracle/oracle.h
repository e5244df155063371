/*
 * oracle.h -- CPU restatement of the pnnl/s-blas algorithms on the hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by or
 * called from the product (libsblas).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the timed
 * CPU baseline.  Each function cites the reference file:line it restates
 * (paths relative to the reference checkout).
 *
 * Pinning (see DESIGN.md "Oracle"):
 *   - Matrix-Market loader (mmio_data semantics) and the serial sync-free SpTRSV
 *     are checked bit-exactly against the reference's own host sources compiled
 *     in place (oracle/ref/Makefile -> oracle/_ref/libsblas_ref.so).
 *   - SpMV/SpMM arithmetic lives in cuSPARSE (csrmv / csrmv_mp / csrmm, CUDA 9.0
 *     per the prebuilt spmm/test/test_spmm linkage; README.md:53 "CUDA 10.1 or
 *     newer") which is absent here: restated as its published definition
 *     y = alpha*A*x + beta*y, sequential per-row sum in storage order.  Parity is
 *     anchored on the reference's call sites and its test (abs 1e-3,
 *     spmv/test/dspmv_test.cu:390-401) plus the stated fp64 bound in DESIGN.md.
 */
#ifndef SBLAS_ORACLE_H
#define SBLAS_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* alpha/beta exactly as test_spmv draws them: unseeded glibc rand()
 * (spmv/test/dspmv_test.cu:281-282).  `skip` = rand() calls made before
 * (the 'g' generator draws one per nnz first, dspmv_test.cu:191). */
void orc_ref_alpha_beta(long long skip, double *alpha, double *beta);

/* ---- Matrix-Market ---------------------------------------------------- */
/* Banner + size line.  flags bit0 pattern, bit1 real, bit2 complex,
 * bit3 integer, bit4 symmetric/hermitian.  mmio.h:254 / :339. */
int orc_mm_info(const char *path, int *m, int *n, long long *nnz_file, int *flags);

/* test_spmv 'f' loader (dspmv_test.cu:101-136, rowptr :217-251): COO kept in
 * FILE ORDER, rowptr from row counts (quirk Q1), no symmetric expansion (Q2),
 * data_type 'b' -> every value 1e-5.  Arrays sized from orc_mm_info. */
int orc_mm_load_testspmv(const char *path, char data_type, long long *rowptr,
                         int *col, double *val);

/* mmio_data (sptrsv/sptrsv_v1/src/mmio_highlevel.h:137-296): pattern/int/real/
 * complex(real part), symmetric expansion, rows bucketed in file order.
 * Two calls: with rowptr==NULL only *nnz is returned. */
int orc_mm_load_mmio(const char *path, int *m, int *n, int *nnz, int *is_sym,
                     int *rowptr, int *col, double *val);

/* ---- SpMV -------------------------------------------------------------- */
/* cusparseDcsrmv semantics (call sites dspmv_mgpu_baseline.cu:163-167):
 * y[i] = alpha * sum_j a_ij x_j + beta * y[i]; sum in storage order; beta==0
 * does not read y. */
void orc_csr_spmv(int m, const long long *rowptr, const int *col,
                  const double *val, const double *x, double alpha, double beta,
                  double *y);
/* Same arithmetic, OpenMP over rows (CPU baseline on all host cores). */
void orc_csr_spmv_omp(int m, const long long *rowptr, const int *col,
                      const double *val, const double *x, double alpha,
                      double beta, double *y, int nthreads);
/* Checker helper (tests only): the per-row fp64 bound of DESIGN.md §3,
 * bound[i] = 4*gamma_k*sum_j |alpha*a_ij*x_j| + 4u*|beta*y0[i]| + 1e-300,
 * gamma_k = k*u/(1-k*u), u = 2^-53, k = row length.  OpenMP over rows. */
void orc_spmv_bound(int m, const long long *rowptr, const int *col, const double *val,
                    const double *x, double alpha, double beta, const double *y0,
                    double *bound);

/* The reference's binary search, verbatim semantics (spmv_helper.cu:16-39). */
int orc_get_row_from_index_ref(int n, const long long *a, long long idx);
/* Fixed (Q5): last row r with rowptr[r] <= idx (upper bound - 1). */
int orc_row_of_index(int m, const long long *rowptr, long long idx);

/* spMV_mgpu_baseline row-block split (dspmv_mgpu_baseline.cu:60-87):
 * rows [floor(d*m/g), floor((d+1)*m/g)). row_start has g+1 entries. */
void orc_partition_rowblock(int m, int g, int *row_start);

/* spMV_mgpu_v1 nnz split (dspmv_mgpu_v1.cu:60-94), Q5 fixed. */
void orc_partition_nnz(int m, long long nnz, const long long *rowptr, int g,
                       long long *start_idx, long long *end_idx, int *start_row,
                       int *end_row, int *start_flag);

/* Whole spMV_mgpu_v1 / baseline dataflow on the CPU: per-partition csrmv on
 * the local slice with a local int32 rowptr (dspmv_mgpu_v1.cu:125-133), then
 * the host fix-up y[r] += part_{d-1} - beta*y0 (:235-248). */
void orc_spmv_mgpu_v1(int m, int n, long long nnz, double alpha,
                      const double *val, const long long *rowptr,
                      const int *col, const double *x, double beta, double *y,
                      int g);
void orc_spmv_mgpu_baseline(int m, int n, long long nnz, double alpha,
                            const double *val, const long long *rowptr,
                            const int *col, const double *x, double beta,
                            double *y, int g);

/* ---- generators -------------------------------------------------------- */
/* test_spmv 'g n' (dspmv_test.cu:137-208): first m/8 rows ceil(0.9n) cols
 * 0..; others ceil(0.01n); val = rand()/RAND_MAX (unseeded).  Blocks clamped
 * to m (quirk Q3).  orc_gen_ref_nnz gives the size first. */
long long orc_gen_ref_nnz(int n);
void orc_gen_ref(int n, int *coo_row, int *coo_col, double *coo_val);

/* Scaled synthetic (DESIGN.md "Synthetic"): rows < n/8 get `heavy` nnz,
 * the rest `light`; columns distinct, uniform (or prefix 0..d-1), sorted;
 * per-row SplitMix64 stream seeded from (seed,row); values U[0,1).
 * rowptr only: orc_gen_synth_rowptr. */
void orc_gen_synth_rowptr(int n, int heavy, int light, long long *rowptr);
void orc_gen_synth(int n, int heavy, int light, int prefix_cols,
                   unsigned long long seed, const long long *rowptr, int *col,
                   double *val);
/* Dense vector U[0,1) from one SplitMix64 stream. */
void orc_gen_vector(int n, unsigned long long seed, double *v);

/* ---- transpose / triangular solve -------------------------------------- */
/* tranpose.h:6-43: histogram, exclusive scan, stable row-order scatter. */
void orc_transpose(int m, int n, int nnz, const int *rowptr, const int *col,
                   const double *val, int *colptr, int *rowidx, double *cval);

/* L (forward) or U (backward) with unit diagonal from A's pattern
 * (sptrsv_v1/src/main.cu:150-186); off-diagonal values rand()%10+1 after
 * srand(seed) (the reference seeds with time(NULL), quirk Q8). Returns nnz;
 * with out arrays NULL only counts. */
int orc_build_tri(int m, const int *rowptr, const int *col, int substitution,
                  unsigned seed, int *trowptr, int *tcol, double *tval);

/* x_ref[i] = rand()%10+1 continuing the same rand() stream
 * (main.cu:329-332), and b = L*x_ref by CSC SpMV (main.cu:344-355). */
void orc_tri_rhs(int n, const int *colptr, const int *rowidx, const double *val,
                 double *x_ref, double *b);

/* Serial sync-free SpTRSV (sptrsv_syncfree_serialref.h:6-108). */
int orc_sptrsv_serial(const int *colptr, const int *rowidx, const double *val,
                      int n, int substitution, int rhs, const double *b,
                      double *x);

/* Level sets of a lower-triangular CSC matrix (findlevel.h:71-147):
 * returns nlevel; level_of[i] = level of row/column i. */
int orc_levels_lower(int n, const int *colptr, const int *rowidx, int *level_of);

/* ---- SpMM -------------------------------------------------------------- */
/* cusparseDcsrmm semantics (dspmm_mgpu_baseline.cu:225-240): C(m x n, ld=m,
 * column-major) = alpha*A(m x k)*B(k x n, ld=k) + beta*C; per (row, col of
 * C) sum in storage order. */
void orc_spmm(int m, int n, int k, double alpha, const int *rowptr,
              const int *col, const double *val, const double *B, int ldb,
              double beta, double *C, int ldc);
/* orc_spmm's arithmetic (same per-entry storage-order sum) in OpenMP over
 * rows, for full-size checks; if bound != NULL also the per-entry fp64 bound
 * (ld = ldc) 4*gamma_k*sum_j |alpha*a_ij*b_jc| + 4u*|beta*c0|, computed
 * from the C passed in (before it is overwritten).  B is read with stride
 * ldb per column when b_rowmajor == 0 (column-major, ld = ldb) and as
 * B[j*ldb + c] when b_rowmajor != 0. */
void orc_spmm_omp(int m, int n, double alpha, const int *rowptr, const int *col,
                  const double *val, const double *B, int ldb, int b_rowmajor, double beta,
                  double *C, int ldc, double *bound, int nthreads);

/* qsort-by-(row,col) COO -> CSR as test_spmm does
 * (spmm/test/dspmm_baseline_test.cu:41-55,461-493). */
void orc_coo_sort_to_csr(int m, int nnz, int *coo_row, int *coo_col,
                         double *coo_val, int *rowptr);

#ifdef __cplusplus
}
#endif
#endif
