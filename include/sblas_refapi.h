/*
 * sblas_refapi.h -- the reference's operator API with its original C++
 * linkage, exported by libsblas.so so a driver written against the
 * reference headers links unchanged:
 *   spmv/include/spmv_kernel.h:11-36    (spMV_mgpu_baseline/v1/v2, helpers)
 *   spmm/include/spmm_kernel.h:6-31     (cusparse_mgpu_csrmm[_omp])
 *   sptrsv/sptrsv_v1/src/sptrsv_syncfree_cuda.h:287-300 (sptrsv_syncfree_cuda)
 *   sptrsv/sptrsv_v3/src/sptrsv_syncfree_cuda.h:227-241 (its `int task` overload)
 *   sptrans/sptrans_v1/src/sptrans_cuda.h:11-23, sptrans_kernal.h:80-93
 *                                       (cuda_sptrans, kernal_sptrans)
 * Each forwards to the extern "C" sblas_* entry of the same arguments
 * (include/sblas.h).  No cuSPARSE is involved despite the names.
 */
#ifndef SBLAS_REFAPI_H
#define SBLAS_REFAPI_H

#ifdef __cplusplus
int spMV_mgpu_baseline(int m, int n, long long nnz, double *alpha, double *csrVal,
                       long long *csrRowPtr, int *csrColIndex, double *x, double *beta,
                       double *y, int ngpu);
int spMV_mgpu_v1(int m, int n, long long nnz, double *alpha, double *csrVal,
                 long long *csrRowPtr, int *csrColIndex, double *x, double *beta, double *y,
                 int ngpu, int kernel);
int spMV_mgpu_v2(int m, int n, long long nnz, double *alpha, double *csrVal,
                 long long *csrRowPtr, int *csrColIndex, double *x, double *beta, double *y,
                 int ngpu, int kernel, long long nb, int copy_of_workspace);
int get_row_from_index(int n, long long *a, long long idx);
double get_time();
double get_gpu_availble_mem(int ngpu);

int cusparse_mgpu_csrmm(const int m, const int n, const int k, const double *alpha,
                        const int nnz_A, int *csrRowPtr_A, int *csrColIndex_A,
                        double *csrVal_A, const double *beta, double *B_dense,
                        double *C_dense, const int ngpu);
int cusparse_mgpu_csrmm_omp(const int m, const int n, const int k, const double *alpha,
                            const int nnz_A, int *csrRowPtr_A, int *csrColIndex_A,
                            double *csrVal_A, const double *beta, double *B_dense,
                            double *C_dense, const int ngpu);

int sptrsv_syncfree_cuda(const int *cscColPtrTR, const int *cscRowIdxTR,
                         const double *cscValTR, int m, int n, int nnzTR, int substitution,
                         int rhs, int opt, double *x, const double *b, const double *x_ref,
                         double *gflops, int ngpu);
/* sptrsv/sptrsv_v3/src/sptrsv_syncfree_cuda.h:227-241: ngpu*task
 * equal-column tasks, task d on device d % ngpu (single process here). */
int sptrsv_syncfree_cuda(const int *cscColPtrTR, const int *cscRowIdxTR,
                         const double *cscValTR, int m, int n, int nnzTR, int substitution,
                         int rhs, int opt, double *x, const double *b, const double *x_ref,
                         double *gflops, int ngpu, int task);

int cuda_sptrans(const int m, const int n, const int nnz, const int *csrRowPtr,
                 const int *csrColIdx, const double *csrVal, int *cscRowIdx, int *cscColPtr,
                 double *cscVal, const int *cscRowIdx_ref, const int *cscColPtr_ref,
                 const double *cscVal_ref);
int kernal_sptrans(const int m, const int n, const int nnz, int ngpu, const int *csrRowPtr,
                   const int *csrColIdx, const double *csrVal, int *cscRowIdx, int *cscColPtr,
                   double *cscVal, const int *cscRowIdx_ref, const int *cscColPtr_ref,
                   const double *cscVal_ref);
#endif

#endif
