// ref_driver.cpp -- exposes the reference's own host-side C code, compiled IN
// PLACE from /root/reference (never copied), behind a few extern "C" entry
// points so tests can pin the oracle restatement against it.
//
// TEST INFRASTRUCTURE ONLY: built into oracle/_ref/libsblas_ref.so by
// oracle/ref/Makefile when /root/reference is present.  Only the headers that
// compile from their own sources are used:
//   sptrsv/sptrsv_v1/src/{common.h, mmio.h, mmio_highlevel.h,
//                         sptrsv_syncfree_serialref.h}
// tranpose.h / findlevel.h / utils.h need cusparse.h (absent) -> unbuildable
// here; their semantics are pinned through the restatement instead.
#include "common.h"
#include "mmio_highlevel.h"
#include "sptrsv_syncfree_serialref.h"

extern "C" {

// mm_read_banner + mm_read_mtx_crd_size (mmio.h:254, :339)
int ref_mm_header(const char *path, int *m, int *n, int *nz, int *flags)
{
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    MM_typecode t;
    if (mm_read_banner(f, &t) != 0) { fclose(f); return -2; }
    int rc = mm_read_mtx_crd_size(f, m, n, nz);
    fclose(f);
    if (rc != 0) return -3;
    int fl = 0;
    if (mm_is_pattern(t)) fl |= 1;
    if (mm_is_real(t)) fl |= 2;
    if (mm_is_complex(t)) fl |= 4;
    if (mm_is_integer(t)) fl |= 8;
    if (mm_is_symmetric(t) || mm_is_hermitian(t)) fl |= 16;
    *flags = fl;
    return 0;
}

// mmio_info + mmio_data (mmio_highlevel.h:8-296)
int ref_mmio_info(const char *path, int *m, int *n, int *nnz, int *is_sym)
{
    return mmio_info(m, n, nnz, is_sym, const_cast<char *>(path));
}
int ref_mmio_data(const char *path, int *rowptr, int *col, double *val)
{
    return mmio_data(rowptr, col, val, const_cast<char *>(path));
}

// sptrsv_syncfree_analyser + _executor (sptrsv_syncfree_serialref.h:6-108)
int ref_sptrsv_serial(const int *colptr, const int *rowidx, const double *val,
                      int n, int nnz, int substitution, int rhs,
                      const double *b, double *x)
{
    int *deg = (int *)malloc(sizeof(int) * n);
    sptrsv_syncfree_analyser(rowidx, n, n, nnz, deg);
    int rc = sptrsv_syncfree_executor(colptr, rowidx, val, deg, n, n,
                                      substitution, rhs, b, x);
    free(deg);
    return rc;
}

// The same two calls timed apart, the way sptrsv_syncfree_serialref
// (sptrsv_syncfree_serialref.h:110-155) times and prints them: analyser ms
// and executor ms (the executor figure is the reference's CPU baseline for
// configs[4]).  bench.py's cpu_baseline child only.
int ref_sptrsv_serial_timed(const int *colptr, const int *rowidx, const double *val,
                            int n, int nnz, int substitution, int rhs,
                            const double *b, double *x, double *analyser_ms, double *executor_ms)
{
    int *deg = (int *)malloc(sizeof(int) * n);
    struct timeval t1, t2;
    gettimeofday(&t1, NULL);
    sptrsv_syncfree_analyser(rowidx, n, n, nnz, deg);
    gettimeofday(&t2, NULL);
    *analyser_ms = (t2.tv_sec - t1.tv_sec) * 1000.0 + (t2.tv_usec - t1.tv_usec) / 1000.0;
    gettimeofday(&t1, NULL);
    int rc = sptrsv_syncfree_executor(colptr, rowidx, val, deg, n, n, substitution, rhs, b, x);
    gettimeofday(&t2, NULL);
    *executor_ms = (t2.tv_sec - t1.tv_sec) * 1000.0 + (t2.tv_usec - t1.tv_usec) / 1000.0;
    free(deg);
    return rc;
}

}  // extern "C"
