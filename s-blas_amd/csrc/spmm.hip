// spmm.hip -- fp64 CSR x dense SpMM for gfx950.
//
// Replaces cusparseDcsrmm (spmm/src/dspmm_mgpu_baseline.cu:225-240):
// C(m x n, col-major, ldc) = alpha * A(m x k, CSR) * B(k x n) + beta * C.
//
// Layout: B is consumed ROW-major (row j of B = the n values A's column j
// multiplies), so each nonzero a_ij pulls one contiguous n*8-byte row of B
// (512 B at n = 64: one wave load).  A column-major B (the reference's
// host layout) is transposed once into a row-major panel owned by the
// handle (k_transpose_B, LDS-tiled 64x64).
//
// Kernel: one wave per (row of A, 64-column slab of C).  The wave loads 64
// (col, val) pairs of the row with one coalesced load each, then broadcasts
// them lane-to-lane (__shfl) while every lane FMAs its column of B; eight
// independent B-row loads are kept in flight.  Accumulation order per C entry
// is the row's storage order (same as the oracle).
#include <vector>

#include "sblas_internal.hpp"

namespace sblas {

template <bool kBeta>
__global__ __launch_bounds__(256) void k_spmm_rowwave(
    const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ B, long long ldb,
    int m, int n, int nslab, double alpha, double beta, double *__restrict__ C,
    long long ldc)
{
    const int lane = threadIdx.x & 63;
    const long long w = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= (long long)m * nslab) return;
    const int r = (int)(w / nslab);
    const int c = (int)(w % nslab) * 64 + lane;
    const bool live = c < n;
    const int cc = live ? c : 0;
    const int a0 = rowptr[r], a1 = rowptr[r + 1];
    double acc = 0.0;
    for (int base = a0; base < a1; base += 64) {
        const int cnt = min(64, a1 - base);
        const int my_j = lane < cnt ? col[base + lane] : 0;
        const double my_a = lane < cnt ? val[base + lane] : 0.0;
        int q = 0;
        for (; q + 8 <= cnt; q += 8) {
            double b[8], a[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = __shfl(my_j, q + u, 64);
                a[u] = __shfl(my_a, q + u, 64);
                b[u] = B[(long long)j * ldb + cc];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += a[u] * b[u];
        }
        for (; q < cnt; ++q) {
            const int j = __shfl(my_j, q, 64);
            const double a = __shfl(my_a, q, 64);
            acc += a * B[(long long)j * ldb + cc];
        }
    }
    if (live) {
        double *o = C + (long long)c * ldc + r;
        *o = kBeta ? alpha * acc + beta * *o : alpha * acc;
    }
}

// col-major B (k x n, ld=ldb) -> row-major panel Bt (k x n, ld=n)
__global__ void k_transpose_B(const double *__restrict__ B, long long ldb, int k, int n,
                              double *__restrict__ Bt)
{
    __shared__ double tile[64][65];
    const int j0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 64 x 4
    for (int cc = ty; cc < 64; cc += 4) {
        const int j = j0 + tx, c = c0 + cc;
        if (j < k && c < n) tile[cc][tx] = B[(long long)c * ldb + j];
    }
    __syncthreads();
    for (int jj = ty; jj < 64; jj += 4) {
        const int j = j0 + jj, c = c0 + tx;
        if (j < k && c < n) Bt[(long long)j * n + c] = tile[tx][jj];
    }
}

struct SpmmScratch {
    double *bt = nullptr;
    size_t bytes = 0;
};
static thread_local SpmmScratch g_scratch[64];

int launch_spmm(const sblas_csr_s &A, int n, double alpha, const double *B, int ldb,
                int b_layout, double beta, double *C, int ldc, hipStream_t s)
{
    if (A.m == 0 || n == 0) return SBLAS_OK;
    const double *Brow = B;
    long long ldr = ldb;
    if (b_layout == 0) {
        SpmmScratch &S = g_scratch[A.device & 63];
        const size_t need = sizeof(double) * (size_t)A.n * (size_t)n;
        if (S.bytes < need) {
            (void)hipFree(S.bt);
            S.bt = nullptr;
            S.bytes = 0;
            SBLAS_HIP(hipMalloc(&S.bt, need));
            S.bytes = need;
        }
        if (A.n > 0) {
            dim3 grid((A.n + 63) / 64, (n + 63) / 64);
            hipLaunchKernelGGL(k_transpose_B, grid, dim3(256), 0, s, B, (long long)ldb, A.n, n, S.bt);
        }
        Brow = S.bt;
        ldr = n;
    }
    const int nslab = (n + 63) / 64;
    const long long waves = (long long)A.m * nslab;
    const unsigned nb = (unsigned)((waves + 3) / 4);
    if (beta != 0.0)
        hipLaunchKernelGGL(k_spmm_rowwave<true>, dim3(nb), dim3(256), 0, s, A.rowptr, A.col, A.val,
                           Brow, ldr, A.m, n, nslab, alpha, beta, C, (long long)ldc);
    else
        hipLaunchKernelGGL(k_spmm_rowwave<false>, dim3(nb), dim3(256), 0, s, A.rowptr, A.col, A.val,
                           Brow, ldr, A.m, n, nslab, alpha, beta, C, (long long)ldc);
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

}  // namespace sblas
