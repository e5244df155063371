// assemble.hip -- device-side merge of the per-partition y slices after the
// RCCL allgather (multi-GPU SpMV).
//
// Partition r owns rows [row0[r], row0[r]+nrows[r]); when cont[r] is set its
// first row continues partition r-1's last row (an nnz-balanced split) and
// its first entry is a partial alpha*p to be ADDED, in partition order, as the
// reference's host fix-up does (spmv/src/dspmv_mgpu_v1.cu:235-248).  The
// gathered buffer holds g slices of `stride` doubles (padded equal chunks, as
// all_gather_into_tensor / ncclAllGather require).
#include "sblas_internal.hpp"

namespace sblas {

__global__ void k_assemble_copy(const double *__restrict__ gathered, int g, long long stride,
                                const int *__restrict__ meta, double *__restrict__ y)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)g * stride) return;
    const int r = (int)(i / stride);
    const int k = (int)(i - (long long)r * stride);
    const int row0 = meta[3 * r], nrows = meta[3 * r + 1], cont = meta[3 * r + 2];
    if (k >= nrows || (k == 0 && cont)) return;
    y[row0 + k] = gathered[i];
}

// Carries in partition order (deterministic), then -- if this rank's local
// slice is given -- prepare it as the next call's y input: its continuation
// entry is zeroed (partial = alpha*p only) and its last entry takes the
// assembled value when the next partition continues that row.
__global__ void k_assemble_carry(const double *__restrict__ gathered, int g, long long stride,
                                 const int *__restrict__ meta, double *__restrict__ y, int self,
                                 double *__restrict__ y_local)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    for (int r = 0; r < g; ++r)
        if (meta[3 * r + 2] && meta[3 * r + 1] > 0) y[meta[3 * r]] += gathered[(long long)r * stride];
    if (y_local && self >= 0 && self < g) {
        const int row0 = meta[3 * self], nrows = meta[3 * self + 1];
        if (nrows > 0) {
            if (self + 1 < g && meta[3 * (self + 1) + 2]) y_local[nrows - 1] = y[row0 + nrows - 1];
            if (meta[3 * self + 2]) y_local[0] = 0.0;
        }
    }
}

// Cyclic row-chunk distribution (sblas_dist.CyclicPlan): chunk j = rows
// [j*R, min((j+1)*R, m)) lives on rank j % g at local rows (j / g)*R + ...;
// every rank owns whole rows, so there is nothing to carry.  One thread per
// GLOBAL row: y is written in order and each chunk is read contiguously.
__global__ void k_assemble_cyclic(const double *__restrict__ gathered, int g, long long stride,
                                  long long R, long long m, double *__restrict__ y)
{
    const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const long long j = r / R;
    const int d = (int)(j % g);
    const long long k = (j / g) * R + (r - j * R);
    y[r] = gathered[(long long)d * stride + k];
}

}  // namespace sblas

using namespace sblas;

extern "C" int sblas_assemble_cyclic(const double *d_gathered, int g, long long stride,
                                     long long chunk_rows, long long m, double *d_y, void *stream)
{
    if (g <= 0 || stride < 0 || chunk_rows <= 0 || m < 0 || !d_gathered || !d_y)
        return SBLAS_ERR_INVALID;
    // every rank's local rows must fit its slice: ceil(nchunks / g) chunks
    const long long nchunks = (m + chunk_rows - 1) / chunk_rows;
    if (((nchunks + g - 1) / g) * chunk_rows > stride) return SBLAS_ERR_INVALID;
    if (m == 0) return SBLAS_OK;
    hipLaunchKernelGGL(k_assemble_cyclic, dim3((unsigned)((m + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, d_gathered, g, stride, chunk_rows, m, d_y);
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

extern "C" int sblas_assemble_slices(const double *d_gathered, int g, long long stride,
                                     const int *d_meta, double *d_y, int self,
                                     double *d_y_local, void *stream)
{
    if (g <= 0 || stride < 0 || !d_meta || !d_y) return SBLAS_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    const long long total = (long long)g * stride;
    if (total > 0)
        hipLaunchKernelGGL(k_assemble_copy, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           d_gathered, g, stride, d_meta, d_y);
    hipLaunchKernelGGL(k_assemble_carry, dim3(1), dim3(64), 0, s, d_gathered, g, stride, d_meta, d_y,
                       self, d_y_local);
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}
