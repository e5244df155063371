// transpose.hip -- device CSR -> CSC transpose with bit-exact indices.
//
// Semantics of sptrsv/sptrsv_v1/src/tranpose.h:6-43 (matrix_transposition):
// column histogram, exclusive scan, then a STABLE scatter in row order, so
// row indices ascend inside every column and equal-(row,col) duplicates keep
// their CSR order.  GPU form:
//   1. histogram of columns (int atomics) into colptr[c+1];
//   2. in-place inclusive scan (multi-block, recursive) -> colptr;
//   3. scatter the CSR element index e of every nonzero to an atomic slot of
//      its column (order inside a column is arbitrary here);
//   4. segmented sort of each column's element indices (e ascending == CSR
//      order == the reference's stable order): per-thread insertion sort for
//      short columns, LDS bitonic sort per workgroup up to 4096, a
//      global-memory merge sort per workgroup beyond;
//   5. gather: rowidx = row of e (binary search of rowptr), cval = val[e].
#include <algorithm>
#include <climits>
#include <vector>

#include "sblas_internal.hpp"

namespace sblas {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

// Inclusive scan of each 2048-element tile; tile totals to bsum.
__global__ __launch_bounds__(kScanThreads) void k_scan_tiles(int *__restrict__ a, long long len,
                                                             int *__restrict__ bsum)
{
    __shared__ int wtot[kScanThreads / 64];
    const long long base = (long long)blockIdx.x * kScanTile + (long long)threadIdx.x * kScanItems;
    int v[kScanItems];
    int run = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const long long i = base + k;
        run += (i < len) ? a[i] : 0;
        v[k] = run;
    }
    const int incl = wave_incl_scan(run);
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) wtot[wid] = incl;
    __syncthreads();
    int woff = 0;
    for (int w = 0; w < wid; ++w) woff += wtot[w];
    const int off = woff + incl - run;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const long long i = base + k;
        if (i < len) a[i] = v[k] + off;
    }
    if (threadIdx.x == kScanThreads - 1) bsum[blockIdx.x] = woff + incl;
}

__global__ void k_scan_add(int *__restrict__ a, long long len, const int *__restrict__ bsum)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long tile = i / kScanTile;
    if (i < len && tile > 0) a[i] += bsum[tile - 1];
}

// In-place inclusive scan; scratch must hold >= sum over levels of tiles.
int scan_inclusive(int *a, long long len, int *scratch, hipStream_t s)
{
    if (len <= 0) return SBLAS_OK;
    const long long tiles = (len + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)tiles), dim3(kScanThreads), 0, s, a, len, scratch);
    if (tiles > 1) {
        SBLAS_TRY(scan_inclusive(scratch, tiles, scratch + tiles, s));
        hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, a, len,
                           scratch);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

__global__ void k_col_hist(const int *__restrict__ col, long long nnz, int *__restrict__ cnt1)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nnz) atomicAdd(&cnt1[col[e] + 1], 1);
}

__global__ void k_col_scatter(const int *__restrict__ col, long long nnz, int *__restrict__ next,
                              int *__restrict__ perm)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nnz) perm[atomicAdd(&next[col[e]], 1)] = (int)e;
}

// Short columns sorted in place by their own thread; others queued.
__global__ void k_sort_short(const int *__restrict__ colptr, int n, int *__restrict__ perm,
                             int *__restrict__ qcount, int *__restrict__ qmed,
                             int *__restrict__ qbig)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const int a = colptr[c], b = colptr[c + 1];
    const int len = b - a;
    if (len <= 32) {
        for (int i = a + 1; i < b; ++i) {
            const int key = perm[i];
            int j = i - 1;
            while (j >= a && perm[j] > key) {
                perm[j + 1] = perm[j];
                --j;
            }
            perm[j + 1] = key;
        }
    } else if (len <= 4096) {
        qmed[atomicAdd(&qcount[0], 1)] = c;
    } else {
        qbig[atomicAdd(&qcount[1], 1)] = c;
    }
}

__global__ __launch_bounds__(256) void k_sort_medium(const int *__restrict__ colptr,
                                                     int *__restrict__ perm,
                                                     const int *__restrict__ qcount,
                                                     const int *__restrict__ qmed)
{
    __shared__ int sk[4096];
    const int nq = qcount[0];
    for (int q = blockIdx.x; q < nq; q += gridDim.x) {
        const int c = qmed[q];
        const int a = colptr[c], len = colptr[c + 1] - a;
        int P = 64;
        while (P < len) P <<= 1;
        for (int i = threadIdx.x; i < P; i += 256) sk[i] = i < len ? perm[a + i] : INT_MAX;
        __syncthreads();
        for (int k = 2; k <= P; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = threadIdx.x; i < P; i += 256) {
                    const int ixj = i ^ j;
                    if (ixj > i) {
                        const bool up = (i & k) == 0;
                        const int x = sk[i], y = sk[ixj];
                        if (up ? x > y : x < y) {
                            sk[i] = y;
                            sk[ixj] = x;
                        }
                    }
                }
                __syncthreads();
            }
        }
        for (int i = threadIdx.x; i < len; i += 256) perm[a + i] = sk[i];
        __syncthreads();
    }
}

// Bottom-up merge sort of one long column per workgroup in global memory
// (ping-pong with tmp, same offsets).  Keys are unique.
__global__ __launch_bounds__(256) void k_sort_big(const int *__restrict__ colptr,
                                                  int *__restrict__ perm, int *__restrict__ tmp,
                                                  const int *__restrict__ qcount,
                                                  const int *__restrict__ qbig)
{
    const int nq = qcount[1];
    for (int q = blockIdx.x; q < nq; q += gridDim.x) {
        const int c = qbig[q];
        const int a = colptr[c], len = colptr[c + 1] - a;
        int *src = perm + a, *dst = tmp + a;
        for (int w = 1; w < len; w <<= 1) {
            for (int i = threadIdx.x; i < len; i += 256) {
                const int run = i / (2 * w);
                const int s0 = run * 2 * w;
                const int m0 = min(s0 + w, len), e0 = min(s0 + 2 * w, len);
                const int key = src[i];
                int pos;
                if (i < m0) {  // left run: count right-run keys < key
                    int lo = m0, hi = e0;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (src[mid] < key) lo = mid + 1;
                        else hi = mid;
                    }
                    pos = s0 + (i - s0) + (lo - m0);
                } else {  // right run: count left-run keys < key
                    int lo = s0, hi = m0;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (src[mid] < key) lo = mid + 1;
                        else hi = mid;
                    }
                    pos = s0 + (i - m0) + (lo - s0);
                }
                dst[pos] = key;
            }
            __syncthreads();
            int *t = src;
            src = dst;
            dst = t;
        }
        if (src != perm + a)
            for (int i = threadIdx.x; i < len; i += 256) perm[a + i] = src[i];
        __syncthreads();
    }
}

__global__ void k_gather_csc(const int *__restrict__ rowptr, int m, const double *__restrict__ val,
                             const int *__restrict__ perm, long long nnz, int *__restrict__ rowidx,
                             double *__restrict__ cval)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nnz) return;
    const int e = perm[p];
    int lo = 0, hi = m - 1;  // row r: rowptr[r] <= e < rowptr[r+1]
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rowptr[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    if (rowidx) rowidx[p] = lo;
    if (cval) cval[p] = val[e];
}

struct TransposeScratch {
    int *buf = nullptr;
    size_t ints = 0;
};
static thread_local TransposeScratch g_tscratch[64];

int launch_transpose(const sblas_csr_s &A, int *colptr, int *rowidx, double *cval, hipStream_t s)
{
    const long long nnz = A.nnz;
    const int n = A.n;
    SBLAS_HIP(hipMemsetAsync(colptr, 0, sizeof(int) * ((size_t)n + 1), s));
    if (nnz == 0) return SBLAS_OK;
    // scratch: next[n+1] | perm[nnz] | tmp[nnz] | q[2] | qmed[n] | qbig[n] | scan
    const size_t scan_ints = (size_t)((n + 1) / kScanTile + 64) * 2;
    const size_t need = (size_t)(n + 1) + 2 * (size_t)nnz + 4 + 2 * (size_t)n + scan_ints;
    TransposeScratch &S = g_tscratch[A.device & 63];
    if (S.ints < need) {
        if (S.buf) SBLAS_HIP(hipStreamSynchronize(s));  // earlier work on s may still use it
        (void)hipFree(S.buf);
        S.buf = nullptr;
        S.ints = 0;
        SBLAS_HIP(hipMalloc(&S.buf, need * sizeof(int)));
        S.ints = need;
    }
    int *next = S.buf;
    int *perm = next + (n + 1);
    int *tmp = perm + nnz;
    int *qc = tmp + nnz;
    int *qmed = qc + 4;
    int *qbig = qmed + n;
    int *scan = qbig + n;
    const unsigned gb = (unsigned)((nnz + 255) / 256);
    hipLaunchKernelGGL(k_col_hist, dim3(gb), dim3(256), 0, s, A.col, nnz, colptr);
    SBLAS_TRY(scan_inclusive(colptr, (long long)n + 1, scan, s));
    SBLAS_HIP(hipMemcpyAsync(next, colptr, sizeof(int) * ((size_t)n + 1), hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_col_scatter, dim3(gb), dim3(256), 0, s, A.col, nnz, next, perm);
    SBLAS_HIP(hipMemsetAsync(qc, 0, sizeof(int) * 4, s));
    hipLaunchKernelGGL(k_sort_short, dim3((n + 255) / 256), dim3(256), 0, s, colptr, n, perm, qc,
                       qmed, qbig);
    hipLaunchKernelGGL(k_sort_medium, dim3(1024), dim3(256), 0, s, colptr, perm, qc, qmed);
    hipLaunchKernelGGL(k_sort_big, dim3(256), dim3(256), 0, s, colptr, perm, tmp, qc, qbig);
    hipLaunchKernelGGL(k_gather_csc, dim3(gb), dim3(256), 0, s, A.rowptr, A.m, A.val, perm, nnz,
                       rowidx, cval);
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}


// ---- multi-device CSR -> CSC (sptrans_v1 kernal_sptrans,
// sptrans/sptrans_v1/src/sptrans_kernal.h:80-555) -------------------------
// Rows are split into g nnz-balanced blocks of whole rows; block d is
// transposed on device d % count by the single-device path above (stable:
// rows ascend within a column).  The pieces then travel to device 0 (peer DMA
// over xGMI) and one element-parallel kernel composes them: block d's column
// c lands after blocks 0..d-1's entries of c, so the result is the global
// stable transpose, bit for bit.  (The reference's compose leaves row indices
// block-local, a quirk not inherited.)
__global__ void k_compose_ptr(const int *__restrict__ ptrs, int g, int n, int *__restrict__ colptr,
                              int *__restrict__ base)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c > n) return;
    int tot = 0;
    for (int d = 0; d < g; ++d) tot += ptrs[(size_t)d * (n + 1) + c];
    colptr[c] = tot;
    if (c == n) return;
    int acc = tot;
    for (int d = 0; d < g; ++d) {
        base[(size_t)d * n + c] = acc;
        acc += ptrs[(size_t)d * (n + 1) + c + 1] - ptrs[(size_t)d * (n + 1) + c];
    }
}

__global__ void k_compose_val(const int *__restrict__ ptrs, const int *__restrict__ base,
                              const long long *__restrict__ start, const int *__restrict__ row0,
                              int g, int n, long long nnz, const int *__restrict__ rid_cat,
                              const double *__restrict__ val_cat, int *__restrict__ rowidx,
                              double *__restrict__ cval)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nnz) return;
    int d = 0;
    while (d + 1 < g && start[d + 1] <= p) ++d;
    const int e = (int)(p - start[d]);
    const int *cp = ptrs + (size_t)d * (n + 1);
    int lo = 0, hi = n - 1;  // column c: cp[c] <= e < cp[c+1]
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (cp[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    const int dst = base[(size_t)d * n + lo] + (e - cp[lo]);
    rowidx[dst] = rid_cat[p] + row0[d];
    cval[dst] = val_cat[p];
}

}  // namespace sblas

extern "C" int sblas_csr2csc_mgpu(int m, int n, int nnz, int ngpu, const int *rowptr, const int *col,
                                  const double *val, int *colptr_out, int *rowidx_out,
                                  double *cval_out, double *ms_transpose, double *ms_compose)
{
    using namespace sblas;
    if (m < 0 || n < 0 || nnz < 0 || ngpu <= 0 || !rowptr || !colptr_out ||
        (nnz && (!col || !val || !rowidx_out || !cval_out)) || rowptr[m] != nnz)
        return SBLAS_ERR_INVALID;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SBLAS_ERR_NODEV;
    const int g = ngpu;
    // nnz-balanced whole-row blocks
    std::vector<int> rb(g + 1, m);
    rb[0] = 0;
    for (int d = 1; d < g; ++d) {
        const long long target = (long long)nnz * d / g;
        int lo = rb[d - 1], hi = m;  // first row r with rowptr[r] >= target
        while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (rowptr[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        rb[d] = lo;
    }
    struct Blk {
        int phys = 0;
        sblas_csr_s A;
        int *cp = nullptr, *ri = nullptr;
        double *cv = nullptr;
        hipStream_t s = nullptr;
    };
    std::vector<Blk> B(g);
    // one stream per physical device: blocks that wrap onto the same GPU run
    // in order (they share that device's transpose scratch)
    std::vector<hipStream_t> streams((size_t)std::min(count, g), nullptr);
    int *h_ptrs = nullptr, *h_base = nullptr, *h_rid = nullptr, *h_row0 = nullptr, *h_cp = nullptr,
        *h_ri = nullptr;
    double *h_val = nullptr, *h_cv = nullptr;
    long long *h_start = nullptr;
    hipStream_t s0 = nullptr;
    auto cleanup = [&]() {
        for (auto &b : B) {
            DeviceGuard gd(b.phys);
            (void)hipFree(b.A.rowptr);
            (void)hipFree(b.A.col);
            (void)hipFree(b.A.val);
            (void)hipFree(b.cp);
            (void)hipFree(b.ri);
            (void)hipFree(b.cv);
        }
        for (size_t p = 0; p < streams.size(); ++p)
            if (streams[p]) {
                DeviceGuard gd((int)p);
                (void)hipStreamDestroy(streams[p]);
            }
        DeviceGuard gd(0);
        for (void *p : {(void *)h_ptrs, (void *)h_base, (void *)h_rid, (void *)h_row0, (void *)h_cp,
                        (void *)h_ri, (void *)h_val, (void *)h_cv, (void *)h_start})
            (void)hipFree(p);
        if (s0) (void)hipStreamDestroy(s0);
    };
#define TG(expr)                                                               \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            set_error("csr2csc_mgpu: %s -> %s", #expr, hipGetErrorString(e_)); \
            cleanup();                                                         \
            return SBLAS_ERR_HIP;                                              \
        }                                                                      \
    } while (0)
    // upload the blocks
    std::vector<long long> start(g + 1, 0);
    for (int d = 0; d < g; ++d) {
        Blk &b = B[d];
        b.phys = d % count;
        DeviceGuard gd(b.phys);
        if (!streams[(size_t)b.phys]) TG(hipStreamCreateWithFlags(&streams[(size_t)b.phys], hipStreamNonBlocking));
        b.s = streams[(size_t)b.phys];
        const int r0 = rb[d], r1 = rb[d + 1];
        const int e0 = rowptr[r0], e1 = rowptr[r1];
        std::vector<int> lrp((size_t)(r1 - r0) + 1);
        for (int r = r0; r <= r1; ++r) lrp[(size_t)(r - r0)] = rowptr[r] - e0;
        b.A.device = b.phys;
        b.A.m = r1 - r0;
        b.A.n = n;
        b.A.nnz = e1 - e0;
        start[d + 1] = start[d] + (e1 - e0);
        TG(hipMalloc(&b.A.rowptr, sizeof(int) * lrp.size()));
        TG(hipMalloc(&b.A.col, sizeof(int) * std::max(e1 - e0, 1)));
        TG(hipMalloc(&b.A.val, sizeof(double) * std::max(e1 - e0, 1)));
        TG(hipMalloc(&b.cp, sizeof(int) * ((size_t)n + 1)));
        TG(hipMalloc(&b.ri, sizeof(int) * std::max(e1 - e0, 1)));
        TG(hipMalloc(&b.cv, sizeof(double) * std::max(e1 - e0, 1)));
        TG(hipMemcpy(b.A.rowptr, lrp.data(), sizeof(int) * lrp.size(), hipMemcpyHostToDevice));
        if (e1 > e0) {
            TG(hipMemcpy(b.A.col, col + e0, sizeof(int) * (e1 - e0), hipMemcpyHostToDevice));
            TG(hipMemcpy(b.A.val, val + e0, sizeof(double) * (e1 - e0), hipMemcpyHostToDevice));
        }
    }
    {
        DeviceGuard gd(0);
        TG(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
        TG(hipMalloc(&h_ptrs, sizeof(int) * (size_t)g * (n + 1)));
        TG(hipMalloc(&h_base, sizeof(int) * std::max<size_t>((size_t)g * n, 1)));
        TG(hipMalloc(&h_rid, sizeof(int) * std::max(nnz, 1)));
        TG(hipMalloc(&h_val, sizeof(double) * std::max(nnz, 1)));
        TG(hipMalloc(&h_row0, sizeof(int) * g));
        TG(hipMalloc(&h_start, sizeof(long long) * (g + 1)));
        TG(hipMalloc(&h_cp, sizeof(int) * ((size_t)n + 1)));
        TG(hipMalloc(&h_ri, sizeof(int) * std::max(nnz, 1)));
        TG(hipMalloc(&h_cv, sizeof(double) * std::max(nnz, 1)));
        TG(hipMemcpy(h_row0, rb.data(), sizeof(int) * g, hipMemcpyHostToDevice));
        TG(hipMemcpy(h_start, start.data(), sizeof(long long) * (g + 1), hipMemcpyHostToDevice));
    }
    for (int p = 0; p < std::min(count, g); ++p) {
        DeviceGuard gd(p);
        TG(hipDeviceSynchronize());
    }
    // 1) block transposes, concurrently on their devices
    const double t0 = sblas_get_time();
    for (int d = 0; d < g; ++d) {
        Blk &b = B[d];
        DeviceGuard gd(b.phys);
        const int st = launch_transpose(b.A, b.cp, b.ri, b.cv, b.s);
        if (st != SBLAS_OK) {
            cleanup();
            return st;
        }
    }
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(B[d].phys);
        TG(hipStreamSynchronize(B[d].s));
    }
    const double t1 = sblas_get_time();
    // 2) pieces to device 0 (peer DMA) and compose there
    {
        DeviceGuard gd(0);
        for (int d = 0; d < g; ++d) {
            const Blk &b = B[d];
            const long long k = start[d + 1] - start[d];
            TG(hipMemcpyPeerAsync(h_ptrs + (size_t)d * (n + 1), 0, b.cp, b.phys, sizeof(int) * ((size_t)n + 1), s0));
            if (k) {
                TG(hipMemcpyPeerAsync(h_rid + start[d], 0, b.ri, b.phys, sizeof(int) * k, s0));
                TG(hipMemcpyPeerAsync(h_val + start[d], 0, b.cv, b.phys, sizeof(double) * k, s0));
            }
        }
        hipLaunchKernelGGL(k_compose_ptr, dim3((n + 1 + 255) / 256), dim3(256), 0, s0, h_ptrs, g, n, h_cp,
                           h_base);
        if (nnz && n > 0)
            hipLaunchKernelGGL(k_compose_val, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s0, h_ptrs,
                               h_base, h_start, h_row0, g, n, (long long)nnz, h_rid, h_val, h_ri, h_cv);
        TG(hipGetLastError());
        TG(hipStreamSynchronize(s0));
    }
    const double t2 = sblas_get_time();
    if (ms_transpose) *ms_transpose = (t1 - t0) * 1e3;
    if (ms_compose) *ms_compose = (t2 - t1) * 1e3;
    {
        DeviceGuard gd(0);
        TG(hipMemcpy(colptr_out, h_cp, sizeof(int) * ((size_t)n + 1), hipMemcpyDeviceToHost));
        if (nnz) {
            TG(hipMemcpy(rowidx_out, h_ri, sizeof(int) * nnz, hipMemcpyDeviceToHost));
            TG(hipMemcpy(cval_out, h_cv, sizeof(double) * nnz, hipMemcpyDeviceToHost));
        }
    }
#undef TG
    cleanup();
    return SBLAS_OK;
}

namespace sblas {
}  // namespace sblas
