// capi.hip -- persistent device API of libsblas (include/sblas.h, layer 2).
#include <algorithm>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "sblas_internal.hpp"

namespace sblas {

int resolve_device(int ordinal, int *phys)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error("no HIP device available");
        return SBLAS_ERR_NODEV;
    }
    *phys = ordinal % count;
    return SBLAS_OK;
}

static int alloc_padded(sblas_csr_s &A, long long nnz)
{
    const long long cap = ((nnz + 3) & ~3LL) + 4;  // 16-B vector over-read pad
    SBLAS_HIP(hipMalloc(&A.col, sizeof(int) * cap));
    SBLAS_HIP(hipMalloc(&A.val, sizeof(double) * cap));
    SBLAS_HIP(hipMemset(A.col + nnz, 0, sizeof(int) * (cap - nnz)));
    SBLAS_HIP(hipMemset(A.val + nnz, 0, sizeof(double) * (cap - nnz)));
    SBLAS_HIP(hipMalloc(&A.rowptr, sizeof(int) * ((size_t)A.m + 1)));
    return SBLAS_OK;
}

}  // namespace sblas

using namespace sblas;

namespace sblas {
LaunchTimer &launch_timer()
{
    static thread_local LaunchTimer t;
    return t;
}

// Test hooks: planner overrides set through sblas_test_set_option (never
// from the environment), read when a plan is built.
namespace {
std::mutex g_opt_mu;
std::map<std::string, double> g_opt;
}  // namespace

bool test_option(const char *name, double *value)
{
    std::lock_guard<std::mutex> lk(g_opt_mu);
    auto it = g_opt.find(name);
    if (it == g_opt.end()) return false;
    if (value) *value = it->second;
    return true;
}

bool deterministic_default()
{
    static const bool on = [] {
        const char *e = getenv("SBLAS_DETERMINISTIC");
        return e && atoi(e) != 0;
    }();
    return on;
}
}  // namespace sblas

extern "C" {

int sblas_test_set_option(const char *name, double value, int set)
{
    if (!name) return SBLAS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(g_opt_mu);
    if (set) g_opt[name] = value;
    else g_opt.erase(name);
    return SBLAS_OK;
}

const char *sblas_status_string(int s)
{
    switch (s) {
    case SBLAS_OK: return "ok";
    case SBLAS_ERR_INVALID: return "invalid argument";
    case SBLAS_ERR_HIP: return "HIP runtime error";
    case SBLAS_ERR_NOMEM: return "insufficient device memory";
    case SBLAS_ERR_NODEV: return "no device";
    case SBLAS_ERR_UNSUPPORTED: return "unsupported";
    case SBLAS_ERR_RCCL: return "RCCL error";
    case SBLAS_ERR_IO: return "I/O error";
    default: return s == -1 ? "footprint exceeds 0.8 x free device memory" : "unknown";
    }
}

int sblas_version(void) { return 100; }

int sblas_device_count(int *count)
{
    if (!count) return SBLAS_ERR_INVALID;
    *count = 0;
    if (hipGetDeviceCount(count) != hipSuccess) {
        *count = 0;
        return SBLAS_ERR_NODEV;
    }
    return SBLAS_OK;
}

int sblas_csr_upload_slice(sblas_csr *out, int device, int n, const long long *rowptr,
                           const int *col, const double *val, int row_begin, int row_end,
                           long long idx_begin, long long idx_end, void *stream)
{
    if (!out || !rowptr || row_begin < 0 || row_end < row_begin || idx_end < idx_begin || n < 0)
        return SBLAS_ERR_INVALID;
    const long long dnnz = idx_end - idx_begin;
    if (dnnz >= (long long)std::numeric_limits<int>::max()) {
        set_error("local nnz %lld >= 2^31: partition across more devices", dnnz);
        return SBLAS_ERR_UNSUPPORTED;
    }
    int phys;
    SBLAS_TRY(resolve_device(device, &phys));
    DeviceGuard g(phys);
    hipStream_t s = (hipStream_t)stream;
    auto *A = new sblas_csr_s();
    A->device = phys;
    A->m = row_end - row_begin;
    A->n = n;
    A->nnz = dnnz;
    A->h_rowptr.resize((size_t)A->m + 1);
    // local int32 rowptr: [0]=0, [m]=dnnz, middle rebased (dspmv_mgpu_v1.cu:125-133)
    A->h_rowptr[0] = 0;
    if (A->m > 0) A->h_rowptr[(size_t)A->m] = (int)dnnz;
    for (int j = 1; j < A->m; ++j) A->h_rowptr[(size_t)j] = (int)(rowptr[row_begin + j] - idx_begin);
    int st = alloc_padded(*A, dnnz);
    if (st != SBLAS_OK) {
        sblas_csr_destroy(A);
        return st;
    }
#define UP_CHECK(expr)                                                         \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            set_error("%s -> %s", #expr, hipGetErrorString(e_));               \
            sblas_csr_destroy(A);                                              \
            return SBLAS_ERR_HIP;                                              \
        }                                                                      \
    } while (0)
    UP_CHECK(hipMemcpyAsync(A->rowptr, A->h_rowptr.data(), sizeof(int) * ((size_t)A->m + 1),
                            hipMemcpyHostToDevice, s));
    if (dnnz) {
        UP_CHECK(hipMemcpyAsync(A->col, col + idx_begin, sizeof(int) * dnnz, hipMemcpyHostToDevice, s));
        UP_CHECK(hipMemcpyAsync(A->val, val + idx_begin, sizeof(double) * dnnz, hipMemcpyHostToDevice, s));
    }
    UP_CHECK(hipStreamSynchronize(s));
#undef UP_CHECK
    *out = A;
    return SBLAS_OK;
}

int sblas_csr_from_device(sblas_csr *out, int device, int m, int n, int nnz, const int *d_rowptr,
                          const int *d_col, const double *d_val, void *stream)
{
    if (!out || m < 0 || n < 0 || nnz < 0 || !d_rowptr) return SBLAS_ERR_INVALID;
    int phys;
    SBLAS_TRY(resolve_device(device, &phys));
    DeviceGuard g(phys);
    hipStream_t s = (hipStream_t)stream;
    auto *A = new sblas_csr_s();
    A->device = phys;
    A->m = m;
    A->n = n;
    A->nnz = nnz;
    int st = alloc_padded(*A, nnz);
    if (st == SBLAS_OK) {
        A->h_rowptr.resize((size_t)m + 1);
        hipError_t e = hipMemcpyAsync(A->rowptr, d_rowptr, sizeof(int) * ((size_t)m + 1),
                                      hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && nnz)
            e = hipMemcpyAsync(A->col, d_col, sizeof(int) * (size_t)nnz, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess && nnz)
            e = hipMemcpyAsync(A->val, d_val, sizeof(double) * (size_t)nnz, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(A->h_rowptr.data(), d_rowptr, sizeof(int) * ((size_t)m + 1),
                               hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            set_error("sblas_csr_from_device: %s", hipGetErrorString(e));
            st = SBLAS_ERR_HIP;
        }
    }
    if (st != SBLAS_OK) {
        sblas_csr_destroy(A);
        return st;
    }
    if (A->h_rowptr[0] != 0 || A->h_rowptr[(size_t)m] != nnz) {
        sblas_csr_destroy(A);
        set_error("rowptr must start at 0 and end at nnz");
        return SBLAS_ERR_INVALID;
    }
    *out = A;
    return SBLAS_OK;
}

int sblas_csr_destroy(sblas_csr A)
{
    if (!A) return SBLAS_OK;
    {
        DeviceGuard g(A->device);
        free_plans(*A);
        (void)hipFree(A->spmm_bt);
        (void)hipFree(A->spmm_part);
        (void)hipFree(A->rowptr);
        (void)hipFree(A->col);
        (void)hipFree(A->val);
    }
    delete A;
    return SBLAS_OK;
}

int sblas_csr_info(sblas_csr A, int *m, int *n, long long *nnz)
{
    if (!A) return SBLAS_ERR_INVALID;
    if (m) *m = A->m;
    if (n) *n = A->n;
    if (nnz) *nnz = A->nnz;
    return SBLAS_OK;
}

namespace {
// SBLAS_SPMV_AUTO's locality probe: one wave per sampled row (rows
// w*m/S, S <= 65536), at most its first 1024 entries; counts the entries
// whose column lies within 16 columns (one 128-B line of x) of the previous
// entry's -- for a row's first entry, the previous row's last (lanes of the
// row split read neighbouring rows together, so a diagonal counts as local).
// cnt = {adjacent, counted, then the sampled entries per eighth of the
// columns [k*n/8, (k+1)*n/8): how evenly the x gathers would spread over the
// XCDs' column groups of the column-sorted kernel}.
constexpr int kProbeWords = 12;  // adjacent, counted, 8 eighths, scattered rows, sampled rows
__global__ __launch_bounds__(256) void k_col_adjacency(const int *__restrict__ rowptr,
                                                       const int *__restrict__ col, int m, int n, int S,
                                                       unsigned long long *cnt)
{
    const int w = (int)(blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    const int lane = threadIdx.x & 63;
    // waves past S count nothing (no early return: the block reduces below)
    const int r = w < S ? (int)((long long)w * m / S) : 0;
    const int a = w < S ? rowptr[r] : 0;
    const int b = w < S ? min(rowptr[r + 1], a + 1024) : 0;
    unsigned adj = 0, tot = 0, h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int cmin = 0x7fffffff, cmax = -1;
    for (int e = a + lane; e < b; e += 64) {
        const int c = col[e];
        cmin = min(cmin, c);
        cmax = max(cmax, c);
        const int k = (int)min(7LL, max(0LL, (long long)c * 8 / max(n, 1)));
#pragma unroll
        for (int q = 0; q < 8; ++q) h[q] += q == k ? 1u : 0u;
        if (e >= 1) {
            const int d = c - col[e - 1];
            adj += (d > -16 && d < 16) ? 1u : 0u;
            ++tot;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        adj += __shfl_down(adj, o, 64);
        tot += __shfl_down(tot, o, 64);
        cmin = min(cmin, __shfl_down(cmin, o, 64));
        cmax = max(cmax, __shfl_down(cmax, o, 64));
#pragma unroll
        for (int q = 0; q < 8; ++q) h[q] += __shfl_down(h[q], o, 64);
    }
    // a row whose columns span more than a quarter of x ("scattered": its
    // gathers cannot stay in one XCD's share of x)
    const unsigned wide = (w < S && b > a && (long long)(cmax - cmin) * 4 > (long long)n) ? 1u : 0u;
    const unsigned sampled = (w < S && b > a) ? 1u : 0u;
    // one partial per workgroup (its waves' sums added in LDS), stored plainly
    // to part[blockIdx.x][10]; the host adds them (no memory-side atomics on
    // ten shared words, which serialised the probe to ~5 ms on config 2)
    __shared__ unsigned s_c[4][kProbeWords];
    const int wv = (int)(threadIdx.x / 64);
    if (lane == 0) {
        s_c[wv][0] = adj;
        s_c[wv][1] = tot;
#pragma unroll
        for (int q = 0; q < 8; ++q) s_c[wv][2 + q] = h[q];
        s_c[wv][10] = wide;
        s_c[wv][11] = sampled;
    }
    __syncthreads();
    if (threadIdx.x < kProbeWords) {
        unsigned long long v = 0;
        for (int k = 0; k < (int)(blockDim.x / 64); ++k) v += s_c[k][threadIdx.x];
        cnt[(size_t)blockIdx.x * kProbeWords + threadIdx.x] = v;
    }
}

constexpr long long kAutoXsortMinNnz = 2000000;  // bench slices: xsort leads from ~2M nnz

}  // namespace

extern "C++" {
namespace sblas {
// The column-locality probe (k_col_adjacency), run once per handle: fills
// A.col_adjacency and A.col_maxshare.  Used by AUTO (pick_algo) and by the
// CSR5 plan's panel choice (spmv.hip).
int probe_columns(sblas_csr_s &A, hipStream_t s)
{
    if (A.col_adjacency >= 0.0) return SBLAS_OK;
    double adj = 0.0, share = 0.0;
    const int S = (int)std::min<long long>(A.m, 65536);
    if (S > 0 && A.nnz > 1) {
        const int nb = (S + 3) / 4;
        std::vector<unsigned long long> part((size_t)nb * kProbeWords);
        unsigned long long *d = nullptr;
        hipError_t e = hipMalloc(&d, sizeof(unsigned long long) * part.size());
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_col_adjacency, dim3(nb), dim3(256), 0, s, A.rowptr, A.col, A.m, A.n, S, d);
            e = hipGetLastError();
        }
        if (e == hipSuccess)
            e = hipMemcpyAsync(part.data(), d, sizeof(unsigned long long) * part.size(), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (d) (void)hipFree(d);
        if (e != hipSuccess) {
            set_error("column probe: %s", hipGetErrorString(e));
            return SBLAS_ERR_HIP;
        }
        unsigned long long h[kProbeWords] = {};
        for (int b = 0; b < nb; ++b)
            for (int q = 0; q < kProbeWords; ++q) h[q] += part[(size_t)b * kProbeWords + q];
        A.col_scattered = h[11] ? (double)h[10] / (double)h[11] : 0.0;
        adj = h[1] ? (double)h[0] / (double)h[1] : 0.0;
        unsigned long long hs = 0, hm = 0;
        for (int q = 0; q < 8; ++q) {
            hs += h[2 + q];
            hm = std::max(hm, h[2 + q]);
        }
        share = hs ? (double)hm / (double)hs : 1.0;
    }
    A.col_adjacency = adj;
    A.col_maxshare = share;
    return SBLAS_OK;
}
}  // namespace sblas
}  // extern "C++"

namespace {

int pick_algo(sblas_csr_s &A, hipStream_t s)
{
    if (A.auto_algo) return A.auto_algo;
    if (const int st = probe_columns(A, s)) return -st;
    const double adj = A.col_adjacency, share = A.col_maxshare;
    // The column-sorted kernel wherever it applies at size and its column
    // groups share the work: it leads on random columns (config 2: 0.51 of
    // 8 TB/s vs 0.21 row split) and on banded / stencil matrices too (3-D
    // 27-point stencil 0.84 vs 0.55, 7-point 0.71 vs 0.58), but
    // columns crowded into one eighth (the reference generator's prefix
    // columns) leave one XCD all of it: the row split there (0.68), as for
    // any matrix whose rows read neighbouring x lines; the XCD-panel row
    // split below 2M nonzeros.
    const bool spread = share <= 0.25;  // no eighth of the columns holds > 2x its share
    int algo;
    if (A.nnz >= kAutoXsortMinNnz && (long long)A.n * 8 <= (120LL << 20) && spread) algo = SBLAS_SPMV_XSORT;
    else if (adj >= 0.5 || !spread) algo = SBLAS_SPMV_ROWSPLIT;
    else algo = SBLAS_SPMV_PANEL;
    if (const char *o = getenv("SBLAS_AUTO")) {
        const int v = atoi(o);
        if (v >= SBLAS_SPMV_ROWSPLIT && v <= SBLAS_SPMV_XSORT) algo = v;
    }
    A.auto_algo = algo;
    return algo;
}

// algo, or AUTO resolved (negative: -status)
int resolve_algo(sblas_csr_s &A, int algo, hipStream_t s)
{
    return algo == SBLAS_SPMV_AUTO ? pick_algo(A, s) : algo;
}

bool plan_ready(const sblas_csr_s &A, int algo)
{
    switch (algo) {
    case SBLAS_SPMV_ROWSPLIT: return A.rs.ready;
    case SBLAS_SPMV_CSR5:
    case SBLAS_SPMV_CSR5_ALT: return A.c5.ready;
    case SBLAS_SPMV_PANEL: return A.pn.ready;
    case SBLAS_SPMV_XSORT: return A.xs.ready;
    default: return false;
    }
}
} // namespace

int sblas_csr_set_deterministic(sblas_csr A, int on)
{
    if (!A) return SBLAS_ERR_INVALID;
    A->deterministic = on != 0;
    return SBLAS_OK;
}

int sblas_csr_get_deterministic(sblas_csr A, int *on)
{
    if (!A || !on) return SBLAS_ERR_INVALID;
    *on = A->deterministic ? 1 : 0;
    return SBLAS_OK;
}

int sblas_csr_xsort_info(sblas_csr A, long long *info)
{
    if (!A || !info) return SBLAS_ERR_INVALID;
    const XsPlan &P = A->xs;
    const long long v[8] = {P.ready ? 1 : 0, P.nranges, P.nwide, P.nitems, P.grid, P.solo ? 1 : 0, P.nchunks,
                            P.maxc};
    for (int i = 0; i < 8; ++i) info[i] = v[i];
    return SBLAS_OK;
}

int sblas_csr_pick(sblas_csr A, void *stream, int *algo)
{
    if (!A || !algo) return SBLAS_ERR_INVALID;
    DeviceGuard g(A->device);
    const int a = pick_algo(*A, (hipStream_t)stream);
    if (a < 0) return -a;
    *algo = a;
    return SBLAS_OK;
}

int sblas_csr_analyse(sblas_csr A, int algo, void *stream)
{
    if (!A) return SBLAS_ERR_INVALID;
    DeviceGuard g(A->device);
    hipStream_t s = (hipStream_t)stream;
    const bool auto_pick = algo == SBLAS_SPMV_AUTO;
    algo = resolve_algo(*A, algo, s);
    if (algo < 0) return -algo;
    if (algo < SBLAS_SPMV_ROWSPLIT || algo > SBLAS_SPMV_XSORT) return SBLAS_ERR_INVALID;
    if (auto_pick && algo == SBLAS_SPMV_XSORT) {
        const int st = sblas_csr_analyse(A, SBLAS_SPMV_XSORT, stream);
        if (st != SBLAS_ERR_UNSUPPORTED) return st;
        A->auto_algo = SBLAS_SPMV_PANEL;  // the column groups do not apply to this matrix
        algo = SBLAS_SPMV_PANEL;
    }
    // device bytes the plan holds: free memory before - after (the builders
    // synchronise before returning)
    size_t f0 = 0, f1 = 0, tot = 0;
    (void)hipMemGetInfo(&f0, &tot);
    int st = SBLAS_ERR_INVALID;
    switch (algo) {
    case SBLAS_SPMV_ROWSPLIT: st = build_rowsplit_plan(*A, s); break;
    case SBLAS_SPMV_CSR5:
    case SBLAS_SPMV_CSR5_ALT: st = build_csr5_plan(*A, s); break;
    case SBLAS_SPMV_PANEL: st = build_panel_plan(*A, s); break;
    case SBLAS_SPMV_XSORT: st = build_xsort_plan(*A, s); break;
    }
    if (st == SBLAS_OK && A->plan_bytes[algo] == 0 && hipMemGetInfo(&f1, &tot) == hipSuccess && f0 > f1)
        A->plan_bytes[algo] = (long long)(f0 - f1);
    return st;
}

int sblas_csr_panels(sblas_csr A, int algo, int *panels)
{
    if (!A || !panels) return SBLAS_ERR_INVALID;
    switch (algo) {
    case SBLAS_SPMV_ROWSPLIT: *panels = A->rs.ready && A->rs.panels ? A->pn.P : 0; break;
    case SBLAS_SPMV_CSR5:
    case SBLAS_SPMV_CSR5_ALT: *panels = A->c5.ready ? A->c5.P : 0; break;
    case SBLAS_SPMV_PANEL: *panels = A->pn.ready && !A->pn.degenerate ? A->pn.P : 0; break;
    default: *panels = 0; break;
    }
    return SBLAS_OK;
}

long long sblas_csr_plan_bytes(sblas_csr A, int algo)
{
    if (!A || algo < 0 || algo > SBLAS_SPMV_XSORT) return -1;
    return A->plan_bytes[algo];
}

int sblas_spmv(sblas_csr A, int algo, double alpha, const double *d_x, double beta, double *d_y,
               void *stream)
{
    if (!A || (!d_x && A->nnz) || (!d_y && A->m)) return SBLAS_ERR_INVALID;
    DeviceGuard g(A->device);
    hipStream_t s = (hipStream_t)stream;
    if (algo == SBLAS_SPMV_AUTO) {  // resolve (and analyse, with its fallback) once
        if (!A->auto_algo || !plan_ready(*A, A->auto_algo)) SBLAS_TRY(sblas_csr_analyse(A, SBLAS_SPMV_AUTO, stream));
        algo = A->auto_algo;
    }
    switch (algo) {
    case SBLAS_SPMV_ROWSPLIT:
        if (!A->rs.ready) SBLAS_TRY(build_rowsplit_plan(*A, s));
        return launch_spmv_rowsplit(*A, alpha, d_x, beta, d_y, s);
    case SBLAS_SPMV_CSR5:
    case SBLAS_SPMV_CSR5_ALT:
        if (!A->c5.ready) SBLAS_TRY(build_csr5_plan(*A, s));
        return launch_spmv_csr5(*A, alpha, d_x, beta, d_y, s);
    case SBLAS_SPMV_PANEL:
        if (!A->pn.ready) SBLAS_TRY(build_panel_plan(*A, s));
        return launch_spmv_panel(*A, alpha, d_x, beta, d_y, s);
    case SBLAS_SPMV_XSORT:
        if (!A->xs.ready) SBLAS_TRY(build_xsort_plan(*A, s));
        return launch_spmv_xsort(*A, alpha, d_x, beta, d_y, s);
    default: return SBLAS_ERR_INVALID;
    }
}

// y = alpha*A*x + beta*y with the call's device span measured: every kernel
// of the call goes through hipExtLaunchKernelGGL with events stamped at the
// first kernel's start and at the last kernel's end (SBLAS_LAUNCH), then the
// call waits for the stop event.  ms = 0 when the call launches nothing.
int sblas_spmv_timed(sblas_csr A, int algo, double alpha, const double *d_x, double beta, double *d_y,
                     void *stream, float *ms)
{
    if (!A || !ms) return SBLAS_ERR_INVALID;
    DeviceGuard g(A->device);
    // build any plan first, untimed (the plan build launches its own kernels)
    hipStream_t s = (hipStream_t)stream;
    if (algo == SBLAS_SPMV_AUTO) {  // resolve (and analyse, with its fallback) once
        if (!A->auto_algo || !plan_ready(*A, A->auto_algo)) SBLAS_TRY(sblas_csr_analyse(A, SBLAS_SPMV_AUTO, stream));
        algo = A->auto_algo;
    }
    switch (algo) {
    case SBLAS_SPMV_ROWSPLIT: if (!A->rs.ready) SBLAS_TRY(build_rowsplit_plan(*A, s)); break;
    case SBLAS_SPMV_CSR5:
    case SBLAS_SPMV_CSR5_ALT: if (!A->c5.ready) SBLAS_TRY(build_csr5_plan(*A, s)); break;
    case SBLAS_SPMV_PANEL: if (!A->pn.ready) SBLAS_TRY(build_panel_plan(*A, s)); break;
    case SBLAS_SPMV_XSORT: if (!A->xs.ready) SBLAS_TRY(build_xsort_plan(*A, s)); break;
    default: return SBLAS_ERR_INVALID;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    SBLAS_HIP(hipEventCreate(&e0));
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        set_error("sblas_spmv_timed: hipEventCreate failed");
        return SBLAS_ERR_HIP;
    }
    LaunchTimer &lt = launch_timer();
    lt.start = e0;
    lt.stop = e1;
    lt.pending_start = true;
    int rc = sblas_spmv(A, algo, alpha, d_x, beta, d_y, stream);
    const bool launched = !lt.pending_start;
    lt = LaunchTimer{};
    *ms = 0.0f;
    hipError_t e = hipSuccess;
    if (rc == SBLAS_OK && launched) {
        e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(ms, e0, e1);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc != SBLAS_OK) return rc;
    if (e != hipSuccess) {
        set_error("sblas_spmv_timed: %s", hipGetErrorString(e));
        return SBLAS_ERR_HIP;
    }
    return SBLAS_OK;
}

// Compulsory traffic: each array touched once.
long long sblas_spmv_algorithmic_bytes(sblas_csr A, int beta_nonzero)
{
    if (!A) return 0;
    return A->nnz * 12LL + ((long long)A->m + 1) * 4LL + (long long)A->n * 8LL +
           (long long)A->m * 8LL + (beta_nonzero ? (long long)A->m * 8LL : 0LL);
}

int sblas_spmm(sblas_csr A, int n, double alpha, const double *d_B, int ldb, int b_layout,
               double beta, double *d_C, int ldc, void *stream)
{
    if (!A || n < 0 || (b_layout != 0 && b_layout != 1)) return SBLAS_ERR_INVALID;
    if (b_layout == 0 && ldb < A->n) return SBLAS_ERR_INVALID;
    if (b_layout == 1 && ldb < n) return SBLAS_ERR_INVALID;
    if (ldc < A->m) return SBLAS_ERR_INVALID;
    DeviceGuard g(A->device);
    if (!A->mm.ready) SBLAS_TRY(build_spmm_plan(*A, n, (hipStream_t)stream));
    return launch_spmm(*A, n, alpha, d_B, ldb, b_layout, beta, d_C, ldc, (hipStream_t)stream);
}

int sblas_csr_transpose(sblas_csr A, int *d_colptr, int *d_rowidx, double *d_cval, void *stream)
{
    if (!A || !d_colptr) return SBLAS_ERR_INVALID;
    DeviceGuard g(A->device);
    return launch_transpose(*A, d_colptr, d_rowidx, d_cval, (hipStream_t)stream);
}

}  // extern "C"
