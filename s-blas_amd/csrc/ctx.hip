// ctx.hip -- single-process multi-GPU SpMV context over RCCL (include/sblas.h
// "3. Multi-GPU context").
//
// Replaces the reference's host-driven multi-GPU SpMV (spmv/src/
// dspmv_mgpu_v1.cu:16-280: per-call H2D of every slice, csrmv per GPU, D2H
// and a host merge of the split rows, :224-248) for C/C++ callers that keep
// the matrix: ONE process drives g GPUs, each GPU keeps its slice resident,
// x is replicated with ncclBroadcast, and after the per-device kernels the y
// slices are exchanged with ONE ncclAllGather over xGMI and placed by a
// device kernel, so every GPU ends with the full, bit-identical y (SURVEY §5
// "Distributed communication backend", §8 G1).  The communicator comes from
// ncclCommInitAll over the context's devices.
//
// Partitions: 0 = cyclic row chunks (chunk j of ceil(m / (g*8)) rows on
// device j % g, whole rows, equal padded slices: no split rows, no carries;
// sblas_dist.CyclicPlan is the same distribution for one-process-per-GPU
// runs); 1 = spMV_mgpu_v1's nnz-balanced split (dspmv_mgpu_v1.cu:60-94, Q5
// fixed) with the split rows added in partition order on the device
// (k_assemble_carry).
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

#include "sblas_internal.hpp"

struct sblas_ctx_s {
    int g = 0;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;  // [g][3]: start, after kernel, after exchange + placement
    // the matrix (absent until sblas_ctx_matrix_upload)
    bool loaded = false;
    int m = 0, n = 0, algo = 0, partition = 0, exchange = 0;
    long long nnz = 0, stride = 0, chunk_rows = 0;
    long long ylen = 0;                // doubles in each ylocal buffer
    std::vector<sblas_csr> A;
    std::vector<double *> x, ylocal, gathered, yfull;
    std::vector<int *> meta;           // nnz partition: {row0, nrows, cont} per partition
    std::vector<int> h_meta;
    std::vector<double *> bar;         // one word per device: the timing protocol's aligning all-reduce
    std::vector<long long> lrows;      // rows per device
    std::vector<long long> lnnz;       // entries per device
    std::vector<long long> yoff;       // the kernel's y = ylocal[d] + yoff[d]
    std::vector<double> last;          // stats of the last sblas_ctx_spmv_ex (3 + 3g)
    bool pending = false;              // a step was issued without waiting (wait = 0)
    // loopback rehearsal (SBLAS_CTX_LOOPBACK=1): ranks may share a GPU, no
    // communicator; the collectives are stream-ordered device copies / sums
    bool loopback = false;
    std::vector<hipEvent_t> evx, evy;  // [g] cross-stream sync events
    std::vector<const double **> yptr; // allreduce: per device, the g send buffers
    // overlapped exchange (cyclic partition + all-gather, parts > 1): each
    // device's local chunks cut into `parts` consecutive groups, each its own
    // handle; part p's all-gather + placement run on the device's comm stream
    // while the kernel of part p + 1 runs on the main stream
    // (dspmv_mgpu_v2.cu:128-170's per-task copies overlapping compute)
    int parts = 1;
    std::vector<long long> plo;        // [parts + 1] local chunk bounds of the parts
    std::vector<sblas_csr> P;          // [g * parts] part handles (device-major)
    std::vector<hipStream_t> cst;      // [g] comm streams
    std::vector<hipEvent_t> evp;       // [g * parts] part kernel done (main stream)
    std::vector<int> evp_dev;          // [g * parts] the device each evp event was created on
    std::vector<hipEvent_t> evc;       // [g] comm stream done (joins the main stream)
    std::vector<int> palgo;            // [g] the algorithm the part handles run (AUTO resolved)
    int parts_req = 1;                 // requested by sblas_ctx_matrix_upload_parts
    // one device, one part: nothing to exchange; yfull[0] IS ylocal[0] (its
    // first m rows are y in row order under either partition)
    bool yalias = false;
    // SBLAS_CTX_NOALIAS=1 (read once, at sblas_ctx_create): a one-device
    // context still runs the exchange (ncclAllGather + placement, or
    // ncclAllReduce + re-prime) on its 1-rank communicator, so the
    // collectives execute on a one-GPU box
    bool noalias = false;
    // loopback all-reduce: peer access this context enabled (a -> b), undone on destroy
    std::vector<std::pair<int, int>> peers;
};

// Per-row weight of the cost-weighted partition (2): a row end costs the
// CSR5 segmented-sum kernel (over 4 XCD panels) about 3 entries' time --
// configs[2]'s N = 8 ranks of the uniform config 2 at equal nnz: 552k light
// rows 60 us, 52k heavy rows 46 us (profiles/r05/c5P/), i.e. ~9 us per M
// entries + ~28 us per M rows.
constexpr double kCtxRowCost = 3.0;

// Bound context for the reference API: spMV_mgpu_v1 with ngpu == the bound
// context's size runs on it (device-resident slices for the call, x
// broadcast, kernels, ncclAllGather, device merge) instead of the per-device
// host merge.  Process-global, as the reference's device state is.
namespace sblas {
static sblas_ctx g_bound = nullptr;
sblas_ctx bound_ctx() { return g_bound; }

namespace {
struct PeerLink {
    int refs = 0;
    bool owned = false;  // enabled by the library (disabled at the last release)
};
std::mutex g_peer_mu;
std::map<std::pair<int, int>, PeerLink> g_peer;
bool g_peer_deny = false;
}  // namespace

bool peer_denied() { return g_peer_deny; }

int peer_acquire(int a, int b, const char *who)
{
    std::lock_guard<std::mutex> lk(g_peer_mu);
    if (g_peer_deny) {
        set_error("%s: peer access %d -> %d refused (sblas_test_deny_peer_access)", who, a, b);
        return SBLAS_ERR_UNSUPPORTED;
    }
    auto it = g_peer.find({a, b});
    if (it == g_peer.end()) {  // first user: enable the link
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) {
            (void)hipGetLastError();
            set_error("%s: no peer access between devices %d and %d", who, a, b);
            return SBLAS_ERR_UNSUPPORTED;
        }
        DeviceGuard g(a);
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        PeerLink L;
        if (e == hipErrorPeerAccessAlreadyEnabled) {  // enabled outside the library: use, never disable
            (void)hipGetLastError();
            L.owned = false;
        } else if (e != hipSuccess) {
            set_error("%s: hipDeviceEnablePeerAccess(%d -> %d): %s", who, a, b, hipGetErrorString(e));
            return SBLAS_ERR_HIP;
        } else {
            L.owned = true;
        }
        it = g_peer.emplace(std::make_pair(a, b), L).first;
    }
    ++it->second.refs;
    return SBLAS_OK;
}

void peer_release(int a, int b)
{
    std::lock_guard<std::mutex> lk(g_peer_mu);
    auto it = g_peer.find({a, b});
    if (it == g_peer.end() || it->second.refs <= 0) return;
    if (--it->second.refs == 0) {
        if (it->second.owned) {
            DeviceGuard g(a);
            (void)hipDeviceDisablePeerAccess(b);
            (void)hipGetLastError();
        }
        g_peer.erase(it);
    }
}
}  // namespace sblas

extern "C" int sblas_test_deny_peer_access(int on)
{
    std::lock_guard<std::mutex> lk(sblas::g_peer_mu);
    sblas::g_peer_deny = on != 0;
    return SBLAS_OK;
}

extern "C" int sblas_peer_refs(int a, int b)
{
    std::lock_guard<std::mutex> lk(sblas::g_peer_mu);
    auto it = sblas::g_peer.find({a, b});
    return it == sblas::g_peer.end() ? 0 : it->second.refs;
}

namespace {

using namespace sblas;

#define SBLAS_NCCL(expr)                                                        \
    do {                                                                        \
        ncclResult_t r_ = (expr);                                               \
        if (r_ != ncclSuccess) {                                                \
            ::sblas::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,     \
                               ncclGetErrorString(r_));                         \
            return SBLAS_ERR_RCCL;                                              \
        }                                                                       \
    } while (0)

// Inside ncclGroupStart/End: on failure close the group before returning, so
// the calling thread's later collectives are not queued into a group that
// never runs.
#define SBLAS_NCCL_G(expr)                                                      \
    do {                                                                        \
        ncclResult_t r_ = (expr);                                               \
        if (r_ != ncclSuccess) {                                                \
            (void)ncclGroupEnd();                                               \
            ::sblas::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,     \
                               ncclGetErrorString(r_));                         \
            return SBLAS_ERR_RCCL;                                              \
        }                                                                       \
    } while (0)

// Timing aid of sblas_ctx_spmv_ex: hold the stream for `ticks` of the 100-MHz
// constant clock, so that the host can enqueue every device's step before any
// device starts it (the host's launch latency then stays out of the spans).
__global__ void k_ctx_delay(unsigned long long ticks)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// allreduce exchange: after the sum, the device's own rows of the full y
// become its next input (a continuation row restarts from 0: the previous
// partition adds beta*y for it).
__global__ void k_ctx_reprime(const double *__restrict__ yfull, double *__restrict__ ysend, long long nr,
                              int cont)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nr) return;
    ysend[i] = (i == 0 && cont) ? 0.0 : yfull[i];
}

// loopback allreduce: dst = sum of the g send buffers, in rank order
__global__ void k_ctx_sum(const double *const *__restrict__ src, int g, long long m, double *__restrict__ dst)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    double s = 0.0;
    for (int r = 0; r < g; ++r) s += src[r][i];
    dst[i] = s;
}

// loopback: every stream waits for everything issued so far on every stream
int lb_barrier(sblas_ctx_s &C, std::vector<hipEvent_t> &ev)
{
    for (int d = 0; d < C.g; ++d) {
        DeviceGuard gd(C.dev[d]);
        SBLAS_HIP(hipEventRecord(ev[d], C.st[d]));
    }
    for (int d = 0; d < C.g; ++d) {
        DeviceGuard gd(C.dev[d]);
        for (int e = 0; e < C.g; ++e)
            if (e != d) SBLAS_HIP(hipStreamWaitEvent(C.st[d], ev[e], 0));
    }
    return SBLAS_OK;
}

// x from device 0 to every device (ncclBroadcast)
int xchg_broadcast_x(sblas_ctx_s &C)
{
    if (!C.loopback) {
        SBLAS_NCCL(ncclGroupStart());
        for (int d = 0; d < C.g; ++d) {
            DeviceGuard g(C.dev[d]);
            SBLAS_NCCL_G(ncclBroadcast(C.x[d], C.x[d], (size_t)C.n, ncclDouble, 0, C.comm[d], C.st[d]));
        }
        SBLAS_NCCL(ncclGroupEnd());
        return SBLAS_OK;
    }
    SBLAS_TRY(lb_barrier(C, C.evx));
    for (int d = 1; d < C.g; ++d) {
        DeviceGuard g(C.dev[d]);
        SBLAS_HIP(hipMemcpyAsync(C.x[d], C.x[0], sizeof(double) * C.n, hipMemcpyDeviceToDevice, C.st[d]));
    }
    return lb_barrier(C, C.evy);
}

// the timing protocol's aligning one-word all-reduce
int xchg_barrier(sblas_ctx_s &C)
{
    if (!C.loopback) {
        SBLAS_NCCL(ncclGroupStart());
        for (int d = 0; d < C.g; ++d) {
            DeviceGuard gd(C.dev[d]);
            SBLAS_NCCL_G(ncclAllReduce(C.bar[d], C.bar[d], 1, ncclDouble, ncclSum, C.comm[d], C.st[d]));
        }
        SBLAS_NCCL(ncclGroupEnd());
        return SBLAS_OK;
    }
    return lb_barrier(C, C.evx);
}

// the step's exchange: all-gather of the padded slices or all-reduce of the
// zero-padded y
int xchg_spmv(sblas_ctx_s &C)
{
    const int g = C.g;
    if (!C.loopback) {
        SBLAS_NCCL(ncclGroupStart());
        for (int d = 0; d < g; ++d) {
            DeviceGuard gd(C.dev[d]);
            if (C.exchange == SBLAS_CTX_ALLGATHER)  // one all-gather of equal padded slices over xGMI
                SBLAS_NCCL_G(ncclAllGather(C.ylocal[d], C.gathered[d], (size_t)C.stride, ncclDouble, C.comm[d],
                                           C.st[d]));
            else  // BASELINE configs[2]: the literal all-reduce of the zero-padded y
                SBLAS_NCCL_G(ncclAllReduce(C.ylocal[d], C.yfull[d], (size_t)C.m, ncclDouble, ncclSum, C.comm[d],
                                           C.st[d]));
        }
        SBLAS_NCCL(ncclGroupEnd());
        return SBLAS_OK;
    }
    SBLAS_TRY(lb_barrier(C, C.evx));  // every slice written
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C.dev[d]);
        if (C.exchange == SBLAS_CTX_ALLGATHER) {
            for (int r = 0; r < g; ++r)
                SBLAS_HIP(hipMemcpyAsync(C.gathered[d] + (size_t)r * C.stride, C.ylocal[r], sizeof(double) * C.stride,
                                         hipMemcpyDeviceToDevice, C.st[d]));
        } else if (C.m > 0) {
            hipLaunchKernelGGL(k_ctx_sum, dim3((unsigned)((C.m + 255) / 256)), dim3(256), 0, C.st[d], C.yptr[d], g,
                               (long long)C.m, C.yfull[d]);
            SBLAS_HIP(hipGetLastError());
        }
    }
    return lb_barrier(C, C.evy);  // every slice read before any is re-primed
}

// overlapped form, part p: rows of global chunks [plo[p]*g, plo[p+1]*g)
struct PartGeom {
    long long stride;  // rows of one device's (padded) part slice
    long long lrow0;   // first local row of the part on every device
    long long grow0;   // first global row of the part
    long long rows;    // global rows of the part
};

PartGeom part_geom(const sblas_ctx_s &C, int p)
{
    const long long R = C.chunk_rows, g = C.g;
    PartGeom q;
    q.stride = (C.plo[p + 1] - C.plo[p]) * R;
    q.lrow0 = C.plo[p] * R;
    q.grow0 = std::min<long long>(C.m, C.plo[p] * g * R);
    q.rows = std::min<long long>(C.m, C.plo[p + 1] * g * R) - q.grow0;
    return q;
}

// part p's exchange on the comm streams (each first waits for every
// device's part-p kernel when in loopback, for its own under RCCL): one
// all-gather of the part slices, then their placement into yfull
int xchg_part(sblas_ctx_s &C, int p)
{
    const int g = C.g;
    const PartGeom q = part_geom(C, p);
    if (!C.loopback) {
        for (int d = 0; d < g; ++d) {
            DeviceGuard gd(C.dev[d]);
            SBLAS_HIP(hipStreamWaitEvent(C.cst[d], C.evp[(size_t)d * C.parts + p], 0));
        }
        if (q.stride > 0) {
            SBLAS_NCCL(ncclGroupStart());
            for (int d = 0; d < g; ++d) {
                DeviceGuard gd(C.dev[d]);
                SBLAS_NCCL_G(ncclAllGather(C.ylocal[d] + q.lrow0, C.gathered[d] + (size_t)g * q.lrow0,
                                           (size_t)q.stride, ncclDouble, C.comm[d], C.cst[d]));
            }
            SBLAS_NCCL(ncclGroupEnd());
        }
    } else {
        for (int d = 0; d < g; ++d) {
            DeviceGuard gd(C.dev[d]);
            for (int e = 0; e < g; ++e) SBLAS_HIP(hipStreamWaitEvent(C.cst[d], C.evp[(size_t)e * C.parts + p], 0));
            for (int r = 0; r < g && q.stride > 0; ++r)
                SBLAS_HIP(hipMemcpyAsync(C.gathered[d] + (size_t)g * q.lrow0 + (size_t)r * q.stride,
                                         C.ylocal[r] + q.lrow0, sizeof(double) * q.stride,
                                         hipMemcpyDeviceToDevice, C.cst[d]));
        }
    }
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C.dev[d]);
        if (q.rows > 0)
            SBLAS_TRY(sblas_assemble_cyclic(C.gathered[d] + (size_t)g * q.lrow0, g, q.stride, C.chunk_rows, q.rows,
                                            C.yfull[d] + q.grow0, C.cst[d]));
    }
    return SBLAS_OK;
}

void free_parts(sblas_ctx_s &C)
{
    for (size_t i = 0; i < C.P.size(); ++i) {
        DeviceGuard g(C.dev[i / std::max(1, C.parts)]);
        sblas_csr_destroy(C.P[i]);
    }
    C.P.clear();
    C.plo.clear();
    C.parts = 1;
}

void free_matrix(sblas_ctx_s &C)
{
    free_parts(C);
    for (int d = 0; d < (int)C.A.size(); ++d) {
        DeviceGuard g(C.dev[d]);
        sblas_csr_destroy(C.A[d]);
        (void)hipFree(C.x[d]);
        (void)hipFree(C.ylocal[d]);
        (void)hipFree(C.gathered[d]);
        if (!C.yalias) (void)hipFree(C.yfull[d]);
        (void)hipFree(C.meta[d]);
        (void)hipFree(C.bar[d]);
        if (d < (int)C.yptr.size()) (void)hipFree(C.yptr[d]);
    }
    C.yptr.clear();
    C.A.clear();
    C.x.clear();
    C.ylocal.clear();
    C.gathered.clear();
    C.yfull.clear();
    C.yalias = false;
    C.meta.clear();
    C.bar.clear();
    C.h_meta.clear();
    C.lrows.clear();
    C.lnnz.clear();
    C.yoff.clear();
    C.last.clear();
    C.pending = false;
    C.loaded = false;
}

// comm streams and part events, created on the first overlapped upload
int ensure_overlap_streams(sblas_ctx_s &C)
{
    const int g = C.g;
    if (C.cst.empty()) {
        C.cst.assign(g, nullptr);
        C.evc.assign(g, nullptr);
    }
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C.dev[d]);
        if (!C.cst[d]) SBLAS_HIP(hipStreamCreateWithFlags(&C.cst[d], hipStreamNonBlocking));
        if (!C.evc[d]) SBLAS_HIP(hipEventCreateWithFlags(&C.evc[d], hipEventDisableTiming));
    }
    const size_t need = (size_t)g * C.parts;
    if (C.evp.size() != need) {
        // device-major: event i belongs to device i / parts.  Rebuilt whenever
        // the part count changes (a re-upload with fewer parts must not record
        // an event created on another device), each old event destroyed on
        // the device it was created on
        for (size_t i = 0; i < C.evp.size(); ++i) {
            DeviceGuard gd(C.evp_dev[i]);
            if (C.evp[i]) (void)hipEventDestroy(C.evp[i]);
        }
        C.evp.assign(need, nullptr);
        C.evp_dev.assign(need, 0);
        for (size_t i = 0; i < need; ++i) {
            C.evp_dev[i] = C.dev[i / C.parts];
            DeviceGuard gd(C.evp_dev[i]);
            SBLAS_HIP(hipEventCreateWithFlags(&C.evp[i], hipEventDisableTiming));
        }
    }
    return SBLAS_OK;
}

// device d's part handles: part p = its local rows of local chunks
// [plo[p], plo[p+1]), all run with the whole slice's algorithm (AUTO
// resolved once on the whole slice, after sblas_csr_analyse has applied its
// fallback, so every part runs the same kernel the plain path would)
int upload_parts(sblas_ctx_s &C, int d, const std::vector<long long> &lrp, const std::vector<int> &lcol,
                 const std::vector<double> &lval)
{
    const long long lm = (long long)lrp.size() - 1, R = C.chunk_rows;
    int a = C.algo;
    if (a == SBLAS_SPMV_AUTO) SBLAS_TRY(sblas_csr_pick(C.A[d], C.st[d], &a));
    C.palgo[d] = a;
    for (int p = 0; p < C.parts; ++p) {
        const long long r0 = std::min(lm, C.plo[p] * R), r1 = std::min(lm, C.plo[p + 1] * R);
        if (r1 <= r0) continue;
        sblas_csr &H = C.P[(size_t)d * C.parts + p];
        SBLAS_TRY(sblas_csr_upload_slice(&H, C.dev[d], C.n, lrp.data(), lcol.data(), lval.data(), (int)r0,
                                         (int)r1, lrp[r0], lrp[r1], C.st[d]));
        SBLAS_TRY(sblas_csr_analyse(H, a, C.st[d]));
    }
    return SBLAS_OK;
}

// The loopback all-reduce (k_ctx_sum) reads every rank's send buffer from
// the summing rank's device: ranks wrapped onto distinct GPUs need peer
// access between them (refused if a pair has none).  Only this exchange
// needs it -- the all-gather's device-to-device copies do not.  The links
// are reference-counted process-wide (peer_acquire), so a second context or
// a trsv_mgpu handle on the same pair keeps its access when this context is
// destroyed.
int enable_loopback_peers(sblas_ctx_s &C)
{
    for (int a = 0; a < C.g; ++a)
        for (int b = 0; b < C.g; ++b) {
            const int da = C.dev[a], db = C.dev[b];
            if (da == db) continue;
            if (std::find(C.peers.begin(), C.peers.end(), std::make_pair(da, db)) != C.peers.end()) continue;
            SBLAS_TRY(peer_acquire(da, db, "sblas_ctx_matrix_upload (loopback all-reduce)"));
            C.peers.emplace_back(da, db);
        }
    return SBLAS_OK;
}

}  // namespace

extern "C" {

int sblas_cyclic_plan(long long m, int g, int chunks_per_rank, long long *chunk_rows,
                      long long *stride)
{
    if (m < 0 || g <= 0 || chunks_per_rank <= 0 || !chunk_rows || !stride) return SBLAS_ERR_INVALID;
    const long long R = std::max(1LL, (m + (long long)g * chunks_per_rank - 1) / ((long long)g * chunks_per_rank));
    const long long nchunks = m ? (m + R - 1) / R : 0;
    *chunk_rows = R;
    *stride = std::max(1LL, ((nchunks + g - 1) / g) * R);
    return SBLAS_OK;
}

int sblas_cyclic_local_csr(int m, const long long *rowptr, const int *col, const double *val, int g,
                           long long chunk_rows, int d, long long *local_m, long long *local_nnz,
                           long long *lrowptr, int *lcol, double *lval)
{
    if (m < 0 || !rowptr || g <= 0 || chunk_rows <= 0 || d < 0 || d >= g || !local_m || !local_nnz)
        return SBLAS_ERR_INVALID;
    const long long nchunks = m ? (m + chunk_rows - 1) / chunk_rows : 0;
    long long lm = 0, lz = 0;
    for (long long j = d; j < nchunks; j += g) {
        const long long a = j * chunk_rows, b = std::min<long long>(m, a + chunk_rows);
        if (lrowptr) {
            for (long long r = a; r < b; ++r) lrowptr[lm + (r - a) + 1] = lz + (rowptr[r + 1] - rowptr[a]);
            if (lm == 0) lrowptr[0] = 0;
        }
        const long long cnt = rowptr[b] - rowptr[a];
        if (lcol && cnt) std::memcpy(lcol + lz, col + rowptr[a], sizeof(int) * (size_t)cnt);
        if (lval && cnt) std::memcpy(lval + lz, val + rowptr[a], sizeof(double) * (size_t)cnt);
        lm += b - a;
        lz += cnt;
    }
    if (lrowptr && lm == 0) lrowptr[0] = 0;
    *local_m = lm;
    *local_nnz = lz;
    return SBLAS_OK;
}

int sblas_ctx_create(sblas_ctx *out, int ngpu, const int *devlist)
{
    if (!out || ngpu <= 0) return SBLAS_ERR_INVALID;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SBLAS_ERR_NODEV;
    // loopback rehearsal: ranks may share GPUs (ordinals wrap), no RCCL
    const char *lbe = getenv("SBLAS_CTX_LOOPBACK");
    const bool loopback = lbe && atoi(lbe) != 0;
    std::vector<int> dev(ngpu);
    for (int d = 0; d < ngpu; ++d) {
        dev[d] = devlist ? devlist[d] : loopback ? d % count : d;
        if (dev[d] < 0 || dev[d] >= count) {
            set_error("sblas_ctx_create: device %d of %d visible (one rank per GPU: no wrapping)",
                      dev[d], count);
            return SBLAS_ERR_INVALID;
        }
        for (int e = 0; e < d && !loopback; ++e)
            if (dev[e] == dev[d]) {
                set_error("sblas_ctx_create: device %d listed twice", dev[d]);
                return SBLAS_ERR_INVALID;
            }
    }
    auto *C = new sblas_ctx_s();
    C->g = ngpu;
    C->dev = dev;
    C->loopback = loopback;
    const char *nae = getenv("SBLAS_CTX_NOALIAS");
    C->noalias = nae && atoi(nae) != 0;
    C->comm.assign(ngpu, nullptr);
    if (!loopback) {
        ncclResult_t r = ncclCommInitAll(C->comm.data(), ngpu, dev.data());
        if (r != ncclSuccess) {
            set_error("ncclCommInitAll(%d): %s", ngpu, ncclGetErrorString(r));
            C->comm.clear();
            sblas_ctx_destroy(C);
            return SBLAS_ERR_RCCL;
        }
    }
    C->st.assign(ngpu, nullptr);
    C->ev.assign((size_t)3 * ngpu, nullptr);
    C->evx.assign(ngpu, nullptr);
    C->evy.assign(ngpu, nullptr);
    for (int d = 0; d < ngpu; ++d) {
        DeviceGuard g(dev[d]);
        hipError_t e = hipStreamCreateWithFlags(&C->st[d], hipStreamNonBlocking);
        for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreate(&C->ev[(size_t)3 * d + k]);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&C->evx[d], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&C->evy[d], hipEventDisableTiming);
        if (e != hipSuccess) {
            set_error("sblas_ctx_create: %s", hipGetErrorString(e));
            sblas_ctx_destroy(C);
            return SBLAS_ERR_HIP;
        }
    }
    *out = C;
    return SBLAS_OK;
}

int sblas_ctx_destroy(sblas_ctx C)
{
    if (!C) return SBLAS_OK;
    if (g_bound == C) g_bound = nullptr;
    free_matrix(*C);
    for (int d = 0; d < C->g; ++d) {
        DeviceGuard g(C->dev[d]);
        if (d < (int)C->comm.size() && C->comm[d]) (void)ncclCommDestroy(C->comm[d]);
        if (d < (int)C->st.size() && C->st[d]) (void)hipStreamDestroy(C->st[d]);
        for (int k = 0; k < 3; ++k)
            if ((size_t)3 * d + k < C->ev.size() && C->ev[(size_t)3 * d + k])
                (void)hipEventDestroy(C->ev[(size_t)3 * d + k]);
        if (d < (int)C->evx.size() && C->evx[d]) (void)hipEventDestroy(C->evx[d]);
        if (d < (int)C->evy.size() && C->evy[d]) (void)hipEventDestroy(C->evy[d]);
        if (d < (int)C->cst.size() && C->cst[d]) (void)hipStreamDestroy(C->cst[d]);
        if (d < (int)C->evc.size() && C->evc[d]) (void)hipEventDestroy(C->evc[d]);
    }
    for (size_t i = 0; i < C->evp.size(); ++i) {
        DeviceGuard g(C->evp_dev[i]);
        if (C->evp[i]) (void)hipEventDestroy(C->evp[i]);
    }
    for (const auto &pr : C->peers) peer_release(pr.first, pr.second);
    (void)hipGetLastError();
    delete C;
    return SBLAS_OK;
}

int sblas_ctx_ngpu(sblas_ctx C, int *ngpu)
{
    if (!C || !ngpu) return SBLAS_ERR_INVALID;
    *ngpu = C->g;
    return SBLAS_OK;
}

int sblas_ctx_comm_info(sblas_ctx C, int *nranks, int *devices)
{
    if (!C) return SBLAS_ERR_INVALID;
    const bool has_comm = !C->comm.empty() && C->comm[0];
    if (nranks) {
        *nranks = 0;
        if (has_comm) SBLAS_NCCL(ncclCommCount(C->comm[0], nranks));
    }
    for (int d = 0; devices && d < C->g; ++d) {
        devices[d] = C->dev[d];
        if (has_comm && d < (int)C->comm.size() && C->comm[d]) SBLAS_NCCL(ncclCommCuDevice(C->comm[d], &devices[d]));
    }
    return SBLAS_OK;
}

int sblas_ctx_matrix_upload_ex(sblas_ctx C, int m, int n, const long long *rowptr, const int *col,
                               const double *val, int algo, int partition, int exchange)
{
    if (!C || m < 0 || n < 0 || !rowptr || partition < 0 || partition > 2) return SBLAS_ERR_INVALID;
    if (algo < SBLAS_SPMV_AUTO || algo > SBLAS_SPMV_XSORT) return SBLAS_ERR_INVALID;
    if (exchange != SBLAS_CTX_ALLGATHER && exchange != SBLAS_CTX_ALLREDUCE) return SBLAS_ERR_INVALID;
    if (exchange == SBLAS_CTX_ALLREDUCE && partition == 0) {
        set_error("sblas_ctx_matrix_upload: the allreduce exchange needs a contiguous-range partition (1 or 2): each "
                  "device's rows must be one contiguous range of the zero-padded y");
        return SBLAS_ERR_INVALID;
    }
    free_matrix(*C);
    const int g = C->g;
    if (C->loopback && exchange == SBLAS_CTX_ALLREDUCE) SBLAS_TRY(enable_loopback_peers(*C));
    C->m = m;
    C->n = n;
    C->nnz = rowptr[m];
    C->algo = algo;
    C->partition = partition;
    C->exchange = exchange;
    C->A.assign(g, nullptr);
    C->x.assign(g, nullptr);
    C->ylocal.assign(g, nullptr);
    C->gathered.assign(g, nullptr);
    C->yfull.assign(g, nullptr);
    C->meta.assign(g, nullptr);
    C->bar.assign(g, nullptr);
    C->lrows.assign(g, 0);
    C->lnnz.assign(g, 0);
    C->yoff.assign(g, 0);
    std::vector<long long> si(g), ei(g);
    std::vector<int> sr(g), er(g), sf(g);
    if (partition == 0) {
        SBLAS_TRY(sblas_cyclic_plan(m, g, 8, &C->chunk_rows, &C->stride));
    } else {
        if (partition == 1) {
            SBLAS_TRY(sblas_partition_nnz(m, C->nnz, rowptr, g, si.data(), ei.data(), sr.data(), er.data(),
                                          sf.data()));
        } else {  // cost-weighted whole rows: per-row weight kCtxRowCost
            SBLAS_TRY(sblas_partition_cost(m, rowptr, g, kCtxRowCost, si.data(), ei.data(),
                                           sr.data(), er.data(), sf.data()));
        }
        C->h_meta.assign((size_t)3 * g, 0);
        long long mx = 1;
        for (int d = 0; d < g; ++d) {
            const long long nr = std::max(0, er[d] - sr[d] + 1);
            C->h_meta[(size_t)3 * d] = sr[d];
            C->h_meta[(size_t)3 * d + 1] = (int)nr;
            C->h_meta[(size_t)3 * d + 2] = sf[d];
            mx = std::max(mx, nr);
        }
        C->stride = mx;
    }
    // allgather: each device's padded slice of `stride` rows; allreduce: a
    // zero-padded full-length y whose own rows the kernel writes in place
    C->ylen = exchange == SBLAS_CTX_ALLREDUCE ? std::max(m, 1) : C->stride;
    // overlapped exchange: parts of consecutive local chunks (at most one
    // part per chunk of a device's slice)
    if (partition == 0 && exchange == SBLAS_CTX_ALLGATHER && C->parts_req > 1 && m > 0) {
        const long long ncmax = C->stride / C->chunk_rows;
        C->parts = (int)std::min<long long>(C->parts_req, ncmax);
        if (C->parts > 1) {
            C->plo.resize((size_t)C->parts + 1);
            for (int p = 0; p <= C->parts; ++p) C->plo[p] = (long long)p * ncmax / C->parts;
            C->P.assign((size_t)g * C->parts, nullptr);
            C->palgo.assign(g, algo);
            SBLAS_TRY(ensure_overlap_streams(*C));
        }
    }
    C->yalias = g == 1 && C->parts <= 1 && !C->noalias;
    int st = SBLAS_OK;
    for (int d = 0; d < g && st == SBLAS_OK; ++d) {
        DeviceGuard gd(C->dev[d]);
        if (partition == 0) {
            long long lm = 0, lz = 0;
            SBLAS_TRY(sblas_cyclic_local_csr(m, rowptr, col, val, g, C->chunk_rows, d, &lm, &lz,
                                             nullptr, nullptr, nullptr));
            std::vector<long long> lrp((size_t)lm + 1);
            std::vector<int> lcol((size_t)std::max(lz, 1LL));
            std::vector<double> lval((size_t)std::max(lz, 1LL));
            SBLAS_TRY(sblas_cyclic_local_csr(m, rowptr, col, val, g, C->chunk_rows, d, &lm, &lz,
                                             lrp.data(), lcol.data(), lval.data()));
            C->lrows[d] = lm;
            C->lnnz[d] = lz;
            st = sblas_csr_upload_slice(&C->A[d], C->dev[d], n, lrp.data(), lcol.data(), lval.data(), 0,
                                        (int)lm, 0, lz, C->st[d]);
            if (st == SBLAS_OK) st = sblas_csr_analyse(C->A[d], algo, C->st[d]);
            if (st == SBLAS_OK && C->parts > 1) st = upload_parts(*C, d, lrp, lcol, lval);
        } else {
            C->lrows[d] = std::max(0, er[d] - sr[d] + 1);
            C->lnnz[d] = C->lrows[d] > 0 ? ei[d] + 1 - si[d] : 0;
            if (exchange == SBLAS_CTX_ALLREDUCE) C->yoff[d] = sr[d];
            st = sblas_csr_upload_slice(&C->A[d], C->dev[d], n, rowptr, col, val, sr[d], er[d] + 1,
                                        si[d], ei[d] + 1, C->st[d]);
            if (st == SBLAS_OK) st = sblas_csr_analyse(C->A[d], algo, C->st[d]);
        }
        if (st != SBLAS_OK) break;
        hipError_t e = hipMalloc(&C->x[d], sizeof(double) * std::max(n, 1));
        if (e == hipSuccess) e = hipMalloc(&C->ylocal[d], sizeof(double) * C->ylen);
        if (e == hipSuccess && exchange == SBLAS_CTX_ALLGATHER && !C->yalias)
            e = hipMalloc(&C->gathered[d], sizeof(double) * C->stride * g);
        if (e == hipSuccess && C->yalias)
            C->yfull[d] = C->ylocal[d];
        else if (e == hipSuccess)
            e = hipMalloc(&C->yfull[d], sizeof(double) * std::max(m, 1));
        if (e == hipSuccess) e = hipMalloc(&C->bar[d], sizeof(double));
        if (e == hipSuccess) e = hipMemsetAsync(C->bar[d], 0, sizeof(double), C->st[d]);
        if (e == hipSuccess) e = hipMemsetAsync(C->ylocal[d], 0, sizeof(double) * C->ylen, C->st[d]);
        if (e == hipSuccess && partition != 0) {
            e = hipMalloc(&C->meta[d], sizeof(int) * 3 * g);
            if (e == hipSuccess)
                e = hipMemcpyAsync(C->meta[d], C->h_meta.data(), sizeof(int) * 3 * g, hipMemcpyHostToDevice,
                                   C->st[d]);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(C->st[d]);
        if (e != hipSuccess) {
            set_error("sblas_ctx_matrix_upload: %s", hipGetErrorString(e));
            st = SBLAS_ERR_HIP;
        }
    }
    if (st == SBLAS_OK && C->loopback && exchange == SBLAS_CTX_ALLREDUCE) {
        C->yptr.assign(g, nullptr);
        for (int d = 0; d < g && st == SBLAS_OK; ++d) {
            DeviceGuard gd(C->dev[d]);
            std::vector<const double *> h(C->ylocal.begin(), C->ylocal.end());
            if (hipMalloc(&C->yptr[d], sizeof(double *) * g) != hipSuccess ||
                hipMemcpy(C->yptr[d], h.data(), sizeof(double *) * g, hipMemcpyHostToDevice) != hipSuccess) {
                set_error("sblas_ctx_matrix_upload: loopback pointer table");
                st = SBLAS_ERR_HIP;
            }
        }
    }
    if (st != SBLAS_OK) {
        free_matrix(*C);
        return st;
    }
    C->last.assign((size_t)3 + 3 * g, 0.0);
    C->loaded = true;
    return SBLAS_OK;
}

int sblas_ctx_matrix_upload_parts(sblas_ctx C, int m, int n, const long long *rowptr, const int *col,
                                  const double *val, int algo, int parts)
{
    if (!C || parts < 1) return SBLAS_ERR_INVALID;
    C->parts_req = parts;
    const int st = sblas_ctx_matrix_upload_ex(C, m, n, rowptr, col, val, algo, 0, SBLAS_CTX_ALLGATHER);
    C->parts_req = 1;
    return st;
}

int sblas_ctx_parts(sblas_ctx C, int *parts)
{
    if (!C || !parts) return SBLAS_ERR_INVALID;
    *parts = C->loaded ? C->parts : 0;
    return SBLAS_OK;
}

int sblas_ctx_matrix_upload(sblas_ctx C, int m, int n, const long long *rowptr, const int *col,
                            const double *val, int algo, int partition)
{
    return sblas_ctx_matrix_upload_ex(C, m, n, rowptr, col, val, algo, partition, SBLAS_CTX_ALLGATHER);
}

int sblas_ctx_slice_info(sblas_ctx C, int d, long long *rows, long long *nnz, long long *alg_bytes_beta)
{
    if (!C || !C->loaded || d < 0 || d >= C->g) return SBLAS_ERR_INVALID;
    if (rows) *rows = C->lrows[d];
    if (nnz) *nnz = C->lnnz[d];
    if (alg_bytes_beta) *alg_bytes_beta = sblas_spmv_algorithmic_bytes(C->A[d], 1);
    return SBLAS_OK;
}

int sblas_ctx_slice_algo(sblas_ctx C, int d, int *algo)
{
    if (!C || !C->loaded || d < 0 || d >= C->g || !algo) return SBLAS_ERR_INVALID;
    if (C->algo != SBLAS_SPMV_AUTO) {
        *algo = C->algo;
        return SBLAS_OK;
    }
    return sblas_csr_pick(C->A[d], C->st[d], algo);
}

int sblas_ctx_set_x(sblas_ctx C, const double *x)
{
    if (!C || !C->loaded || !x) return SBLAS_ERR_INVALID;
    if (C->n == 0) return SBLAS_OK;
    {
        DeviceGuard g(C->dev[0]);
        SBLAS_HIP(hipMemcpyAsync(C->x[0], x, sizeof(double) * C->n, hipMemcpyHostToDevice, C->st[0]));
    }
    // replicate x from device 0 over xGMI
    SBLAS_TRY(xchg_broadcast_x(*C));
    for (int d = 0; d < C->g; ++d) {
        DeviceGuard g(C->dev[d]);
        SBLAS_HIP(hipStreamSynchronize(C->st[d]));
    }
    return SBLAS_OK;
}

int sblas_ctx_set_y(sblas_ctx C, const double *y)
{
    if (!C || !C->loaded || !y) return SBLAS_ERR_INVALID;
    std::vector<double> h((size_t)C->ylen);
    for (int d = 0; d < C->g; ++d) {
        std::fill(h.begin(), h.end(), 0.0);
        long long o = 0;
        if (C->partition == 0) {
            const long long nch = C->m ? (C->m + C->chunk_rows - 1) / C->chunk_rows : 0;
            for (long long j = d; j < nch; j += C->g) {
                const long long a = j * C->chunk_rows, b = std::min<long long>(C->m, a + C->chunk_rows);
                std::memcpy(h.data() + o, y + a, sizeof(double) * (size_t)(b - a));
                o += b - a;
            }
        } else {
            const int r0 = C->h_meta[(size_t)3 * d], nr = C->h_meta[(size_t)3 * d + 1];
            double *dst = h.data() + C->yoff[d];
            if (nr > 0) std::memcpy(dst, y + r0, sizeof(double) * nr);
            if (nr > 0 && C->h_meta[(size_t)3 * d + 2]) dst[0] = 0.0;  // continuation: partial only
        }
        DeviceGuard g(C->dev[d]);
        SBLAS_HIP(hipMemcpyAsync(C->ylocal[d], h.data(), sizeof(double) * C->ylen, hipMemcpyHostToDevice,
                                 C->st[d]));
        SBLAS_HIP(hipStreamSynchronize(C->st[d]));
    }
    return SBLAS_OK;
}

// The overlapped step: part p's kernels on the main streams, its exchange on
// the comm streams (xchg_part) while part p + 1's kernels run; the main
// streams then join their comm streams.  Events: start, after the last part
// kernel (kernel span), after the join (whole step).
static int ctx_step_overlapped(sblas_ctx_s &C, double alpha, double beta)
{
    const int g = C.g;
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C.dev[d]);
        SBLAS_HIP(hipEventRecord(C.ev[(size_t)3 * d], C.st[d]));
    }
    for (int p = 0; p < C.parts; ++p) {
        const long long lrow0 = C.plo[p] * C.chunk_rows;
        for (int d = 0; d < g; ++d) {
            DeviceGuard gd(C.dev[d]);
            sblas_csr H = C.P[(size_t)d * C.parts + p];
            if (H) SBLAS_TRY(sblas_spmv(H, C.palgo[d], alpha, C.x[d], beta, C.ylocal[d] + lrow0, C.st[d]));
            SBLAS_HIP(hipEventRecord(C.evp[(size_t)d * C.parts + p], C.st[d]));
        }
        SBLAS_TRY(xchg_part(C, p));
    }
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C.dev[d]);
        SBLAS_HIP(hipEventRecord(C.ev[(size_t)3 * d + 1], C.st[d]));
        SBLAS_HIP(hipEventRecord(C.evc[d], C.cst[d]));
        SBLAS_HIP(hipStreamWaitEvent(C.st[d], C.evc[d], 0));
    }
    // loopback: the next step's kernels overwrite slices other devices read
    if (C.loopback) SBLAS_TRY(lb_barrier(C, C.evy));
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C.dev[d]);
        SBLAS_HIP(hipEventRecord(C.ev[(size_t)3 * d + 2], C.st[d]));
    }
    return SBLAS_OK;
}

// Waits for the step issued last and fills C->last (3 + 3g doubles, ms):
// max over devices of kernel / exchange / step, then per device the same.
static int ctx_collect(sblas_ctx_s *C)
{
    const int g = C->g;
    double kmax = 0.0, xmax = 0.0, tmax = 0.0;
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C->dev[d]);
        SBLAS_HIP(hipEventSynchronize(C->ev[(size_t)3 * d + 2]));
        float k = 0.f, t = 0.f;
        SBLAS_HIP(hipEventElapsedTime(&k, C->ev[(size_t)3 * d], C->ev[(size_t)3 * d + 1]));
        SBLAS_HIP(hipEventElapsedTime(&t, C->ev[(size_t)3 * d], C->ev[(size_t)3 * d + 2]));
        C->last[(size_t)3 + 3 * d] = k;
        C->last[(size_t)4 + 3 * d] = (double)t - k;
        C->last[(size_t)5 + 3 * d] = t;
        kmax = std::max(kmax, (double)k);
        xmax = std::max(xmax, (double)(t - k));
        tmax = std::max(tmax, (double)t);
    }
    C->last[0] = kmax;
    C->last[1] = xmax;
    C->last[2] = tmax;
    C->pending = false;
    return SBLAS_OK;
}

int sblas_ctx_spmv_ex(sblas_ctx C, double alpha, double beta, double delay_us, int wait, double *stats)
{
    if (!C || !C->loaded || delay_us < 0.0 || delay_us > 1e5) return SBLAS_ERR_INVALID;
    const int g = C->g;
    if (delay_us > 0.0) {
        // timing protocol: every stream waits on the device while the host
        // enqueues the whole step, then a one-element all-reduce lines the
        // devices up, so each device's span (start event .. after the
        // exchange) starts together with the others'
        for (int d = 0; d < g; ++d) {
            DeviceGuard gd(C->dev[d]);
            hipLaunchKernelGGL(k_ctx_delay, dim3(1), dim3(1), 0, C->st[d],
                               (unsigned long long)(delay_us * 100.0));
            SBLAS_HIP(hipGetLastError());
        }
        SBLAS_TRY(xchg_barrier(*C));
    }
    if (C->parts > 1) {
        SBLAS_TRY(ctx_step_overlapped(*C, alpha, beta));
        C->pending = true;
        if (!wait) return SBLAS_OK;
        SBLAS_TRY(ctx_collect(C));
        if (stats) std::copy(C->last.begin(), C->last.end(), stats);
        return SBLAS_OK;
    }
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C->dev[d]);
        SBLAS_HIP(hipEventRecord(C->ev[(size_t)3 * d], C->st[d]));
        if (C->lrows[d] > 0)
            SBLAS_TRY(sblas_spmv(C->A[d], C->algo, alpha, C->x[d], beta, C->ylocal[d] + C->yoff[d],
                                 C->st[d]));
        SBLAS_HIP(hipEventRecord(C->ev[(size_t)3 * d + 1], C->st[d]));
    }
    if (!C->yalias) SBLAS_TRY(xchg_spmv(*C));
    for (int d = 0; d < g; ++d) {
        DeviceGuard gd(C->dev[d]);
        if (C->yalias) {
            // single device: the kernel wrote y in place
        } else if (C->exchange == SBLAS_CTX_ALLREDUCE) {
            const long long nr = C->lrows[d];
            if (nr > 0) {
                hipLaunchKernelGGL(k_ctx_reprime, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, C->st[d],
                                   C->yfull[d] + C->yoff[d], C->ylocal[d] + C->yoff[d], nr,
                                   C->h_meta[(size_t)3 * d + 2]);
                SBLAS_HIP(hipGetLastError());
            }
        } else if (C->partition == 0) {
            SBLAS_TRY(sblas_assemble_cyclic(C->gathered[d], g, C->stride, C->chunk_rows, C->m, C->yfull[d],
                                            C->st[d]));
        } else {  // also re-primes this device's slice as the next call's y input
            SBLAS_TRY(sblas_assemble_slices(C->gathered[d], g, C->stride, C->meta[d], C->yfull[d], d,
                                            C->ylocal[d], C->st[d]));
        }
        SBLAS_HIP(hipEventRecord(C->ev[(size_t)3 * d + 2], C->st[d]));
    }
    C->pending = true;
    if (!wait) return SBLAS_OK;
    SBLAS_TRY(ctx_collect(C));
    if (stats) std::copy(C->last.begin(), C->last.end(), stats);
    return SBLAS_OK;
}

int sblas_ctx_sync(sblas_ctx C, double *stats)
{
    if (!C || !C->loaded) return SBLAS_ERR_INVALID;
    if (C->pending) SBLAS_TRY(ctx_collect(C));
    if (stats) std::copy(C->last.begin(), C->last.end(), stats);
    return SBLAS_OK;
}

int sblas_ctx_spmv(sblas_ctx C, double alpha, double beta, double *stats)
{
    if (!C || !C->loaded) return SBLAS_ERR_INVALID;
    SBLAS_TRY(sblas_ctx_spmv_ex(C, alpha, beta, 0.0, 1, nullptr));
    if (stats) std::copy(C->last.begin(), C->last.begin() + 3, stats);
    return SBLAS_OK;
}

int sblas_ctx_get_y(sblas_ctx C, int device_index, double *y)
{
    if (!C || !C->loaded || !y || device_index < 0 || device_index >= C->g) return SBLAS_ERR_INVALID;
    if (C->m == 0) return SBLAS_OK;
    DeviceGuard g(C->dev[device_index]);
    SBLAS_HIP(hipMemcpyAsync(y, C->yfull[device_index], sizeof(double) * C->m, hipMemcpyDeviceToHost,
                             C->st[device_index]));
    SBLAS_HIP(hipStreamSynchronize(C->st[device_index]));
    return SBLAS_OK;
}

}  // extern "C"

extern "C" int sblas_ctx_bind(sblas_ctx C)
{
    sblas::g_bound = C;
    return SBLAS_OK;
}
