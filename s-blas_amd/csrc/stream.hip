// stream.hip -- out-of-core SpMV executor (the task pool of
// spMV_mgpu_v2, spmv/src/dspmv_mgpu_v2.cu:33-441, with its Hyper-Q streams).
//
// The matrix stays in HOST memory and is streamed through the GPUs chunk by
// chunk, so it may exceed the aggregate HBM:
//   * chunks = nnz-balanced element ranges (sblas_partition_nnz; a row may
//     span chunks);
//   * one host thread per physical GPU takes chunks from a shared counter
//     (dynamic, like v2's OpenMP task loop) and cycles them over its
//     `nstreams` stream slots, so the H2D of chunk t+1 overlaps the kernel of
//     chunk t;
//   * col/val are DMA'd straight from the caller's arrays (pinned in place
//     with hipHostRegister for the call; already-pinned memory is accepted);
//     rowptr is rebased to int32 on the host into pinned staging, and the
//     row-split plan of the chunk is built there too;
//   * x is uploaded once per GPU (v2 re-sends the full x with every task);
//   * streams, device buffers and pinned staging persist per device across
//     calls (a call only grows them), so repeated calls pay only the DMA;
//   * every chunk returns its rows of y; a chunk that starts inside a row
//     (continuation) computes that row's partial with y0 zeroed and the
//     partial is added after all chunks are merged -- the v1 fix-up
//     (dspmv_mgpu_v1.cu:235-248) generalised to rows spanning many chunks.
#include <atomic>
#include <mutex>
#include <cstring>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "sblas_internal.hpp"

using namespace sblas;

namespace {

struct Chunk {
    int r0, r1;        // rows [r0, r1] (inclusive)
    long long i0, i1;  // elements [i0, i1] (inclusive)
    bool cont;         // first row continues the previous chunk
};

struct Slot {
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    int *d_rowptr = nullptr, *d_col = nullptr;
    double *d_val = nullptr, *d_y = nullptr, *d_partial = nullptr;
    RowBlock *d_blocks = nullptr;
    int4 *d_long = nullptr;
    // pinned host staging
    int *h_rowptr = nullptr;
    RowBlock *h_blocks = nullptr;
    int4 *h_long = nullptr;
    double *h_y = nullptr;
    int chunk = -1;  // chunk whose result is in flight (-1: none)
    int cap_rows = 0;
    long long cap_nnz = 0;
};

// Per-device resources kept across calls (streams, events, device buffers
// and pinned staging are costly to create; a call only grows them).
struct DevPool {
    std::mutex mu;
    double *d_x = nullptr;
    int cap_x = 0;
    std::vector<Slot> slots;
};
DevPool g_pool[64];

void free_slot(Slot &q)
{
    (void)hipFree(q.d_rowptr);
    (void)hipFree(q.d_col);
    (void)hipFree(q.d_val);
    (void)hipFree(q.d_y);
    (void)hipFree(q.d_partial);
    (void)hipFree(q.d_blocks);
    (void)hipFree(q.d_long);
    (void)hipHostFree(q.h_rowptr);
    (void)hipHostFree(q.h_blocks);
    (void)hipHostFree(q.h_long);
    (void)hipHostFree(q.h_y);
    Slot keep;
    keep.s = q.s;
    keep.done = q.done;
    q = keep;
}

}  // namespace

extern "C" int sblas_spmv_ooc(int m, int n, long long nnz, double alpha, const long long *rowptr,
                              const int *col, const double *val, const double *x, double beta,
                              double *y, int ngpu, long long chunk_nnz, int nstreams,
                              double *stats)
{
    if (m < 0 || n < 0 || nnz < 0 || ngpu <= 0 || nstreams <= 0 || chunk_nnz <= 0 || !rowptr ||
        (nnz && (!col || !val)) || (n && !x) || (m && !y) || rowptr[m] != nnz)
        return SBLAS_ERR_INVALID;
    if (m == 0) return SBLAS_OK;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SBLAS_ERR_NODEV;
    const double t_start = sblas_get_time();
    // chunks
    chunk_nnz = std::min<long long>(chunk_nnz, (1LL << 30));
    const long long T64 = std::max<long long>(1, (nnz + chunk_nnz - 1) / chunk_nnz);
    if (T64 > (1 << 24)) return SBLAS_ERR_INVALID;
    const int T = (int)T64;
    std::vector<long long> si(T), ei(T);
    std::vector<int> sr(T), er(T), sf(T);
    SBLAS_TRY(sblas_partition_nnz(m, nnz, rowptr, T, si.data(), ei.data(), sr.data(), er.data(), sf.data()));
    std::vector<Chunk> chunks(T);
    int max_rows = 1;
    long long max_nnz = 1;
    for (int t = 0; t < T; ++t) {
        chunks[t] = {sr[t], er[t], si[t], ei[t], sf[t] != 0};
        max_rows = std::max(max_rows, er[t] - sr[t] + 1);
        max_nnz = std::max(max_nnz, ei[t] - si[t] + 1);
    }
    // pin the caller's arrays in place for the DMA
    const double t_reg0 = sblas_get_time();
    bool reg_col = false, reg_val = false;
    if (nnz) {
        hipError_t e = hipHostRegister((void *)col, sizeof(int) * nnz, hipHostRegisterDefault);
        reg_col = e == hipSuccess;
        if (e != hipSuccess) (void)hipGetLastError();
        e = hipHostRegister((void *)val, sizeof(double) * nnz, hipHostRegisterDefault);
        reg_val = e == hipSuccess;
        if (e != hipSuccess) (void)hipGetLastError();
    }
    const double t_reg = sblas_get_time() - t_reg0;
    std::vector<double> carry(T, 0.0);
    std::atomic<int> next{0};
    std::atomic<long long> setup_ns{0};
    std::atomic<int> status{SBLAS_OK};
    std::atomic<long long> h2d_bytes{0};
    const int ndev = std::min(ngpu, count);
    double t_kernels_end = 0.0;
#pragma omp parallel num_threads(ndev)
    {
        int dev = 0;
#ifdef _OPENMP
        dev = omp_get_thread_num();
#endif
        DevPool &pool = g_pool[dev & 63];
        std::lock_guard<std::mutex> lock(pool.mu);
        if ((int)pool.slots.size() < nstreams) pool.slots.resize(nstreams);
        Slot *slots = pool.slots.data();
        auto fail = [&](int st) {
            int ok = SBLAS_OK;
            status.compare_exchange_strong(ok, st);
        };
        auto check = [&](hipError_t e, const char *what) {
            if (e != hipSuccess) {
                set_error("spmv_ooc: %s -> %s", what, hipGetErrorString(e));
                fail(SBLAS_ERR_HIP);
                return false;
            }
            return true;
        };
        // a finished chunk's rows go to y; its continuation partial to carry
        auto merge = [&](Slot &q) {
            if (q.chunk < 0) return;
            if (!check(hipEventSynchronize(q.done), "event sync")) return;
            const Chunk &c = chunks[q.chunk];
            const int dm = c.r1 - c.r0 + 1;
            if (c.cont) {
                carry[q.chunk] = q.h_y[0];
                if (dm > 1) std::memcpy(y + c.r0 + 1, q.h_y + 1, sizeof(double) * (dm - 1));
            } else {
                std::memcpy(y + c.r0, q.h_y, sizeof(double) * dm);
            }
            q.chunk = -1;
        };
        if (hipSetDevice(dev) == hipSuccess) {
            const double ts = sblas_get_time();
            bool ok = true;
            if (pool.cap_x < n) {
                (void)hipFree(pool.d_x);
                pool.d_x = nullptr;
                pool.cap_x = 0;
                ok = check(hipMalloc(&pool.d_x, sizeof(double) * std::max(n, 1)), "malloc x");
                if (ok) pool.cap_x = n;
            }
            double *d_x = pool.d_x;
            ok = ok && (n == 0 || check(hipMemcpy(d_x, x, sizeof(double) * n, hipMemcpyHostToDevice), "x H2D"));
            for (int qi = 0; qi < nstreams && ok; ++qi) {
                Slot &q = slots[qi];
                q.chunk = -1;
                if (!q.s)
                    ok = check(hipStreamCreateWithFlags(&q.s, hipStreamNonBlocking), "stream") &&
                         check(hipEventCreateWithFlags(&q.done, hipEventDisableTiming), "event");
                if (!ok || (q.cap_rows >= max_rows && q.cap_nnz >= max_nnz)) continue;
                free_slot(q);
                const int cr = std::max(max_rows, q.cap_rows);
                const long long cn = std::max(max_nnz, q.cap_nnz);
                const int cb = cr + (int)(cn / kRsLongChunk) + 2;
                ok = check(hipMalloc(&q.d_rowptr, sizeof(int) * (cr + 1)), "malloc") &&
                     check(hipMalloc(&q.d_col, sizeof(int) * (cn + 8)), "malloc") &&
                     check(hipMalloc(&q.d_val, sizeof(double) * (cn + 8)), "malloc") &&
                     check(hipMemset(q.d_col, 0, sizeof(int) * (cn + 8)), "memset") &&
                     check(hipMemset(q.d_val, 0, sizeof(double) * (cn + 8)), "memset") &&
                     check(hipMalloc(&q.d_y, sizeof(double) * cr), "malloc") &&
                     check(hipMalloc(&q.d_partial, sizeof(double) * cb), "malloc") &&
                     check(hipMalloc(&q.d_blocks, sizeof(RowBlock) * cb), "malloc") &&
                     check(hipMalloc(&q.d_long, sizeof(int4) * cr), "malloc") &&
                     check(hipHostMalloc(&q.h_rowptr, sizeof(int) * (cr + 1), hipHostMallocDefault), "pinned") &&
                     check(hipHostMalloc(&q.h_blocks, sizeof(RowBlock) * cb, hipHostMallocDefault), "pinned") &&
                     check(hipHostMalloc(&q.h_long, sizeof(int4) * cr, hipHostMallocDefault), "pinned") &&
                     check(hipHostMalloc(&q.h_y, sizeof(double) * cr, hipHostMallocDefault), "pinned");
                if (ok) {
                    q.cap_rows = cr;
                    q.cap_nnz = cn;
                } else {
                    free_slot(q);
                }
            }
            setup_ns += (long long)((sblas_get_time() - ts) * 1e9);
            std::vector<RowBlock> blocks;
            std::vector<int4> longs;
            int k = 0;
            while (ok && status.load() == SBLAS_OK) {
                const int t = next.fetch_add(1);
                if (t >= T) break;
                Slot &q = slots[k];
                k = (k + 1) % nstreams;
                merge(q);  // the slot's previous chunk, before its staging is reused
                const Chunk &c = chunks[t];
                const int dm = c.r1 - c.r0 + 1;
                const long long cn = c.i1 - c.i0 + 1;
                // local rowptr (first/last rows clipped to the chunk, v1's
                // [0] = 0 / [dm] = dev_nnz rule, dspmv_mgpu_v1.cu:125-133)
                q.h_rowptr[0] = 0;
                for (int r = 1; r < dm; ++r) q.h_rowptr[r] = (int)(rowptr[c.r0 + r] - c.i0);
                q.h_rowptr[dm] = (int)cn;
                blocks.clear();
                longs.clear();
                int nslots = 0;
                make_row_blocks(q.h_rowptr, dm, blocks, longs, nslots);
                std::memcpy(q.h_blocks, blocks.data(), sizeof(RowBlock) * blocks.size());
                if (!longs.empty()) std::memcpy(q.h_long, longs.data(), sizeof(int4) * longs.size());
                // y0 of the chunk's rows; a continuation row starts from 0 (and
                // is not read: the previous chunk's merge may be writing it)
                if (c.cont) {
                    q.h_y[0] = 0.0;
                    if (dm > 1) std::memcpy(q.h_y + 1, y + c.r0 + 1, sizeof(double) * (dm - 1));
                } else {
                    std::memcpy(q.h_y, y + c.r0, sizeof(double) * dm);
                }
                ok = check(hipMemcpyAsync(q.d_rowptr, q.h_rowptr, sizeof(int) * (dm + 1), hipMemcpyHostToDevice, q.s), "H2D") &&
                     check(hipMemcpyAsync(q.d_blocks, q.h_blocks, sizeof(RowBlock) * blocks.size(), hipMemcpyHostToDevice, q.s), "H2D") &&
                     (longs.empty() || check(hipMemcpyAsync(q.d_long, q.h_long, sizeof(int4) * longs.size(), hipMemcpyHostToDevice, q.s), "H2D")) &&
                     check(hipMemcpyAsync(q.d_col, col + c.i0, sizeof(int) * cn, hipMemcpyHostToDevice, q.s), "H2D") &&
                     check(hipMemcpyAsync(q.d_val, val + c.i0, sizeof(double) * cn, hipMemcpyHostToDevice, q.s), "H2D") &&
                     (beta == 0.0 || check(hipMemcpyAsync(q.d_y, q.h_y, sizeof(double) * dm, hipMemcpyHostToDevice, q.s), "H2D"));
                if (!ok) break;
                const int st = launch_rowsplit_raw(q.d_rowptr, q.d_col, q.d_val, d_x, q.d_blocks, (int)blocks.size(),
                                                   q.d_long, (int)longs.size(), q.d_partial, alpha, beta, q.d_y, q.s);
                if (st != SBLAS_OK) {
                    fail(st);
                    break;
                }
                ok = check(hipMemcpyAsync(q.h_y, q.d_y, sizeof(double) * dm, hipMemcpyDeviceToHost, q.s), "D2H") &&
                     check(hipEventRecord(q.done, q.s), "event");
                q.chunk = t;
                h2d_bytes += (long long)cn * 12 + 4LL * (dm + 1) + (beta != 0.0 ? 8LL * dm : 0);
            }
            for (int qi = 0; qi < nstreams; ++qi) merge(slots[qi]);
        } else {
            fail(SBLAS_ERR_HIP);
        }
        for (int qi = 0; qi < nstreams; ++qi)
            if (slots[qi].s) (void)hipStreamSynchronize(slots[qi].s);
    }
    t_kernels_end = sblas_get_time();
    if (reg_col) (void)hipHostUnregister((void *)col);
    if (reg_val) (void)hipHostUnregister((void *)val);
    if (status.load() != SBLAS_OK) return status.load();
    for (int t = 0; t < T; ++t)
        if (chunks[t].cont) y[chunks[t].r0] += carry[t];
    if (stats) {  // {seconds, H2D GB/s of the streaming phase, chunks, devices, pin s, setup s}
        const double sec = t_kernels_end - t_start;
        const double setup = (double)setup_ns.load() / 1e9 / std::max(ndev, 1);
        const double stream_s = std::max(1e-9, sec - t_reg - setup);
        stats[0] = sec;
        stats[1] = (double)h2d_bytes.load() / stream_s / 1e9;
        stats[2] = T;
        stats[3] = ndev;
        stats[4] = t_reg;
        stats[5] = setup;
    }
    return SBLAS_OK;
}
