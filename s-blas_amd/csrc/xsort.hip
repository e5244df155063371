// xsort.hip -- column-sorted XCD-group CSR SpMV (algo 5) for gfx950.
//
// Replaces the per-device cusparseDcsrmv of spmv/src/dspmv_mgpu_v1.cu:199-210
// (y = alpha*A*x + beta*y, NON_TRANSPOSE, base 0) for matrices whose columns
// scatter over an x far larger than one XCD's 4 MiB L2.
//
// Why: a CSR row-split kernel gathers x[col] one lane per 128-B x line; on
// MI355X such divergent gathers run at ~265 G/s even when every line hits L2
// (profiles/r01_exp_gather.txt), i.e. ~150 us for config 2's 39.75M nonzeros,
// and at ~82 G/s when x (16 MB) misses L2.  Two changes attack both limits:
//  * columns are cut into G = 8q groups of < 2^18 columns (~1 MiB of x); XCD
//    k serves groups [kq, (k+1)q), so its gathers stay in its own L2;
//  * inside a block (row range x group) the entries are sorted by column and
//    the lanes of one gather instruction take CONSECUTIVE entries, so they
//    land on few x lines (the TA merges them): 2x on the gather in the
//    microbenchmark.
// Row sums then arrive in column order, so they accumulate into per-row LDS
// slots with ds_add_f64.  The summation ORDER within a row therefore depends
// on wave timing: results are within the fp64 error bound of the sequential
// row sum (tests) but not bitwise reproducible from run to run, unlike the
// row-split/CSR5/panel kernels.
//
// Storage: each block is padded to whole 256-entry chunks (one wave, 4 entries
// per lane) and every chunk is stored lane-transposed: lane l's 16-byte key
// load holds entries {l, 64+l, 128+l, 192+l} and its two 16-byte value loads
// {l, 64+l} and {128+l, 192+l}.  Streaming therefore runs at the 16-B/lane
// rate while gather j of a wave covers the 64 consecutive entries 64j..64j+63.
// Keys pack (col - g*Wg) << 14 | (row - row0); a padding key has the column
// field all ones (no real column reaches it) and row 0.
//
// Work: a narrow range (short rows) is one sub-item -- it walks all G groups,
// starting at its XCD's first group and wrapping, and writes y; a wide range
// (rows >= 16 entries on average) is 8 sub-items, one per XCD over that XCD's
// q groups, each writing a partial that a reduce pass adds in XCD order.
// Narrow sub-items are bound by gather requests, wide ones by the entry
// stream, so by default every work item PAIRS one of each: the two halves of
// the 1024-thread workgroup (8 waves and 8192 LDS rows each) run them side by
// side and every CU mixes both kinds of traffic.  Items sit in one queue per
// XCD; a persistent grid claims from its own XCD's queue (XCC_ID hardware
// register) and steals when it runs dry.  Inside an item the waves claim
// chunks from LDS counters (xs_stream_dyn), so a team that drains its own
// sub-item continues on its partner's and both halves end together.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <utility>
#include <vector>

#include "sblas_internal.hpp"

namespace sblas {

constexpr int kXsThreads = 1024;
constexpr long long kXsAllWideMaxNnz = 6000000;  // all ranges wide up to this many entries (planner)
// LDS row accumulators per workgroup: 16384 = 128 KiB (default); an
// experiment build may raise it towards the 160 KiB of a gfx950 CU
// (SBLAS_XS_LDS_ROWS=19456: 152 KiB of rows + ~6 KiB of bookkeeping)
#ifndef SBLAS_XS_LDS_ROWS
#define SBLAS_XS_LDS_ROWS 16384
#endif
constexpr int kXsRows = SBLAS_XS_LDS_ROWS;
static_assert(kXsRows % 512 == 0, "two teams of whole 256-row blocks");
constexpr int kXsHalfRows = kXsRows / 2;
constexpr int kXsRowBits = 14;     // packed key: local row in the low 14 bits
constexpr int kXsColBits = 18;     //             group-local column above
constexpr int kXsChunk = 256;      // entries per chunk: one wave, 4 per lane
constexpr int kXsUnroll = 2;       // chunks per wave per pipeline stage
constexpr uint32_t kXsPad = ((1u << kXsColBits) - 1) << kXsRowBits;  // column all ones, row 0
constexpr int kXsTrace = 6;        // longs per trace row
static_assert(kXsRowBits + kXsColBits == 32, "packed key is 32 bits");
static_assert(kXsHalfRows <= (1 << kXsRowBits), "a team's local row must fit the key");
// a range's rows: a team's half, or (unpaired / solo items) the whole
// workgroup's accumulators up to what the key's row field addresses
constexpr int kXsItemRows = kXsRows < (1 << kXsRowBits) ? kXsRows : (1 << kXsRowBits);

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

// XCC_ID hardware register (gfx940+: HW_REG_XCC_ID = 20, bits [3:0]).
__device__ __forceinline__ int xs_xcc_id()
{
    return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7;
}

// Claims a work item: returns its slot in qitems (queue * qstride + index),
// own XCD's queue first, or -1 when every queue is empty.  Called by a whole
// wave: lanes 0-7 read the eight claim heads at once (agent-scope loads that
// go past the XCD's L2, ~1-2 us each under load), so finding every queue
// empty -- what each workgroup does at its end -- costs one round trip
// instead of eight in a row.  The result is valid in every lane.
__device__ __forceinline__ int xs_claim(const XsArgs &a, int xcc)
{
    const int lane = threadIdx.x & 63;
    int qq = (xcc + lane) & 7, ql = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) ql = qq == k ? a.qlen[k] : ql;
    const bool open = lane < 8 &&
                      __hip_atomic_load(&a.qhead[qq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ql;
    unsigned long long mask = __ballot(open);
    while (mask) {
        const int l = __ffsll((long long)mask) - 1;
        mask &= mask - 1;
        const int q = __builtin_amdgcn_readfirstlane((xcc + l) & 7);
        int idx = 0;
        if (lane == 0) idx = atomicAdd(&a.qhead[q], 1);
        idx = __shfl(idx, 0, 64);
        if (idx < a.qlen[q]) return q * a.qstride + idx;
    }
    return -1;
}

// One stream of chunks [c0, c1): consecutive column-group blocks whose chunk
// offsets are bnd[0..ng] (bnd[0] = c0) for groups gb, gb+1, ...  The S waves
// of a team take chunks c0 + w, c0 + w + S, ...; a wave's chunk (hence its
// group) is wave-uniform.
// Software pipeline with ping-pong registers and an even, team-uniform trip
// count (no mid-loop exit, so nothing can be sunk below the adds):
//   gathers(A) | loads(B) | adds(A) | gathers(B) | loads(A') | adds(B)
// sched_barrier pins that issue order; waiting for the gathers (vmcnt counts
// in order) then leaves the next stage's key/value loads in flight.  A wave
// past c1 loads one line (every lane the same address) and adds exact +0.0;
// padding entries add +0.0 too (a select, not a product: x may be inf/nan).
// kMode (timing experiments only, SBLAS_XS_MODE): 0 = the product kernel,
// bit 0 = plain LDS stores instead of ds_add_f64, bit 1 = gathers read x[0],
// bit 3 (xs_stream_dyn only) = no gather at all (a key-derived constant),
// bit 4 (xs_stream_dyn only) = gathers folded into x[0, 65536) (same lane
// pattern, an L2-resident 512 KiB: separates L2 fills from L2 requests).
template <int kMode, int S>
__device__ __forceinline__ void xs_stream(const v4u *__restrict__ key4,
                                          const v2d *__restrict__ val2, int ks, int vs, long long c0,
                                          long long c1, const long long *bnd, int gb, int Wg,
                                          const double *__restrict__ x, double *acc, int wave)
{
    if (c1 <= c0) return;  // team-uniform
    constexpr int U = kXsUnroll;
    const int lane = threadIdx.x & 63;
    int gi = 0;              // the wave's current group (relative to gb)
    long long nb = bnd[1];   // its end
    auto load = [&](long long t, v4u *kk, v2d *va, v2d *vb, int *xo) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long c = c0 + wave + (t * U + u) * S;
            const bool live = c < c1;
            const long long ci = live ? c : c1 - 1;
            kk[u] = __builtin_nontemporal_load(key4 + ci * ks + (live ? lane : 0));
            va[u] = __builtin_nontemporal_load(val2 + ci * vs + (live ? lane : 0));
            vb[u] = __builtin_nontemporal_load(val2 + ci * vs + 64 + (live ? lane : 0));
            while (ci >= nb) nb = bnd[++gi + 1];
            xo[u] = (gb + gi) * Wg;
        }
    };
    auto gather = [&](const v4u *kk, const int *xo, double (*xx)[4]) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = kk[u][j];
                const int idx = k == kXsPad ? xo[u] : xo[u] + (int)(k >> kXsRowBits);
                xx[u][j] = x[(kMode & 2) ? 0 : idx];
            }
    };
    auto accumulate = [&](long long t, const v4u *kk, const v2d *va, const v2d *vb,
                          double (*xx)[4]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool live = c0 + wave + (t * U + u) * S < c1;
            const double v[4] = {va[u].x, va[u].y, vb[u].x, vb[u].y};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = kk[u][j];
                const double p = (live && k != kXsPad) ? v[j] * xx[u][j] : 0.0;
                double *slot = &acc[k & ((1u << kXsRowBits) - 1)];
                if (kMode & 1) *slot = p;
                else atomicAdd(slot, p);
            }
        }
    };
    v4u ka[U], kb[U];
    v2d vaa[U], vab[U], vba[U], vbb[U];
    double xa[U][4], xb[U][4];
    int oa[U], ob[U];
    const long long T = (c1 - c0 + (long long)S * U - 1) / ((long long)S * U);
    load(0, ka, vaa, vab, oa);
    for (long long t = 0; t < T; t += 2) {
        gather(ka, oa, xa);
        __builtin_amdgcn_sched_barrier(0);
        load(t + 1, kb, vba, vbb, ob);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(t, ka, vaa, vab, xa);
        __builtin_amdgcn_sched_barrier(0);
        gather(kb, ob, xb);
        __builtin_amdgcn_sched_barrier(0);
        load(t + 2, ka, vaa, vab, oa);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(t + 1, kb, vba, vbb, xb);
    }
}

// Dynamic form of xs_stream for paired items: instead of the fixed
// wave-interleaved split, every wave claims U consecutive chunks at a time
// from the stream's LDS counter (*ctr, chunks past c0), so a team that has
// finished its own sub-item can drain its partner's: the two halves of a
// pair end together however their narrow/wide costs compare.  Same pipeline
// (gathers | next loads | adds), a claim per stage; claims are monotone per
// wave, so the group walk over bnd[] stays forward-only.
template <int kMode, int U = kXsUnroll>
__device__ __forceinline__ void xs_stream_dyn(const v4u *__restrict__ key4,
                                              const v2d *__restrict__ val2, int ks, int vs, int *ctr,
                                              long long c0, long long c1, const long long *bnd,
                                              int gb, int Wg, const double *__restrict__ x,
                                              double *acc)
{
    if (c1 <= c0) return;  // uniform
    if (__builtin_amdgcn_readfirstlane(
            __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >= c1 - c0)
        return;  // drained already (the common case for a helper)
    const int lane = threadIdx.x & 63;
    int gi = 0;
    long long nb = bnd[1];
    auto claim = [&]() -> long long {
        int v = 0;
        if (lane == 0) v = atomicAdd(ctr, U);
        return c0 + __builtin_amdgcn_readfirstlane(v);
    };
    auto load = [&](long long cb, v4u *kk, v2d *va, v2d *vb, int *xo) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long c = cb + u;
            const bool live = c < c1;
            const long long ci = live ? c : c1 - 1;
            if constexpr ((kMode & 4) != 0) {  // experiment: plain (temporal) loads
                kk[u] = key4[ci * ks + (live ? lane : 0)];
                va[u] = val2[ci * vs + (live ? lane : 0)];
                vb[u] = val2[ci * vs + 64 + (live ? lane : 0)];
            } else {
                kk[u] = __builtin_nontemporal_load(key4 + ci * ks + (live ? lane : 0));
                va[u] = __builtin_nontemporal_load(val2 + ci * vs + (live ? lane : 0));
                vb[u] = __builtin_nontemporal_load(val2 + ci * vs + 64 + (live ? lane : 0));
            }
            while (ci >= nb) nb = bnd[++gi + 1];
            xo[u] = (gb + gi) * Wg;
        }
    };
    auto gather = [&](const v4u *kk, const int *xo, double (*xx)[4]) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = kk[u][j];
                const int idx = k == kXsPad ? xo[u] : xo[u] + (int)(k >> kXsRowBits);
                xx[u][j] = (kMode & 8) ? (double)(k & 1) : x[(kMode & 2) ? 0 : (kMode & 16) ? (idx & 0xffff) : idx];
            }
    };
    auto accumulate = [&](long long cb, const v4u *kk, const v2d *va, const v2d *vb,
                          double (*xx)[4]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool live = cb + u < c1;
            const double v[4] = {va[u].x, va[u].y, vb[u].x, vb[u].y};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = kk[u][j];
                const double p = (live && k != kXsPad) ? v[j] * xx[u][j] : 0.0;
                double *slot = &acc[k & ((1u << kXsRowBits) - 1)];
                if (kMode & 1) *slot = p;
                else atomicAdd(slot, p);
            }
        }
    };
    v4u ka[U], kb[U];
    v2d vaa[U], vab[U], vba[U], vbb[U];
    double xa[U][4], xb[U][4];
    int oa[U], ob[U];
    long long ca = claim();
    if (ca >= c1) return;
    load(ca, ka, vaa, vab, oa);
    for (;;) {
        gather(ka, oa, xa);
        __builtin_amdgcn_sched_barrier(0);
        const long long cb = claim();
        load(cb, kb, vba, vbb, ob);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(ca, ka, vaa, vab, xa);
        __builtin_amdgcn_sched_barrier(0);
        if (cb >= c1) break;
        gather(kb, ob, xb);
        __builtin_amdgcn_sched_barrier(0);
        ca = claim();
        load(ca, ka, vaa, vab, oa);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(cb, kb, vba, vbb, xb);
        __builtin_amdgcn_sched_barrier(0);
        if (ca >= c1) break;
    }
}

// Fused reduce of the wide ranges (replaces k_xsort_reduce when a.fused):
// after its last item a workgroup claims reduce tasks (a wide range's rows
// [r0, r0 + blockDim)) from a global head, waits until all 8 sub-items of
// that range have counted in, and writes y = alpha * sum_k partial[k] (XCD
// order) + beta*y.  Arrival counters are cumulative over launches (a launch
// waits for 8 * epoch), so nothing is reset.  Every sub-item belongs to an
// item already claimed by a running workgroup (the queues are empty when a
// workgroup gets here), so the wait ends; it is bounded all the same.
template <bool kBeta>
__device__ void xs_reduce_phase(const XsArgs &a, double alpha, double beta, double *__restrict__ y)
{
    __shared__ int s_task;
    for (;;) {
        if (threadIdx.x == 0) s_task = atomicAdd(&a.qhead[8], 1);
        __syncthreads();
        const int t = s_task;
        __syncthreads();
        if (t >= a.nrtasks) return;
        const int2 task = a.rtasks[t];
        const XsRange R = a.ranges[task.x];
        if (threadIdx.x == 0) {
            const unsigned want = 8u * a.epoch;
            unsigned spins = 0;
            while (__hip_atomic_load(&a.arrive[R.widx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > (1u << 24)) break;  // bounded: a broken protocol gives a wrong y, not a hang
            }
        }
        __syncthreads();
        const int r = task.y + (int)threadIdx.x;
        if (r < R.nrows) {
            const double *p = a.partial + R.pbase + r;
            double v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                v[k] = __hip_atomic_load(p + (long long)k * R.nrows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k) s += v[k];
            double *yr = y + R.row0 + r;
            *yr = kBeta ? alpha * s + beta * *yr : alpha * s;
        }
    }
}

// kWG threads per workgroup: 1024 (16384 LDS rows, one workgroup per CU) or
// 512 (8192 rows, two independent workgroups per CU).  kPair (1024 only): the
// two halves of the workgroup ("teams", 8 waves and 8192 LDS rows each) run
// the item's two sub-items side by side; otherwise all waves run sub-item 0.
// kDyn (pairs only): the chunks of both sub-items are claimed dynamically
// (xs_stream_dyn); a team drains its own streams, then its partner's.
template <bool kBeta, int kMode, int kWG, bool kPair, int kWA = 8, bool kTrace = false,
          bool kDyn = false, int kU = kXsUnroll>
__global__ __launch_bounds__(kWG) void k_spmv_xsort(const XsArgs a,
                                                    const double *__restrict__ x,
                                                    double alpha, double beta,
                                                    double *__restrict__ y)
{
    static_assert(kWG == 1024 || (kWG == 768 && kPair) || kWG == 512, "workgroup shapes");
    __shared__ double acc_all[(kWG >= 768 || kPair) ? kXsRows : kXsHalfRows];
    __shared__ long long s_bnd_all[2][256];
    __shared__ long long s_rec_all[2][128 + 5];
    __shared__ unsigned long long s_tend[2];
    __shared__ int s_item;
    __shared__ int s_ctr[2][2];  // kDyn: claimed chunks per (team, segment)
    __shared__ int s_par[2][4];  // kDyn: per team {sub valid, k1, g0, n1}
    static_assert(!kDyn || kPair, "dynamic claims pair two sub-items");
    // waves per team: team 0 (the pair's first, normally narrow, sub-item)
    // gets kWA waves, team 1 the rest
    constexpr int SA = kPair ? kWA : kWG / 64;
    constexpr int SB = kPair ? kWG / 64 - kWA : 0;
    static_assert(!kPair || (kWA >= 1 && kWA < kWG / 64), "team split");
    const int half = kPair ? (int)(threadIdx.x >= (unsigned)(SA * 64)) : 0;
    const int NT = half ? SB * 64 : SA * 64;                 // threads in this team
    const int ht = (int)threadIdx.x - half * SA * 64;
    const int hwave = __builtin_amdgcn_readfirstlane(ht >> 6);
    double *acc = acc_all + (kPair ? half * kXsHalfRows : 0);
    long long *s_bnd = s_bnd_all[half];
    const v4u *key4 = reinterpret_cast<const v4u *>(a.key);
    const v2d *val2 = reinterpret_cast<const v2d *>(a.val);
    const int xcc = a.use_xcc ? xs_xcc_id() : (int)(blockIdx.x & 7);
    const long long t_entry = kTrace ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    // First item: static, block b takes index b/8 of queue b%8 (the hardware
    // deals blocks to the XCDs round robin, so queue b%8 is normally b's own
    // XCD's; placement only matters for speed).  Items beyond the static
    // share (a.dynamic) are claimed from the per-XCD queues, whose heads
    // start past the static items.  No atomic on the common path.
    int first = -1;
    {
        const int qb = (int)(blockIdx.x & 7), ib = (int)(blockIdx.x >> 3);
        if (ib < a.qstat[qb]) first = qb * a.qstride + ib;
    }
    // re-arm the other parity's heads for the next launch of this plan
    // (launches of one plan are ordered by their stream; this launch's heads
    // were armed by the previous one or by the plan build)
    if (blockIdx.x == 0 && threadIdx.x == 8)  // the fused reduce's task head
        __hip_atomic_store(&a.qreset[8], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x < 8) {
        int v = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) v = (int)threadIdx.x == k ? a.qstat[k] : v;
        __hip_atomic_store(&a.qreset[threadIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) {
        const int it = (first >= 0 || !a.dynamic) ? first : xs_claim(a, xcc);
        if (threadIdx.x == 0) s_item = it;
    }
    for (;;) {
        __syncthreads();
        const int slot = s_item;
        if (slot < 0) {  // workgroup-uniform
            if (a.fused) xs_reduce_phase<kBeta>(a, alpha, beta, y);
            if (kTrace && threadIdx.x == 0) {  // per-workgroup row: entry .. exit
                const long long ts = 1 + (long long)kXsTrace * atomicAdd((unsigned long long *)a.trace, 1ULL);
                a.trace[ts] = -2;
                a.trace[ts + 1] = -2;
                a.trace[ts + 2] = ((long long)blockIdx.x << 4) | xcc;
                a.trace[ts + 3] = t_entry;
                a.trace[ts + 4] = (long long)__builtin_amdgcn_s_memrealtime();
                a.trace[ts + 5] = 0;
            }
            return;
        }
        // sub = range << 8 | k: k+1 = wide sub-item of XCD k (its q groups
        // [kq, kq+q), partial slot k); 0 = narrow (all G groups, starting at
        // this XCD's first group and wrapping); -1 = nothing for this team
        // the team's item record (host-built per (slot, team)): sub, row0 |
        // nrows << 32, pbase, widx, then the range's G+1 block offsets -- one
        // round trip of independent loads instead of sub -> range -> blocks
        {
            const long long *rec = a.xrec + (long long)(2 * slot + half) * (a.G + 5);
            for (int j = ht; j < a.G + 5; j += NT) s_rec_all[half][j] = rec[j];
        }
        __syncthreads();
        long long *s_rec = s_rec_all[half];
        const int sub = (int)s_rec[0];
        XsRange R{};
        int k1 = 0, g0 = 0, n1 = 0;
        if (sub >= 0) {  // team-uniform
            k1 = sub & 255;
            R.row0 = (int)(s_rec[1] & 0xffffffffLL);
            R.nrows = (int)(s_rec[1] >> 32);
            R.pbase = s_rec[2];
            R.widx = (int)s_rec[3];
            const long long *bo = s_rec + 4;
            g0 = k1 ? (k1 - 1) * a.q : xcc * a.q;
            // s_bnd[j] = first chunk of group g0 + j: segment 1 is groups
            // [g0, g0+n1); a narrow sub-item's segment 2 is groups [0, g0)
            // at s_bnd + 128
            n1 = k1 ? a.q : a.G - g0;
            for (int r = ht; r < R.nrows; r += NT) acc[r] = 0.0;
            for (int j = ht; j <= n1; j += NT) s_bnd[j] = bo[g0 + j];
            if (!k1)
                for (int j = ht; j <= g0; j += NT) s_bnd[128 + j] = bo[j];
        }
        if (kDyn && ht == 0) {
            s_ctr[half][0] = 0;
            s_ctr[half][1] = 0;
            s_par[half][0] = sub;
            s_par[half][1] = k1;
            s_par[half][2] = g0;
            s_par[half][3] = n1;
        }
        if (kTrace && ht == 0) s_tend[half] = 0;
        __syncthreads();
        // claim the next item now; its result is consumed after the stream,
        // so the atomic's latency hides behind the stream's own loads
        int pre = 0;
        long long t0 = 0;
        if (threadIdx.x == 0) {
            if (a.dynamic) pre = atomicAdd(&a.qhead[xcc], 1);
            if (kTrace) t0 = (long long)__builtin_amdgcn_s_memrealtime();
        }
        if constexpr (kDyn) {
            // own segment 1, own segment 2 (narrow wrap), then the partner's
            // two: one inlined stream, its operands chosen per pass
            for (int p = 0; p < 4; ++p) {
                const int h = p < 2 ? half : 1 - half;
                const int seg = p & 1;
                const int hs = s_par[h][0], hk1 = s_par[h][1], hg0 = s_par[h][2], hn1 = s_par[h][3];
                if (hs < 0 || (seg && (hk1 || hg0 == 0))) continue;  // uniform
                const long long *hb = s_bnd_all[h] + (seg ? 128 : 0);
                const int hn = seg ? hg0 : hn1;
                xs_stream_dyn<kMode, kU>(key4, val2, a.kstride, a.vstride, &s_ctr[h][seg], hb[0], hb[hn], hb,
                                             seg ? 0 : hg0, a.Wg, x, acc_all + h * kXsHalfRows);
            }
        } else if (sub >= 0) {
            if (SA == SB || half == 0) {  // one inlined copy when the teams are equal
                xs_stream<kMode, SA>(key4, val2, a.kstride, a.vstride, s_bnd[0], s_bnd[n1], s_bnd, g0, a.Wg, x, acc, hwave);
                if (!k1 && g0 > 0)
                    xs_stream<kMode, SA>(key4, val2, a.kstride, a.vstride, s_bnd[128], s_bnd[128 + g0], s_bnd + 128, 0,
                                         a.Wg, x, acc, hwave);
            } else if constexpr (kPair && SA != SB) {
                xs_stream<kMode, SB>(key4, val2, a.kstride, a.vstride, s_bnd[0], s_bnd[n1], s_bnd, g0, a.Wg, x, acc, hwave);
                if (!k1 && g0 > 0)
                    xs_stream<kMode, SB>(key4, val2, a.kstride, a.vstride, s_bnd[128], s_bnd[128 + g0], s_bnd + 128, 0,
                                         a.Wg, x, acc, hwave);
            }
        }
        if (kTrace && (threadIdx.x & 63) == 0)  // debugging aid: this team's last wave
            atomicMax(&s_tend[half], (unsigned long long)__builtin_amdgcn_s_memrealtime());
        // A narrow sub-item alone in its item (the partner team empty: solo
        // items, SBLAS_XS_SOLO, or a leftover) is written by the whole
        // workgroup: its rows may fill both teams' LDS halves.
        const int s0 = kPair ? (int)s_rec_all[0][0] : -1;
        const bool solo = kPair && (int)s_rec_all[1][0] < 0 && s0 >= 0 && (s0 & 255) == 0;  // uniform
        constexpr int kTeamMin = kPair ? (SA < SB ? SA : SB) * 64 : kWG;
        constexpr int kEp = ((kWG == 1024 && !kPair ? kXsRows : kXsHalfRows) + kTeamMin - 1) / kTeamMin;
        // 4-wave teams (256-VGPR budget): a narrow epilogue's y loads are
        // issued before the barrier below, so their latency overlaps the
        // wait for the workgroup's last wave (at 128 VGPRs they spilled)
        constexpr bool kEarlyY = kBeta && kPair && kWG == 512;
        const bool ynarrow = solo || (sub >= 0 && !k1);
        const int et = solo ? (int)threadIdx.x : ht;
        const int eNT = solo ? kWG : NT;
        const long long rr = solo ? s_rec_all[0][1] : ((long long)(unsigned)R.row0 | ((long long)R.nrows << 32));
        const int row0 = (int)(rr & 0xffffffffLL), nrows = (int)(rr >> 32);
        double y0[kEp];
        if constexpr (kEarlyY) {
            if (ynarrow) {
#pragma unroll
                for (int e = 0; e < kEp; ++e) {
                    const int r = et + e * eNT;
                    y0[e] = r < nrows ? y[row0 + r] : 0.0;
                }
            }
        }
        if (threadIdx.x < 64) {
            const int own = __shfl(pre, 0, 64);
            const int it = !a.dynamic ? -1 : own < a.qlen[xcc] ? xcc * a.qstride + own : xs_claim(a, xcc);
            if (threadIdx.x == 0) s_item = it;
        }
        __syncthreads();
        if (kTrace && threadIdx.x == 0) {  // debugging aid (SBLAS_XS_TRACE): item timeline
            const long long ts = 1 + (long long)kXsTrace * atomicAdd((unsigned long long *)a.trace, 1ULL);
            a.trace[ts] = a.qitems[2 * slot];
            a.trace[ts + 1] = kPair ? a.qitems[2 * slot + 1] : -1;
            a.trace[ts + 2] = ((long long)blockIdx.x << 4) | xcc;
            a.trace[ts + 3] = t0;
            a.trace[ts + 4] = (long long)s_tend[0];
            a.trace[ts + 5] = (long long)s_tend[1];
        }
        if (sub >= 0 && k1) {
            // epilogue: a team owns <= kXsHalfRows rows, at most kEp per
            // thread; every y load of the thread is issued before the first
            // use, so the y latency is paid once, not once per row (a rolled
            // loop put ~10 us of serial latency on the end of every item).
            double *out = a.partial + R.pbase + (long long)(k1 - 1) * R.nrows;
            // agent-scope (sc1) stores when the fused reduce may read them
            // on another XCD (whose L2 is not coherent with this one);
            // plain stores otherwise: the kernel boundary before
            // k_xsort_reduce publishes them
            if (a.fused) {
#pragma unroll
                for (int e = 0; e < kEp; ++e) {
                    const int r = ht + e * NT;
                    if (r < R.nrows) __hip_atomic_store(out + r, acc[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            } else {
#pragma unroll
                for (int e = 0; e < kEp; ++e) {
                    const int r = ht + e * NT;
                    if (r < R.nrows) out[r] = acc[r];
                }
            }
        } else if (solo || sub >= 0) {
            // narrow: y = alpha * acc + beta * y over the sub-item's rows;
            // a solo item's <= kXsRows rows over all kWG threads, a team's
            // <= kXsHalfRows over its NT
            static_assert(!kPair || kEp * kWG >= kXsRows, "a solo item's rows fit the epilogue");
            const double *eacc = solo ? acc_all : acc;
            double *yr = y + row0;
            if constexpr (kBeta && !kEarlyY) {
#pragma unroll
                for (int e = 0; e < kEp; ++e) {
                    const int r = et + e * eNT;
                    y0[e] = r < nrows ? yr[r] : 0.0;
                }
            }
#pragma unroll
            for (int e = 0; e < kEp; ++e) {
                const int r = et + e * eNT;
                if (r < nrows) yr[r] = kBeta ? alpha * eacc[r] + beta * y0[e] : alpha * eacc[r];
            }
        }
        if (a.fused) {
            // count this team's wide sub-item in once every wave's partial
            // stores have drained (vmcnt(0), then the barrier)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (sub >= 0 && k1 && ht == 0)
                // release: this team's partials before its arrival
                (void)__hip_atomic_fetch_add(&a.arrive[R.widx], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        // (the barrier at the loop top orders these reads of acc before the
        // next item's zeroing, and s_bnd's reuse)
    }
}

// Wide ranges: y = alpha * sum_k partial[k] (+ beta*y), XCD slots in order.
// All 8 partial loads (and y) of a row are issued before the first add.
// wr[] holds the wide ranges' records in wide order: one scalar load ahead of
// the partials instead of an index and then the record.
template <bool kBeta>
__global__ __launch_bounds__(256) void k_xsort_reduce(const XsRange *__restrict__ wr,
                                                      const double *__restrict__ partial,
                                                      double alpha, double beta,
                                                      double *__restrict__ y)
{
    const XsRange R = wr[blockIdx.y];
    for (int r = blockIdx.x * 256 + threadIdx.x; r < R.nrows; r += gridDim.x * 256) {
        const double *p = partial + R.pbase + r;
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(p + (long long)k * R.nrows);
        double *yr = y + R.row0 + r;
        const double y0 = kBeta ? *yr : 0.0;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
        *yr = kBeta ? alpha * s + beta * y0 : alpha * s;
    }
}

void free_xsort_plan(sblas_csr_s &A)
{
    XsPlan &P = A.xs;
    (void)hipFree(P.ranges);
    (void)hipFree(P.wide);
    (void)hipFree(P.wranges);
    (void)hipFree(P.blk);
    (void)hipFree(P.key);  // P.val points into the same allocation
    (void)hipFree(P.qitems);
    (void)hipFree(P.qhead);
    (void)hipFree(P.partial);
    (void)hipFree(P.rtasks);
    (void)hipFree(P.xrec);
    (void)hipFree(P.arrive);
    A.xs = XsPlan{};
}

int build_xsort_plan(sblas_csr_s &A, hipStream_t s)
{
    if (A.xs.ready) return SBLAS_OK;
    DeviceGuard dg(A.device);
    XsPlan &P = A.xs;
    const int m = A.m, n = A.n;
    const long long nnz = A.nnz;
    const std::vector<int> &rp = A.h_rowptr;
    // SBLAS_XS_TIMING: plan-build phase times on stderr (seconds since the last mark)
    const bool timing = getenv("SBLAS_XS_TIMING") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto mark = [&](const char *phase) {
        if (!timing) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "xsort plan: %-10s %.3f s\n", phase, std::chrono::duration<double>(t - t_last).count());
        t_last = t;
    };

    // column groups: G = 8q groups of Wg < 2^18 columns (the all-ones column
    // field is the padding key) and ~1 MiB of x (an XCD's current group plus
    // the entry stream must fit its 4 MiB L2)
    const long long wmax = (1LL << kXsColBits) - 1;
    const long long ng = ((long long)std::max(n, 1) + wmax - 1) / wmax;
    const long long nmib = ((long long)std::max(n, 1) * 8 + (1LL << 20) - 1) >> 20;
    P.q = (int)std::max<long long>({1LL, (ng + 7) / 8, (nmib + 7) / 8});
    if (const char *e = getenv("SBLAS_XS_Q"))  // experiments: override, >= the width bound
        P.q = (int)std::max<long long>({1LL, (ng + 7) / 8, (long long)atoi(e)});
    P.G = 8 * P.q;
    if (P.G > 127) {
        set_error("xsort: n = %d needs %d column groups (> 127)", n, P.G);
        return SBLAS_ERR_UNSUPPORTED;
    }
    P.Wg = (int)std::max<long long>(1, ((long long)std::max(n, 1) + P.G - 1) / P.G);
    const int G = P.G, Wg = P.Wg;

    // workgroup shape (SBLAS_XS_WG / SBLAS_XS_PAIR select the experiments'
    // alternatives); resident workgroups = item slots, a paired item holds
    // two sub-items
    // Workgroup: two 4-wave teams (512 threads, 2 waves per SIMD, up to 256
    // VGPRs a wave) -- the register budget lets the compiler keep more of
    // the stream in flight than two 8-wave teams (1024 threads, 128 VGPRs) or
    // two 6-wave teams (768, ~170): with 2 chunks per claim, config 2 N = 1 /
    // 2 / 4 / 8 150.6-152.5 / 96.4-96.7 / 65.5-65.6 / 40.7-40.8 us against
    // 153.0-153.3 / 99.1 / 66.3-66.9 / 42.1-42.5, 27-point 128^3 117 vs 121,
    // 7-point 160^3 83 vs 85, R-MAT equal (profiles/r05/wg512p/).
    // SBLAS_XS_WG = 512p (default) / 768 / 1024 forces a paired shape, 512
    // two unpaired workgroups per CU.
    const char *wge = getenv("SBLAS_XS_WG");
    const bool pair512 = !wge || strcmp(wge, "512p") == 0;
    P.nt = pair512 ? 512 : atoi(wge) == 512 ? 512 : atoi(wge) == 768 ? 768 : kXsThreads;
    P.pair = (P.nt >= 768 || pair512) && !(getenv("SBLAS_XS_PAIR") && atoi(getenv("SBLAS_XS_PAIR")) == 0);
    if (P.nt == 768 && !P.pair) P.nt = kXsThreads;
    if (pair512 && !P.pair) {  // SBLAS_XS_PAIR=0 with the default shape: the unpaired 1024 form
        P.nt = kXsThreads;
    }
    if ((P.nt == 768 || (P.nt == 512 && P.pair)) && getenv("SBLAS_XS_TRACE")) P.nt = kXsThreads;  // trace twins: 1024
    P.split = 8;  // waves of the first (narrow) team of a pair: 5, 6, 7 or 8
    if (const char *e = getenv("SBLAS_XS_SPLIT")) P.split = std::min(8, std::max(5, atoi(e)));
    P.dyn = P.pair && P.split == 8 && !(getenv("SBLAS_XS_DYN") && atoi(getenv("SBLAS_XS_DYN")) == 0);
    if ((P.nt == 768 || (P.nt == 512 && P.pair)) && !P.dyn) P.nt = kXsThreads;  // dynamic-claim kernels only
    int dev = 0, ncu = 0, per_cu = 0;
    SBLAS_HIP(hipGetDevice(&dev));
    SBLAS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    if (P.nt == 512 && P.pair)
        SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, k_spmv_xsort<true, 0, 512, true, 4, false, true, 2>, 512, 0));
    else if (P.nt == 512)
        SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, k_spmv_xsort<true, 0, 512, false>, 512, 0));
    else if (P.nt == 768)
        SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, k_spmv_xsort<true, 0, 768, true, 6, false, true, 2>, 768, 0));
    else
        SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, k_spmv_xsort<true, 0, kXsThreads, true>, kXsThreads, 0));
    const int resident = std::max(1, ncu * std::max(per_cu, 1));
    int kper = 1;
    if (const char *e = getenv("SBLAS_XS_K")) kper = std::max(1, atoi(e));
    const long long slots = (long long)resident * kper * (P.pair ? 2 : 1);  // sub-items
    // every range wide (8 XCD-local sub-items + partials per row) on small
    // matrices: a rank's slice of the uniform config 2 at N = 8 (5.0M
    // entries) 47.0 -> 41.8 us, N = 16 (2.5M) 33.8 -> 29.9, but N = 4 (9.9M)
    // 66.8 -> 104 (profiles/r05/sweep2/): the partials (16 B per row and XCD)
    // outweigh XCD-local gathers beyond ~6M entries.  SBLAS_XS_ALLWIDE=0/1 forces.
    const char *awe = getenv("SBLAS_XS_ALLWIDE");
    const bool all_wide = awe ? atoi(awe) != 0 : nnz <= kXsAllWideMaxNnz;
    const bool no_wide = getenv("SBLAS_XS_NOWIDE") && atoi(getenv("SBLAS_XS_NOWIDE")) != 0;
    const bool nosort = getenv("SBLAS_XS_NOSORT") && atoi(getenv("SBLAS_XS_NOSORT")) != 0;
    int rows_cap = (P.pair || P.nt == 512) ? kXsHalfRows : kXsItemRows;
    if (const char *e = getenv("SBLAS_XS_ROWS")) rows_cap = std::max(1, std::min(rows_cap, atoi(e)));
    // solo narrow items (SBLAS_XS_SOLO=1, paired dynamic kernel): a narrow
    // range is an item of its own -- both teams' waves and all 16,384 LDS
    // rows -- so its blocks are twice as dense (fewer x line requests per
    // entry); wide ranges still pair (wide, wide) at 8,192 rows a team
    // Chosen by default when >= 40% of the rows are empty (power-law graphs:
    // an empty row spends an accumulator row, so 16,384 rows per light range
    // hold what 8,192 would without them): R-MAT scale 21 (50% empty) 158.8
    // -> 147.3 us; config 2 and the stencils have none and keep pairs (solo
    // there: 146.7 vs 131 us; profiles/r04/rmat/).  SBLAS_XS_SOLO=0/1 forces.
    {
        long long empty = 0;
        for (int r = 0; r < m; ++r) empty += rp[r + 1] == rp[r];
        const char *se = getenv("SBLAS_XS_SOLO");
        const bool want = se ? atoi(se) != 0 : (m > 0 && 5 * empty >= 2LL * m);
        P.solo = P.pair && P.dyn && want;
    }
    const int nrows_cap = P.solo ? kXsItemRows : rows_cap;  // narrow ranges
    const double nfac = P.solo ? 2.0 : 1.0;             // a narrow range's cost, in sub-item caps

    // Cost model (work units ~ one streamed entry): a sub-item's time is its
    // entries plus lambda per distinct x line its gathers touch; with uniform
    // columns a block of c entries over L lines touches L*(1 - exp(-c/L))
    // lines.  A narrow sub-item spreads its entries over all of x (G*Lg
    // lines), a wide one its 1/8 share over its XCD's q groups.  lambda = 1.0
    // is the best of a sweep (0.3 .. 1.7) on config 2 with the paired,
    // chunked kernel.
    double lam = 1.0;
    if (const char *e = getenv("SBLAS_XS_LAMBDA")) lam = atof(e);
    // at most this fraction of the entries goes to wide ranges (the rest of
    // the heavy rows is cut into narrow ranges), so that a paired item's two
    // halves carry similar work
    double wbudget = 1.0;
    if (const char *e = getenv("SBLAS_XS_WBUDGET")) wbudget = atof(e);
    const double Lg = std::max(1.0, Wg / 16.0);  // 128-B lines of one group's x slice
    auto narrow_cost = [&](double c) { return c + lam * G * Lg * (1.0 - std::exp(-c / (G * Lg))); };
    auto wide_cost = [&](double c) {
        const double ci = c / 8.0;
        return ci + lam * P.q * Lg * (1.0 - std::exp(-ci / (P.q * Lg)));
    };
    // Row ranges: from row r, a wide candidate takes <= rows_cap rows while
    // one of its 8 sub-items costs <= cap.  It is WIDE (8 sub-items + 8
    // partials per row) when it holds more than one narrow sub-item's work and
    // its rows average >= 16 entries (the partials then cost <= 8 B per
    // entry); otherwise a narrow range of cost <= cap is cut afresh from r.
    std::vector<XsRange> ranges;
    auto build_ranges = [&](double cap) {
        ranges.clear();
        // cut(r): the first row always, then rows while the range's cost stays
        // <= cap, at most rows_cap rows.  The cost grows strictly with the
        // entry count rp[e] - rp[r], so the end is a binary search over e
        // (O(log m) cost evaluations per range instead of one per row: the
        // cap search below runs build_ranges many times over all m rows).
        auto cut = [&](int r, bool wide, long long &cnt) {
            const int start = r;
            const int emax = (int)std::min<long long>(m, (long long)start + (wide ? rows_cap : nrows_cap));
            auto fits = [&](int e) {
                const double c = (double)(rp[e] - rp[start]);
                return wide ? wide_cost(c) <= cap : narrow_cost(c) <= nfac * cap;
            };
            int lo = start + 1, hi = emax;  // answer in [lo, hi]; lo always taken
            while (lo < hi) {
                const int mid = lo + (hi - lo + 1) / 2;
                if (fits(mid)) lo = mid;
                else hi = mid - 1;
            }
            cnt = rp[lo] - rp[start];
            return lo;
        };
        int r = 0;
        long long wide_entries = 0;
        while (r < m) {
            long long cnt;
            int e = cut(r, true, cnt);
            const bool wide = cnt > 0 && !no_wide &&
                              (all_wide || (narrow_cost((double)cnt) > nfac * cap && cnt >= 16LL * (e - r) &&
                                            (double)(wide_entries + cnt) <= wbudget * (double)nnz));
            if (wide) wide_entries += cnt;
            if (!wide) e = cut(r, false, cnt);
            XsRange R{};
            R.row0 = r;
            R.nrows = e - r;
            R.wide = wide ? 1 : 0;
            ranges.push_back(R);
            r = e;
        }
    };
    auto count_subs = [&]() {
        long long c = 0;
        for (const XsRange &R : ranges) c += R.wide ? 8 : P.solo ? 2 : 1;
        return c;
    };
    // grow the sub-item cost until the sub-items fit the resident grid (a
    // second round for a few items would double the kernel's tail)
    double cap = narrow_cost((double)nnz) / (double)slots;
    if (const char *e = getenv("SBLAS_XS_WSTAR")) cap = std::max(1.0, atof(e));
    // Ranges hold at most rows_cap rows, so once ceil(m / rows_cap) exceeds
    // the slots no cap can fit them: stop there (and after 50 growth steps
    // without fewer sub-items) instead of 400 O(m) passes.  Leftover
    // sub-items are still correct: the grid claims them in a second round.
    const long long min_ranges = ((long long)m + rows_cap - 1) / rows_cap;
    long long best_subs = -1;
    for (int it = 0, flat = 0; it < 400; ++it) {
        build_ranges(cap);
        const long long subs = count_subs();
        if (subs <= slots || getenv("SBLAS_XS_WSTAR") || min_ranges > slots) break;
        flat = (best_subs >= 0 && subs >= best_subs) ? flat + 1 : 0;
        if (flat >= 50) break;
        if (best_subs < 0 || subs < best_subs) best_subs = subs;
        cap *= 1.02;
    }
    const int I = (int)ranges.size();
    if ((long long)I >= (1LL << 23)) {
        set_error("xsort: %d row ranges (> 2^23)", I);
        return SBLAS_ERR_UNSUPPORTED;
    }

    mark("planner");
    // host copies of the CSR entries (uninitialised: the copies fill them)
    std::unique_ptr<int[]> hcol(new int[(size_t)std::max<long long>(nnz, 1)]);
    std::unique_ptr<double[]> hval(new double[(size_t)std::max<long long>(nnz, 1)]);
    if (nnz) {
        SBLAS_HIP(hipMemcpy(hcol.get(), A.col, sizeof(int) * nnz, hipMemcpyDeviceToHost));
        SBLAS_HIP(hipMemcpy(hval.get(), A.val, sizeof(double) * nnz, hipMemcpyDeviceToHost));
    }

    mark("d2h");
    // pass 1: every block (range, group) bucketed and sorted by (column, row)
    // once, kept for the fill (both key formats are sized from it).  One
    // range per task for the bucketing (a wide range holds ~13x a narrow
    // one's entries, and they sit together at the heavy rows), then the
    // blocks are sorted as tasks of their own.
    const size_t nblk = (size_t)I * G;
    std::vector<std::vector<std::pair<uint32_t, double>>> bk(nblk);
    bool bad = false;
#pragma omp parallel for schedule(dynamic, 1) reduction(|| : bad)
    for (int i = 0; i < I; ++i) {
        const XsRange &R = ranges[i];
        std::vector<int> cnt(G, 0);
        for (int e = rp[R.row0]; e < rp[R.row0 + R.nrows]; ++e) {
            const int c = hcol[e];
            if (c >= 0 && c < n) ++cnt[c / Wg];
        }
        for (int g = 0; g < G; ++g) bk[(size_t)i * G + g].reserve(cnt[g]);
        for (int r = R.row0; r < R.row0 + R.nrows; ++r) {
            for (int e = rp[r]; e < rp[r + 1]; ++e) {
                const int c = hcol[e];
                if (c < 0 || c >= n) {
                    bad = true;
                    continue;
                }
                const int g = c / Wg;
                const uint32_t cp = (uint32_t)(c - g * Wg), lr = (uint32_t)(r - R.row0);
                if ((long long)cp >= wmax || lr >= (uint32_t)(R.wide ? rows_cap : nrows_cap)) bad = true;
                bk[(size_t)i * G + g].push_back({(cp << kXsRowBits) | lr, hval[e]});
            }
        }
    }
    if (!nosort) {
#pragma omp parallel for schedule(dynamic, 4)
        for (long long k = 0; k < (long long)nblk; ++k) {
            auto &bb = bk[(size_t)k];
            std::stable_sort(bb.begin(), bb.end(),
                             [](const std::pair<uint32_t, double> &u,
                                const std::pair<uint32_t, double> &v) { return u.first < v.first; });
        }
    }
    if (bad) {
        set_error("xsort: column index out of [0, n) or key overflow");
        return SBLAS_ERR_INVALID;
    }
    std::vector<long long> blk(nblk + 1, 0);  // chunk offsets
    for (size_t k = 0; k < nblk; ++k)
        blk[k + 1] = blk[k] + ((long long)bk[k].size() + kXsChunk - 1) / kXsChunk;
    const long long nchunks = blk.back();

    mark("pass1");
    // pass 2: fill every chunk (lane-transposed, header comment)
    // interleaved (default): per chunk 1 KiB of keys then 2 KiB of values,
    // ONE 3-KiB run in HBM; split (SBLAS_XS_KV=0): all keys, then all values
    const bool kv = !(getenv("SBLAS_XS_KV") && atoi(getenv("SBLAS_XS_KV")) == 0);
    const size_t cbytes = (size_t)kXsChunk * (sizeof(uint32_t) + sizeof(double));
    // every byte of every chunk is written by the fill below: no zeroing pass
    struct HostBuf {
        std::unique_ptr<unsigned char[]> p;
        size_t n;
        unsigned char *data() const { return p.get(); }
        size_t size() const { return n; }
    };
    const size_t hb_n = (size_t)std::max<long long>(nchunks, 1) * cbytes;
    const HostBuf hbuf{std::unique_ptr<unsigned char[]>(new unsigned char[hb_n]), hb_n};
    auto chunk_keys = [&](long long c) {
        return (uint32_t *)(hbuf.data() + (kv ? (size_t)c * cbytes : (size_t)c * kXsChunk * sizeof(uint32_t)));
    };
    auto chunk_vals = [&](long long c) {
        return (double *)(hbuf.data() + (kv ? (size_t)c * cbytes + kXsChunk * sizeof(uint32_t)
                                            : (size_t)std::max<long long>(nchunks, 1) * kXsChunk * sizeof(uint32_t) +
                                                  (size_t)c * kXsChunk * sizeof(double)));
    };
    P.kstride = kv ? (int)(cbytes / 16) : kXsChunk * 4 / 16;
    P.vstride = kv ? (int)(cbytes / 16) : kXsChunk * 8 / 16;
#pragma omp parallel for schedule(dynamic, 64)
    for (long long k = 0; k < (long long)nblk; ++k) {
        const auto &bb = bk[(size_t)k];
        const long long c0 = blk[(size_t)k], c1 = blk[(size_t)k + 1];
        for (long long c = c0; c < c1; ++c) {
            uint32_t *kc = chunk_keys(c);
            double *vc = chunk_vals(c);
            for (int p = 0; p < kXsChunk; ++p) {
                const long long src = (c - c0) * kXsChunk + p;
                const bool in = src < (long long)bb.size();
                const int l = p & 63, j = p >> 6;
                kc[4 * l + j] = in ? bb[src].first : kXsPad;
                vc[(j < 2 ? 0 : 128) + 2 * l + (j & 1)] = in ? bb[src].second : 0.0;
            }
        }
    }
    { std::vector<std::vector<std::pair<uint32_t, double>>>().swap(bk); }

    mark("pass2");
    // sub-items, wide partial slots, then items (pairs) in XCD queues
    std::vector<int> wide, nsub;
    std::vector<std::vector<int>> wsub(8);
    long long pbase = 0;
    std::vector<int2> rtasks;  // fused reduce: (range, first row) per kXsThreads rows
    for (int i = 0; i < I; ++i) {
        XsRange &R = ranges[i];
        R.widx = -1;
        if (R.wide) {
            R.pbase = pbase;
            pbase += 8LL * R.nrows;
            R.widx = (int)wide.size();
            for (int r0 = 0; r0 < R.nrows; r0 += kXsThreads) rtasks.push_back(make_int2(i, r0));
            wide.push_back(i);
            for (int k = 0; k < 8; ++k) wsub[k].push_back((i << 8) | (k + 1));
        } else {
            nsub.push_back(i << 8);
        }
    }
    std::vector<std::vector<std::pair<int, int>>> q(8);
    if (!P.pair) {
        for (int k = 0; k < 8; ++k)
            for (int w : wsub[k]) q[k].push_back({w, -1});
        for (size_t j = 0; j < nsub.size(); ++j) q[j % 8].push_back({nsub[j], -1});
        // longest first (estimated cost): the dynamic claims then end evenly
        auto cost = [&](int sub) {
            const XsRange &R = ranges[sub >> 8];
            const double c = (double)(rp[R.row0 + R.nrows] - rp[R.row0]);
            return (sub & 255) ? wide_cost(c) : narrow_cost(c);
        };
        for (int k = 0; k < 8; ++k)
            std::stable_sort(q[k].begin(), q[k].end(),
                             [&](const std::pair<int, int> &u, const std::pair<int, int> &v) {
                                 return cost(u.first) > cost(v.first);
                             });
    } else if (P.solo) {
        // solo narrow items (narrow, -1); wide sub-items paired within their
        // XCD; each queue alternates the two kinds
        std::vector<std::vector<std::pair<int, int>>> qn(8), qw(8);
        for (size_t j = 0; j < nsub.size(); ++j) qn[j % 8].push_back({nsub[j], -1});
        for (int k = 0; k < 8; ++k)
            for (size_t j = 0; j < wsub[k].size(); j += 2)
                qw[k].push_back({wsub[k][j], j + 1 < wsub[k].size() ? wsub[k][j + 1] : -1});
        for (int k = 0; k < 8; ++k)
            for (size_t j = 0; j < std::max(qn[k].size(), qw[k].size()); ++j) {
                if (j < qn[k].size()) q[k].push_back(qn[k][j]);
                if (j < qw[k].size()) q[k].push_back(qw[k][j]);
            }
    } else {
        // a narrow (gather-bound) with a wide (stream-bound) sub-item where
        // possible, the XCDs interleaved so the narrow ones spread evenly;
        // leftovers pair among themselves (wide ones within their XCD)
        size_t ni = 0;
        std::vector<std::vector<int>> wleft(8);
        for (size_t j = 0;; ++j) {
            bool any = false;
            for (int k = 0; k < 8; ++k) {
                if (j >= wsub[k].size()) continue;
                any = true;
                if (ni < nsub.size()) q[k].push_back({nsub[ni++], wsub[k][j]});
                else wleft[k].push_back(wsub[k][j]);
            }
            if (!any) break;
        }
        for (int k = 0; k < 8; ++k)
            for (size_t j = 0; j < wleft[k].size(); j += 2)
                q[k].push_back({wleft[k][j], j + 1 < wleft[k].size() ? wleft[k][j + 1] : -1});
        // leftover light sub-items: two to an item only as far as the grid
        // needs it; the rest run alone (both teams on one sub-item), so an
        // item never carries twice a light sub-item's work while workgroups
        // idle (power-law matrices: most rows light, few heavy sub-items)
        long long items_now = 0;
        for (int k = 0; k < 8; ++k) items_now += (long long)q[k].size();
        const long long left = (long long)(nsub.size() - ni);
        const long long free_slots = std::max<long long>(0, (long long)resident - items_now);
        long long npairs = std::max<long long>(0, left - free_slots);  // items = left - npairs <= free
        if (2 * npairs > left) npairs = left / 2;
        for (int t = 0; ni < nsub.size(); ++t) {
            const int a0 = nsub[ni++];
            const int a1 = (npairs > 0 && ni < nsub.size()) ? nsub[ni++] : -1;
            if (a1 >= 0) --npairs;
            q[t % 8].push_back({a0, a1});
        }
    }
    if (timing) {
        long long empty_subs = 0;
        for (int i : wide)
            for (int k = 0; k < 8; ++k)
                empty_subs += blk[(size_t)i * G + (size_t)(k + 1) * P.q] == blk[(size_t)i * G + (size_t)k * P.q];
        fprintf(stderr, "xsort plan: %d ranges, %zu wide (%lld of their %zu sub-items empty), %zu narrow, "
                        "%lld chunks, G %d, q %d, solo %d\n",
                I, wide.size(), empty_subs, 8 * wide.size(), nsub.size(), nchunks, G, P.q, (int)P.solo);
    }
    P.nranges = I;
    P.nwide = (int)wide.size();
    P.nchunks = nchunks;
    P.qstride = 1;
    P.nitems = 0;
    for (int k = 0; k < 8; ++k) {
        P.qlen[k] = (int)q[k].size();
        P.qstride = std::max(P.qstride, P.qlen[k]);
        P.nitems += P.qlen[k];
    }
    P.grid = std::min(P.nitems, resident);
    // Chunks per dynamic claim (SBLAS_XS_U forces it).  Finer claims balance
    // the waves and shorten the last stage (rounds 2-4, correlated generator:
    // U = 1 won at every N, profiles/r02/slice/); on the uniform matrix two
    // chunks per claim win where waves stream many chunks: the uniform
    // config 2 (~38 chunks per wave) 159.2 -> 156.2 us (three alternating
    // A/B pairs, profiles/r05/sweep2/); one on small plans (N = 8 slice, ~5
    // per wave: 46.9 vs 51.5, profiles/r05/sweep/).
    {
        const char *ue = getenv("SBLAS_XS_U");
        const double per_wave = (double)nchunks / ((double)std::max(P.nitems, 1) * (P.nt / 64));
        // (two 4-wave teams: 2 everywhere, the N = 8 slice 42.7-43.7 -> 40.7-40.8 us)
        P.u = ue ? std::max(1, std::min(4, atoi(ue))) : (P.nt == 512 && P.pair) ? 2 : (per_wave >= 24.0 ? 2 : 1);
    }
    int nstat = 0;
    for (int k = 0; k < 8; ++k) {
        const int blocks_k = P.grid > k ? (P.grid - k + 7) / 8 : 0;  // blocks b < grid with b % 8 == k
        P.qstat[k] = std::min(P.qlen[k], blocks_k);
        nstat += P.qstat[k];
    }
    P.dynamic = nstat < P.nitems ? 1 : 0;
    {  // most chunks of one item (both sub-items), for the plan's statistics
        auto nch = [&](int sub) -> long long {
            if (sub < 0) return 0;
            const size_t i = (size_t)(sub >> 8) * G;
            const int k1 = sub & 255;
            return k1 ? blk[i + (size_t)k1 * P.q] - blk[i + (size_t)(k1 - 1) * P.q] : blk[i + G] - blk[i];
        };
        long long mc = 0;
        for (int k = 0; k < 8; ++k)
            for (const auto &it : q[k]) mc = std::max(mc, nch(it.first) + nch(it.second));
        P.maxc = (int)std::min<long long>(mc, 1 << 30);
    }
    std::vector<int> qflat((size_t)16 * P.qstride, -1);
    for (int k = 0; k < 8; ++k)
        for (size_t j = 0; j < q[k].size(); ++j) {
            qflat[2 * ((size_t)k * P.qstride + j)] = q[k][j].first;
            qflat[2 * ((size_t)k * P.qstride + j) + 1] = q[k][j].second;
        }


    SBLAS_HIP(hipMalloc(&P.ranges, sizeof(XsRange) * std::max(I, 1)));
    SBLAS_HIP(hipMalloc(&P.wide, sizeof(int) * std::max<size_t>(wide.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.wranges, sizeof(XsRange) * std::max<size_t>(wide.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.blk, sizeof(long long) * blk.size()));
    SBLAS_HIP(hipMalloc(&P.key, hbuf.size()));
    P.val = (double *)((unsigned char *)P.key + ((unsigned char *)chunk_vals(0) - hbuf.data()));
    SBLAS_HIP(hipMalloc(&P.qitems, sizeof(int) * qflat.size()));
    SBLAS_HIP(hipMalloc(&P.qhead, sizeof(int) * 32));  // [2 parities][8 claim heads + pad]
    {
        std::vector<int> h(32, 0);
        for (int k = 0; k < 8; ++k) h[k] = h[16 + k] = P.qstat[k];
        SBLAS_HIP(hipMemcpy(P.qhead, h.data(), sizeof(int) * 32, hipMemcpyHostToDevice));
    }
    SBLAS_HIP(hipMalloc(&P.partial, sizeof(double) * std::max<long long>(pbase, 1)));
    // fused reduce (SBLAS_XS_FUSE=1; needs the 1024-thread workgroup, one
    // task = kXsThreads rows).  Not the default: on config 2 its claim ->
    // poll -> load chain lands ~18 us of latency on the kernel's tail
    // against 6 us for the separate k_xsort_reduce launch.
    P.fused = P.nt == kXsThreads && !wide.empty() && getenv("SBLAS_XS_FUSE") &&
              atoi(getenv("SBLAS_XS_FUSE")) != 0;
    P.nrtasks = (int)rtasks.size();
    SBLAS_HIP(hipMalloc(&P.rtasks, sizeof(int2) * std::max<size_t>(rtasks.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.arrive, sizeof(unsigned) * std::max<size_t>(wide.size(), 1)));
    SBLAS_HIP(hipMemset(P.arrive, 0, sizeof(unsigned) * std::max<size_t>(wide.size(), 1)));
    if (!rtasks.empty())
        SBLAS_HIP(hipMemcpy(P.rtasks, rtasks.data(), sizeof(int2) * rtasks.size(), hipMemcpyHostToDevice));
    P.epoch = 0;
    if (I) SBLAS_HIP(hipMemcpy(P.ranges, ranges.data(), sizeof(XsRange) * I, hipMemcpyHostToDevice));
    if (!wide.empty()) {
        SBLAS_HIP(hipMemcpy(P.wide, wide.data(), sizeof(int) * wide.size(), hipMemcpyHostToDevice));
        std::vector<XsRange> wr;
        for (int i : wide) wr.push_back(ranges[(size_t)i]);
        SBLAS_HIP(hipMemcpy(P.wranges, wr.data(), sizeof(XsRange) * wr.size(), hipMemcpyHostToDevice));
    }
    SBLAS_HIP(hipMemcpy(P.blk, blk.data(), sizeof(long long) * blk.size(), hipMemcpyHostToDevice));
    if (nchunks) {
        SBLAS_HIP(hipMemcpy(P.key, hbuf.data(), hbuf.size(), hipMemcpyHostToDevice));
    }
    mark("h2d");
    SBLAS_HIP(hipMemcpy(P.qitems, qflat.data(), sizeof(int) * qflat.size(), hipMemcpyHostToDevice));
    {
        const size_t rl = (size_t)G + 5;
        std::vector<long long> xrec(qflat.size() * rl, -1);
        for (size_t s2 = 0; s2 < qflat.size(); ++s2) {
            const int sub = qflat[s2];
            long long *r = xrec.data() + s2 * rl;
            r[0] = sub;
            if (sub < 0) continue;
            const XsRange &R = ranges[(size_t)(sub >> 8)];
            r[1] = (long long)(unsigned)R.row0 | ((long long)R.nrows << 32);
            r[2] = R.pbase;
            r[3] = R.widx;
            for (int g = 0; g <= G; ++g) r[4 + g] = blk[(size_t)(sub >> 8) * G + g];
        }
        SBLAS_HIP(hipMalloc(&P.xrec, sizeof(long long) * xrec.size()));
        SBLAS_HIP(hipMemcpy(P.xrec, xrec.data(), sizeof(long long) * xrec.size(), hipMemcpyHostToDevice));
    }
    mark("tail");
    P.ready = true;
    return SBLAS_OK;
}

int launch_spmv_xsort(const sblas_csr_s &A, double alpha, const double *x, double beta,
                      double *y, hipStream_t s)
{
    const XsPlan &P = A.xs;
    if (!P.ready) return SBLAS_ERR_INVALID;
    if (A.m == 0 || P.nitems == 0) return SBLAS_OK;
    static const int use_xcc = [] {
        const char *e = getenv("SBLAS_XS_XCC");
        return e ? atoi(e) : 1;
    }();
    static const int mode = [] {
        const char *e = getenv("SBLAS_XS_MODE");
        return e ? atoi(e) : 0;
    }();
    XsArgs a{};
    a.ranges = P.ranges;
    a.blk = P.blk;
    a.key = P.key;
    a.val = P.val;
    a.kstride = P.kstride;
    a.vstride = P.vstride;
    a.qitems = P.qitems;
    a.xrec = P.xrec;
    // parity and epoch advance only once the launch is known to be queued: a
    // launch that failed never re-armed the other parity's heads, so the
    // next launch must reuse this parity's (still armed) heads
    a.qhead = P.qhead + 16 * P.parity;        // this launch's claim heads
    a.qreset = P.qhead + 16 * (1 - P.parity);  // re-armed for the next launch
    a.partial = P.partial;
    for (int k = 0; k < 8; ++k) {
        a.qlen[k] = P.qlen[k];
        a.qstat[k] = P.qstat[k];
    }
    a.dynamic = P.dynamic;
    a.fused = P.fused ? 1 : 0;
    a.rtasks = P.rtasks;
    a.nrtasks = P.nrtasks;
    a.arrive = P.arrive;
    a.epoch = (unsigned)(P.epoch + (P.fused ? 1 : 0));
    a.qstride = P.qstride;
    a.G = P.G;
    a.q = P.q;
    a.Wg = P.Wg;
    a.use_xcc = use_xcc;
    using K = void (*)(const XsArgs, const double *, double, double, double *);
    K kern;
    const bool b = beta != 0.0;
    constexpr int W = kXsThreads;
    if (P.nt == 512 && !P.pair) {
        if (mode == 1) kern = b ? k_spmv_xsort<true, 1, 512, false> : k_spmv_xsort<false, 1, 512, false>;
        else if (mode == 2) kern = b ? k_spmv_xsort<true, 2, 512, false> : k_spmv_xsort<false, 2, 512, false>;
        else if (mode == 3) kern = b ? k_spmv_xsort<true, 3, 512, false> : k_spmv_xsort<false, 3, 512, false>;
        else kern = b ? k_spmv_xsort<true, 0, 512, false> : k_spmv_xsort<false, 0, 512, false>;
    } else if (P.pair) {
        if (mode == 1) kern = b ? k_spmv_xsort<true, 1, W, true> : k_spmv_xsort<false, 1, W, true>;
        else if (mode == 2) kern = b ? k_spmv_xsort<true, 2, W, true> : k_spmv_xsort<false, 2, W, true>;
        else if (mode == 3) kern = b ? k_spmv_xsort<true, 3, W, true> : k_spmv_xsort<false, 3, W, true>;
        else if (P.split == 6) kern = b ? k_spmv_xsort<true, 0, W, true, 6> : k_spmv_xsort<false, 0, W, true, 6>;
        else if (P.split == 5) kern = b ? k_spmv_xsort<true, 0, W, true, 5> : k_spmv_xsort<false, 0, W, true, 5>;
        else if (P.split == 7) kern = b ? k_spmv_xsort<true, 0, W, true, 7> : k_spmv_xsort<false, 0, W, true, 7>;
        else if (P.dyn) kern = b ? k_spmv_xsort<true, 0, W, true, 8, false, true> : k_spmv_xsort<false, 0, W, true, 8, false, true>;
        else kern = b ? k_spmv_xsort<true, 0, W, true> : k_spmv_xsort<false, 0, W, true>;
    } else {
        kern = b ? k_spmv_xsort<true, 0, W, false> : k_spmv_xsort<false, 0, W, false>;
    }
    const int xu = P.u;  // chunks per dynamic claim (planner; SBLAS_XS_U)
    if (P.pair && P.dyn && !b && xu == 1 && mode == 0)
        kern = k_spmv_xsort<false, 0, W, true, 8, false, true, 1>;
    if (P.pair && P.dyn && b && (xu != kXsUnroll || (mode & 28))) {
#define XS_DYN(M, U) k_spmv_xsort<true, M, W, true, 8, false, true, U>
        const int mm = mode & 6;
        if (xu == 1) kern = mm == 0 ? XS_DYN(0, 1) : mm == 2 ? XS_DYN(2, 1) : mm == 4 ? XS_DYN(4, 1) : XS_DYN(6, 1);
        else if (xu == 3) kern = mm == 0 ? XS_DYN(0, 3) : mm == 2 ? XS_DYN(2, 3) : mm == 4 ? XS_DYN(4, 3) : XS_DYN(6, 3);
        else if (xu == 4) kern = mm == 0 ? XS_DYN(0, 4) : mm == 2 ? XS_DYN(2, 4) : mm == 4 ? XS_DYN(4, 4) : XS_DYN(6, 4);
        else kern = mm == 4 ? XS_DYN(4, 2) : XS_DYN(6, 2);
        if ((mode & ~1) == 8 && xu == 1) kern = (mode & 1) ? XS_DYN(9, 1) : XS_DYN(8, 1);  // experiment: no gathers
        if (mode == 16 && xu == 1) kern = XS_DYN(16, 1);  // experiment: L2-resident gathers
#undef XS_DYN
    }
    if (P.nt == 512 && P.pair) {  // 4 + 4 waves (the default shape)
        const int xu = P.u;
        if (b) kern = xu == 1 ? k_spmv_xsort<true, 0, 512, true, 4, false, true, 1>
                      : xu == 3 ? k_spmv_xsort<true, 0, 512, true, 4, false, true, 3>
                      : xu == 4 ? k_spmv_xsort<true, 0, 512, true, 4, false, true, 4>
                                : k_spmv_xsort<true, 0, 512, true, 4, false, true, 2>;
        else kern = xu == 1 ? k_spmv_xsort<false, 0, 512, true, 4, false, true, 1>
                    : xu == 3 ? k_spmv_xsort<false, 0, 512, true, 4, false, true, 3>
                    : xu == 4 ? k_spmv_xsort<false, 0, 512, true, 4, false, true, 4>
                              : k_spmv_xsort<false, 0, 512, true, 4, false, true, 2>;
    }
    if (P.nt == 768) {  // 6 + 6 waves (SBLAS_XS_WG=768), U = P.u chunks per claim
        const int xu = P.u;
        if (b) kern = xu == 1 ? k_spmv_xsort<true, 0, 768, true, 6, false, true, 1>
                      : xu == 3 ? k_spmv_xsort<true, 0, 768, true, 6, false, true, 3>
                      : xu == 4 ? k_spmv_xsort<true, 0, 768, true, 6, false, true, 4>
                                : k_spmv_xsort<true, 0, 768, true, 6, false, true, 2>;
        else kern = xu == 1 ? k_spmv_xsort<false, 0, 768, true, 6, false, true, 1>
                    : xu == 3 ? k_spmv_xsort<false, 0, 768, true, 6, false, true, 3>
                    : xu == 4 ? k_spmv_xsort<false, 0, 768, true, 6, false, true, 4>
                              : k_spmv_xsort<false, 0, 768, true, 6, false, true, 2>;
    }
    static const char *trace_path = getenv("SBLAS_XS_TRACE");
    if (trace_path && mode == 0 && P.split == 8 && P.nt != 768 && !(P.nt == 512 && P.pair)) {  // debugging aid: the timeline-stamping twins
        if (P.nt == 512) kern = b ? k_spmv_xsort<true, 0, 512, false, 8, true> : k_spmv_xsort<false, 0, 512, false, 8, true>;
        else if (P.pair && P.dyn && xu == 1)
            kern = b ? k_spmv_xsort<true, 0, W, true, 8, true, true, 1> : k_spmv_xsort<false, 0, W, true, 8, true, true, 1>;
        else if (P.pair && P.dyn) kern = b ? k_spmv_xsort<true, 0, W, true, 8, true, true> : k_spmv_xsort<false, 0, W, true, 8, true, true>;
        else if (P.pair) kern = b ? k_spmv_xsort<true, 0, W, true, 8, true> : k_spmv_xsort<false, 0, W, true, 8, true>;
        else kern = b ? k_spmv_xsort<true, 0, W, false, 8, true> : k_spmv_xsort<false, 0, W, false, 8, true>;
    }
    std::vector<long long> htrace;
    if (trace_path) {
        const size_t len = 1 + (size_t)kXsTrace * (P.nitems + P.grid);
        SBLAS_HIP(hipMalloc(&a.trace, sizeof(long long) * len));
        SBLAS_HIP(hipMemsetAsync(a.trace, 0, sizeof(long long) * len, s));
        htrace.resize(len);
    }
    SBLAS_LAUNCH(kern, dim3(P.grid), dim3(P.nt), 0, s, a, x, alpha, beta, y);
    SBLAS_HIP(hipGetLastError());
    P.parity ^= 1;
    if (P.fused) ++P.epoch;
    if (trace_path) {  // debugging aid: rows {subA, subB, block<<4|xcc, t0, endA, endB}
        SBLAS_HIP(hipMemcpyAsync(htrace.data(), a.trace, sizeof(long long) * htrace.size(),
                                 hipMemcpyDeviceToHost, s));
        SBLAS_HIP(hipStreamSynchronize(s));
        (void)hipFree(a.trace);
        if (FILE *f = fopen(trace_path, "a")) {
            fprintf(f, "# launch items=%d grid=%d pair=%d\n", P.nitems, P.grid, (int)P.pair);
            for (long long i = 0; i < htrace[0]; ++i) {
                const long long *r = htrace.data() + 1 + kXsTrace * i;
                fprintf(f, "%lld %lld %lld %lld %lld %lld\n", r[0], r[1], r[2], r[3], r[4], r[5]);
            }
            fclose(f);
        }
    }
    if (P.nwide && !P.fused) {
        const dim3 grid((kXsHalfRows + 255) / 256, (unsigned)P.nwide);
        if (b)
            SBLAS_LAUNCH(k_xsort_reduce<true>, grid, dim3(256), 0, s, P.wranges, P.partial, alpha, beta,
                         y);
        else
            SBLAS_LAUNCH(k_xsort_reduce<false>, grid, dim3(256), 0, s, P.wranges, P.partial, alpha, beta,
                         y);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

}  // namespace sblas
