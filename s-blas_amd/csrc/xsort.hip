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
// row sum (tests) but not bitwise reproducible from run to run -- except on
// a deterministic handle (sblas_csr_set_deterministic / SBLAS_DETERMINISTIC),
// whose launches add each stream's chunks in chunk order (xs_stream_dyn
// kDet) and give bit-identical y every time.
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
// stream, so every work item PAIRS one of each: the two halves of the
// 512-thread workgroup (two teams of 4 waves, up to 256 VGPRs a wave, 8192
// LDS rows each) run them side by side and every CU mixes both kinds of
// traffic.  Items sit in one queue per XCD; a persistent grid (one workgroup
// per CU: 128 KiB of LDS rows) claims from its own XCD's queue (XCC_ID
// hardware register) and steals when it runs dry.  Inside an item the waves
// claim chunks from LDS counters (xs_stream_dyn), so a team that drains its
// own sub-item continues on its partner's and both halves end together.
// Matrices with many empty rows (power-law graphs) run their narrow ranges
// as solo items: both teams on one range of up to 16,384 LDS rows.
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

constexpr int kXsThreads = 512;   // two teams of kXsWaves waves
constexpr int kXsWaves = 4;       // waves per team
constexpr int kXsTeam = kXsWaves * 64;
constexpr int kXsU = 2;           // chunks per dynamic claim
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
constexpr uint32_t kXsPad = ((1u << kXsColBits) - 1) << kXsRowBits;  // column all ones, row 0
static_assert(kXsRowBits + kXsColBits == 32, "packed key is 32 bits");
static_assert(kXsHalfRows <= (1 << kXsRowBits), "a team's local row must fit the key");
// a range's rows: a team's half, or (solo items) the whole workgroup's
// accumulators up to what the key's row field addresses
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
// offsets are bnd[0..ng] (bnd[0] = c0) for groups gb, gb+1, ...  Every wave
// claims kXsU consecutive chunks at a time from the stream's LDS counter
// (*ctr, chunks past c0), so a team that has finished its own sub-item can
// drain its partner's: the two halves of a pair end together however their
// narrow/wide costs compare.  A claimed chunk (hence its group) is
// wave-uniform; claims are monotone per wave, so the group walk over bnd[]
// stays forward-only.
// Software pipeline with ping-pong registers, a claim per stage:
//   gathers(A) | claim + loads(B) | adds(A) | gathers(B) | claim + loads(A') | adds(B)
// sched_barrier pins that issue order; waiting for the gathers (vmcnt counts
// in order) then leaves the next stage's key/value loads in flight.  A wave
// past c1 loads one line (every lane the same address) and adds exact +0.0;
// padding entries add +0.0 too (a select, not a product: x may be inf/nan).
// kDet (deterministic plans, sblas_csr_set_deterministic): the adds of a
// stream's chunks land in chunk order -- a wave adds claim c only once the
// stream's LDS turn counter (*done, chunks past c0) has reached c, then
// advances it -- so every row's sum runs in the same order on every launch
// whichever waves took which chunks.  A narrow sub-item's two segments add
// into the same rows, so they share one counter: segment 2's turns start at
// `base` (segment 1's chunks rounded up to whole claims).  The holder of the
// lowest unfinished claim never waits, so the turns always progress.
template <bool kDet>
__device__ __forceinline__ void xs_stream_dyn(const v4u *__restrict__ key4, const v2d *__restrict__ val2,
                                              int ks, int vs, int *ctr, int *done, int base, long long c0,
                                              long long c1, const long long *bnd, int gb, int Wg,
                                              const double *__restrict__ x, double *acc)
{
    constexpr int U = kXsU;
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
                xx[u][j] = x[idx];
            }
    };
    auto accumulate = [&](long long cb, const v4u *kk, const v2d *va, const v2d *vb, double (*xx)[4]) {
        if constexpr (kDet) {  // wait for this claim's turn
            const int want = base + (int)(cb - c0);
            while (__builtin_amdgcn_readfirstlane(
                       __hip_atomic_load(done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != want)
                __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool live = cb + u < c1;
            const double v[4] = {va[u].x, va[u].y, vb[u].x, vb[u].y};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t k = kk[u][j];
                const double p = (live && k != kXsPad) ? v[j] * xx[u][j] : 0.0;
                atomicAdd(&acc[k & ((1u << kXsRowBits) - 1)], p);
            }
        }
        if constexpr (kDet) {  // the adds complete, then the next claim's turn
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            if (lane == 0)
                __hip_atomic_store(done, base + (int)(cb - c0) + U, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
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

// The kernel: one persistent 512-thread workgroup per CU, two teams of 4
// waves.  A work item pairs two sub-items (team 0's, team 1's); the waves of
// both teams claim chunks dynamically (xs_stream_dyn): a team drains its own
// streams, then its partner's.  A narrow sub-item alone in its item (solo)
// is written by the whole workgroup over all 16,384 LDS rows.  kDet: the
// deterministic form (ordered chunk adds, xs_stream_dyn; a narrow sub-item's
// group walk starts at a group fixed by its range, not by the XCD that runs
// it).
template <bool kBeta, bool kDet = false>
__global__ __launch_bounds__(kXsThreads) void k_spmv_xsort(const XsArgs a, const double *__restrict__ x,
                                                           double alpha, double beta, double *__restrict__ y)
{
    __shared__ double acc_all[kXsRows];
    __shared__ long long s_bnd_all[2][256];
    __shared__ long long s_rec_all[2][128 + 5];
    __shared__ int s_item;
    __shared__ int s_ctr[2][2];  // claimed chunks per (team, segment)
    __shared__ int s_done[2][2]; // kDet: turn counter per team's sub-item ([h][0]; both segments)
    __shared__ int s_par[2][4];  // per team {sub valid, k1, g0, n1}
    const int half = (int)(threadIdx.x >= (unsigned)kXsTeam);
    const int ht = (int)threadIdx.x - half * kXsTeam;
    double *acc = acc_all + half * kXsHalfRows;
    long long *s_bnd = s_bnd_all[half];
    const v4u *key4 = reinterpret_cast<const v4u *>(a.key);
    const v2d *val2 = reinterpret_cast<const v2d *>(a.val);
    const int xcc = xs_xcc_id();
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
        if (slot < 0) return;  // workgroup-uniform
        // the team's item record (host-built per (slot, team)): sub, row0 |
        // nrows << 32, pbase, widx, then the range's G+1 block offsets -- one
        // round trip of independent loads instead of sub -> range -> blocks.
        // sub = range << 8 | k: k+1 = wide sub-item of XCD k (its q groups
        // [kq, kq+q), partial slot k); 0 = narrow (all G groups, starting at
        // this XCD's first group and wrapping); -1 = nothing for this team
        {
            const long long *rec = a.xrec + (long long)(2 * slot + half) * (a.G + 5);
            for (int j = ht; j < a.G + 5; j += kXsTeam) s_rec_all[half][j] = rec[j];
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
            g0 = k1 ? (k1 - 1) * a.q : (kDet ? ((sub >> 8) & 7) : xcc) * a.q;
            // s_bnd[j] = first chunk of group g0 + j: segment 1 is groups
            // [g0, g0+n1); a narrow sub-item's segment 2 is groups [0, g0)
            // at s_bnd + 128
            n1 = k1 ? a.q : a.G - g0;
            for (int r = ht; r < R.nrows; r += kXsTeam) acc[r] = 0.0;
            for (int j = ht; j <= n1; j += kXsTeam) s_bnd[j] = bo[g0 + j];
            if (!k1)
                for (int j = ht; j <= g0; j += kXsTeam) s_bnd[128 + j] = bo[j];
        }
        if (ht == 0) {
            s_ctr[half][0] = 0;
            s_ctr[half][1] = 0;
            s_done[half][0] = 0;
            s_done[half][1] = 0;
            s_par[half][0] = sub;
            s_par[half][1] = k1;
            s_par[half][2] = g0;
            s_par[half][3] = n1;
        }
        __syncthreads();
        // claim the next item now; its result is consumed after the stream,
        // so the atomic's latency hides behind the stream's own loads
        int pre = 0;
        if (threadIdx.x == 0 && a.dynamic) pre = atomicAdd(&a.qhead[xcc], 1);
        // own segment 1, own segment 2 (narrow wrap), then the partner's
        // two: one inlined stream, its operands chosen per pass
        for (int p = 0; p < 4; ++p) {
            const int h = p < 2 ? half : 1 - half;
            const int seg = p & 1;
            const int hs = s_par[h][0], hk1 = s_par[h][1], hg0 = s_par[h][2], hn1 = s_par[h][3];
            if (hs < 0 || (seg && (hk1 || hg0 == 0))) continue;  // uniform
            const long long *hb = s_bnd_all[h] + (seg ? 128 : 0);
            const int hn = seg ? hg0 : hn1;
            // kDet: segment 2 continues segment 1's turns (the same rows)
            const int base = seg ? (int)((s_bnd_all[h][hn1] - s_bnd_all[h][0] + kXsU - 1) / kXsU * kXsU) : 0;
            xs_stream_dyn<kDet>(key4, val2, a.kstride, a.vstride, &s_ctr[h][seg], &s_done[h][0], base, hb[0],
                                hb[hn], hb, seg ? 0 : hg0, a.Wg, x, acc_all + h * kXsHalfRows);
        }
        // A narrow sub-item alone in its item (the partner team empty: solo
        // items, or a leftover) is written by the whole workgroup: its rows
        // may fill both teams' LDS halves.
        const int s0 = (int)s_rec_all[0][0];
        const bool solo = (int)s_rec_all[1][0] < 0 && s0 >= 0 && (s0 & 255) == 0;  // uniform
        constexpr int kEp = (kXsHalfRows + kXsTeam - 1) / kXsTeam;
        static_assert(kEp * kXsThreads >= kXsRows, "a solo item's rows fit the epilogue");
        // a narrow epilogue's y loads are issued before the barrier below, so
        // their latency overlaps the wait for the workgroup's last wave
        const bool ynarrow = solo || (sub >= 0 && !k1);
        const int et = solo ? (int)threadIdx.x : ht;
        const int eNT = solo ? kXsThreads : kXsTeam;
        const long long rr = solo ? s_rec_all[0][1] : ((long long)(unsigned)R.row0 | ((long long)R.nrows << 32));
        const int row0 = (int)(rr & 0xffffffffLL), nrows = (int)(rr >> 32);
        double y0[kEp];
        if constexpr (kBeta) {
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
        if (sub >= 0 && k1) {
            // wide: this XCD's alpha-free partial, added by k_xsort_reduce
            // (the kernel boundary publishes the stores).  A team owns <=
            // kXsHalfRows rows, at most kEp per thread, every store issued
            // back to back.
            double *out = a.partial + R.pbase + (long long)(k1 - 1) * R.nrows;
#pragma unroll
            for (int e = 0; e < kEp; ++e) {
                const int r = ht + e * kXsTeam;
                if (r < R.nrows) out[r] = acc[r];
            }
        } else if (solo || sub >= 0) {
            // narrow: y = alpha * acc + beta * y over the sub-item's rows; a
            // solo item's <= kXsRows rows over all threads, a team's <=
            // kXsHalfRows over its kXsTeam
            const double *eacc = solo ? acc_all : acc;
            double *yr = y + row0;
#pragma unroll
            for (int e = 0; e < kEp; ++e) {
                const int r = et + e * eNT;
                if (r < nrows) yr[r] = kBeta ? alpha * eacc[r] + beta * y0[e] : alpha * eacc[r];
            }
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
    (void)hipFree(P.wranges);
    (void)hipFree(P.key);  // P.val points into the same allocation
    (void)hipFree(P.qhead);
    (void)hipFree(P.partial);
    (void)hipFree(P.xrec);
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
    double opt = 0.0;

    // column groups: G = 8q groups of Wg < 2^18 columns (the all-ones column
    // field is the padding key) and ~1 MiB of x (an XCD's current group plus
    // the entry stream must fit its 4 MiB L2)
    const long long wmax = (1LL << kXsColBits) - 1;
    const long long ng = ((long long)std::max(n, 1) + wmax - 1) / wmax;
    const long long nmib = ((long long)std::max(n, 1) * 8 + (1LL << 20) - 1) >> 20;
    P.q = (int)std::max<long long>({1LL, (ng + 7) / 8, (nmib + 7) / 8});
    P.G = 8 * P.q;
    if (P.G > 127) {
        set_error("xsort: n = %d needs %d column groups (> 127)", n, P.G);
        return SBLAS_ERR_UNSUPPORTED;
    }
    P.Wg = (int)std::max<long long>(1, ((long long)std::max(n, 1) + P.G - 1) / P.G);
    const int G = P.G, Wg = P.Wg;

    // Workgroup: two 4-wave teams (512 threads, 2 waves per SIMD, up to 256
    // VGPRs a wave) -- the register budget lets the compiler keep more of the
    // stream in flight than two 8-wave teams (1024 threads, 128 VGPRs) or two
    // 6-wave teams (768, ~170): config 2 N = 1 / 2 / 4 / 8 150.6-152.5 /
    // 96.4-96.7 / 65.5-65.6 / 40.7-40.8 us against 153.0-153.3 / 99.1 /
    // 66.3-66.9 / 42.1-42.5, 27-point 128^3 117 vs 121, 7-point 160^3 83 vs
    // 85, R-MAT equal (profiles/r05/wg512p/).  Resident workgroups = item
    // slots; a paired item holds two sub-items.
    int dev = 0, ncu = 0, per_cu = 0;
    SBLAS_HIP(hipGetDevice(&dev));
    SBLAS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spmv_xsort<true>, kXsThreads, 0));
    const int resident = std::max(1, ncu * std::max(per_cu, 1));
    const long long slots = (long long)resident * 2;  // sub-items
    // every range wide (8 XCD-local sub-items + partials per row) on small
    // matrices: a rank's slice of the uniform config 2 at N = 8 (5.0M
    // entries) 47.0 -> 41.8 us, N = 16 (2.5M) 33.8 -> 29.9, but N = 4 (9.9M)
    // 66.8 -> 104 (profiles/r05/sweep2/): the partials (16 B per row and XCD)
    // outweigh XCD-local gathers beyond ~6M entries.
    const bool all_wide = test_option("xs_allwide", &opt) ? opt != 0.0 : nnz <= kXsAllWideMaxNnz;
    const int rows_cap = kXsHalfRows;
    // Solo narrow items: a narrow range is an item of its own -- both teams'
    // waves and all 16,384 LDS rows -- so its blocks are twice as dense
    // (fewer x line requests per entry); wide ranges still pair (wide, wide)
    // at 8,192 rows a team.  Chosen when >= 40% of the rows are empty
    // (power-law graphs: an empty row spends an accumulator row, so 16,384
    // rows per light range hold what 8,192 would without them): R-MAT scale
    // 21 (50% empty) 158.8 -> 147.3 us; config 2 and the stencils have none
    // and keep pairs (solo there: 146.7 vs 131 us; profiles/r04/rmat/).
    {
        long long empty = 0;
        for (int r = 0; r < m; ++r) empty += rp[r + 1] == rp[r];
        P.solo = test_option("xs_solo", &opt) ? opt != 0.0 : (m > 0 && 5 * empty >= 2LL * m);
    }
    const int nrows_cap = P.solo ? kXsItemRows : rows_cap;  // narrow ranges
    const double nfac = P.solo ? 2.0 : 1.0;                 // a narrow range's cost, in sub-item caps

    // Cost model (work units ~ one streamed entry): a sub-item's time is its
    // entries plus lambda per distinct x line its gathers touch; with uniform
    // columns a block of c entries over L lines touches L*(1 - exp(-c/L))
    // lines.  A narrow sub-item spreads its entries over all of x (G*Lg
    // lines), a wide one its 1/8 share over its XCD's q groups.  lambda = 1.0
    // is the best of a sweep (0.3 .. 1.7) on config 2.
    const double lam = 1.0;
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
        while (r < m) {
            long long cnt;
            int e = cut(r, true, cnt);
            const bool wide = cnt > 0 && (all_wide || (narrow_cost((double)cnt) > nfac * cap &&
                                                      cnt >= 16LL * (e - r)));
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
    // second round for a few items would double the kernel's tail).  The
    // "xs_cap" test hook fixes the cap instead (many small items: the
    // dynamic claims run on small matrices).
    const bool fixed_cap = test_option("xs_cap", &opt);
    double cap = fixed_cap ? std::max(1.0, opt) : narrow_cost((double)nnz) / (double)slots;
    // Ranges hold at most rows_cap rows, so once ceil(m / rows_cap) exceeds
    // the slots no cap can fit them: stop there (and after 50 growth steps
    // without fewer sub-items) instead of 400 O(m) passes.  Leftover
    // sub-items are still correct: the grid claims them in a second round.
    const long long min_ranges = ((long long)m + rows_cap - 1) / rows_cap;
    long long best_subs = -1;
    for (int it = 0, flat = 0; it < 400; ++it) {
        build_ranges(cap);
        const long long subs = count_subs();
        if (subs <= slots || fixed_cap || min_ranges > slots) break;
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

    // host copies of the CSR entries (uninitialised: the copies fill them)
    std::unique_ptr<int[]> hcol(new int[(size_t)std::max<long long>(nnz, 1)]);
    std::unique_ptr<double[]> hval(new double[(size_t)std::max<long long>(nnz, 1)]);
    if (nnz) {
        SBLAS_HIP(hipMemcpy(hcol.get(), A.col, sizeof(int) * nnz, hipMemcpyDeviceToHost));
        SBLAS_HIP(hipMemcpy(hval.get(), A.val, sizeof(double) * nnz, hipMemcpyDeviceToHost));
    }

    // pass 1: every block (range, group) bucketed and sorted by (column, row)
    // once, kept for the fill.  One range per task for the bucketing (a wide
    // range holds ~13x a narrow one's entries, and they sit together at the
    // heavy rows), then the blocks are sorted as tasks of their own.
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
#pragma omp parallel for schedule(dynamic, 4)
    for (long long k = 0; k < (long long)nblk; ++k) {
        auto &bb = bk[(size_t)k];
        std::stable_sort(bb.begin(), bb.end(),
                         [](const std::pair<uint32_t, double> &u, const std::pair<uint32_t, double> &v) {
                             return u.first < v.first;
                         });
    }
    if (bad) {
        set_error("xsort: column index out of [0, n) or key overflow");
        return SBLAS_ERR_INVALID;
    }
    std::vector<long long> blk(nblk + 1, 0);  // chunk offsets
    for (size_t k = 0; k < nblk; ++k)
        blk[k + 1] = blk[k] + ((long long)bk[k].size() + kXsChunk - 1) / kXsChunk;
    const long long nchunks = blk.back();

    // pass 2: fill every chunk (lane-transposed, header comment): per chunk
    // 1 KiB of keys then 2 KiB of values, ONE 3-KiB run in HBM.  Every byte
    // of every chunk is written by the fill below: no zeroing pass.
    const size_t cbytes = (size_t)kXsChunk * (sizeof(uint32_t) + sizeof(double));
    const size_t hb_n = (size_t)std::max<long long>(nchunks, 1) * cbytes;
    std::unique_ptr<unsigned char[]> hbuf(new unsigned char[hb_n]);
    auto chunk_keys = [&](long long c) { return (uint32_t *)(hbuf.get() + (size_t)c * cbytes); };
    auto chunk_vals = [&](long long c) {
        return (double *)(hbuf.get() + (size_t)c * cbytes + kXsChunk * sizeof(uint32_t));
    };
    P.kstride = (int)(cbytes / 16);
    P.vstride = (int)(cbytes / 16);
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

    // sub-items, wide partial slots, then items (pairs) in XCD queues
    std::vector<int> wide, nsub;
    std::vector<std::vector<int>> wsub(8);
    long long pbase = 0;
    for (int i = 0; i < I; ++i) {
        XsRange &R = ranges[i];
        R.widx = -1;
        if (R.wide) {
            R.pbase = pbase;
            pbase += 8LL * R.nrows;
            R.widx = (int)wide.size();
            wide.push_back(i);
            for (int k = 0; k < 8; ++k) wsub[k].push_back((i << 8) | (k + 1));
        } else {
            nsub.push_back(i << 8);
        }
    }
    std::vector<std::vector<std::pair<int, int>>> q(8);
    if (P.solo) {
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

    SBLAS_HIP(hipMalloc(&P.wranges, sizeof(XsRange) * std::max<size_t>(wide.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.key, hb_n));
    P.val = (double *)((unsigned char *)P.key + kXsChunk * sizeof(uint32_t));
    SBLAS_HIP(hipMalloc(&P.qhead, sizeof(int) * 32));  // [2 parities][8 claim heads + pad]
    {
        std::vector<int> h(32, 0);
        for (int k = 0; k < 8; ++k) h[k] = h[16 + k] = P.qstat[k];
        SBLAS_HIP(hipMemcpy(P.qhead, h.data(), sizeof(int) * 32, hipMemcpyHostToDevice));
    }
    SBLAS_HIP(hipMalloc(&P.partial, sizeof(double) * std::max<long long>(pbase, 1)));
    if (!wide.empty()) {
        std::vector<XsRange> wr;
        for (int i : wide) wr.push_back(ranges[(size_t)i]);
        SBLAS_HIP(hipMemcpy(P.wranges, wr.data(), sizeof(XsRange) * wr.size(), hipMemcpyHostToDevice));
    }
    if (nchunks) SBLAS_HIP(hipMemcpy(P.key, hbuf.get(), hb_n, hipMemcpyHostToDevice));
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
    (void)s;
    P.ready = true;
    return SBLAS_OK;
}

int launch_spmv_xsort(const sblas_csr_s &A, double alpha, const double *x, double beta,
                      double *y, hipStream_t s)
{
    const XsPlan &P = A.xs;
    if (!P.ready) return SBLAS_ERR_INVALID;
    if (A.m == 0 || P.nitems == 0) return SBLAS_OK;
    XsArgs a{};
    a.key = P.key;
    a.val = P.val;
    a.kstride = P.kstride;
    a.vstride = P.vstride;
    a.xrec = P.xrec;
    // the parity advances only once the launch is known to be queued: a
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
    a.qstride = P.qstride;
    a.G = P.G;
    a.q = P.q;
    a.Wg = P.Wg;
    const bool b = beta != 0.0;
    if (A.deterministic) {
        if (b) SBLAS_LAUNCH((k_spmv_xsort<true, true>), dim3(P.grid), dim3(kXsThreads), 0, s, a, x, alpha, beta, y);
        else SBLAS_LAUNCH((k_spmv_xsort<false, true>), dim3(P.grid), dim3(kXsThreads), 0, s, a, x, alpha, beta, y);
    } else {
        if (b) SBLAS_LAUNCH(k_spmv_xsort<true>, dim3(P.grid), dim3(kXsThreads), 0, s, a, x, alpha, beta, y);
        else SBLAS_LAUNCH(k_spmv_xsort<false>, dim3(P.grid), dim3(kXsThreads), 0, s, a, x, alpha, beta, y);
    }
    SBLAS_HIP(hipGetLastError());
    P.parity ^= 1;
    if (P.nwide) {
        const dim3 grid((kXsHalfRows + 255) / 256, (unsigned)P.nwide);
        if (b)
            SBLAS_LAUNCH(k_xsort_reduce<true>, grid, dim3(256), 0, s, P.wranges, P.partial, alpha, beta, y);
        else
            SBLAS_LAUNCH(k_xsort_reduce<false>, grid, dim3(256), 0, s, P.wranges, P.partial, alpha, beta, y);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

}  // namespace sblas
