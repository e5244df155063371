// transpose.hip -- device CSR -> CSC transpose with bit-exact indices.
//
// Semantics of sptrsv/sptrsv_v1/src/tranpose.h:6-43 (matrix_transposition):
// column histogram, exclusive scan, then a STABLE scatter in row order, so
// row indices ascend inside every column and equal-(row,col) duplicates keep
// their CSR order.  GPU forms, both stable sorts of the nonzeros (in CSR
// order) by column, so rows ascend inside each column exactly as the
// reference's ordered scatter leaves them:
//  * default (n > 512): MSD -- two stable partition passes on the high column
//    bits (pass A over fixed segments of the CSR order, deriving each entry's
//    row from rowptr; pass B inside each pass-A bucket), then one pass per
//    final bucket of 2^c columns that counts, ranks and writes its run in
//    column order with its colptr entries.  Between the passes an entry
//    travels as one packed word (the key bits still needed + the row or its
//    offset in the segment) and its value;
//  * LSD radix passes of <= 8-bit digits carrying (key, row, value), colptr
//    read off the sorted keys (n <= 512, or SBLAS_TRANSPOSE_ALGO=lsd).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
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

// ---- stable LSD radix sort of (col, row, val) by col -----------------------
// Tiles of kRxTile consecutive nonzeros; 8-bit digits; per pass
//   k_rx_count   : per-tile digit histogram in LDS -> counts[digit][tile]
//   scan         : inclusive scan of counts (digit-major) -> global offsets
//   k_rx_scatter : stable in-tile ranking (wave ballots per digit bit, wave
//                  order through LDS), tile staged in LDS in digit order, then
//                  written out as per-digit runs.
// No global atomics (they execute memory-side, one 64-B request per lane).
constexpr int kRxThreads = 256;
constexpr int kRxItems = 16;
constexpr int kRxTile = kRxThreads * kRxItems;
constexpr int kRxWaves = kRxThreads / 64;

// row of every nonzero: a wave per 64 rows writes them one after another,
// all 64 lanes on one row's entries (consecutive stores).  (A thread per
// row left a long row's lane storing ~100 words alone -- 84 us on the
// config-2 matrix; 16-B stores per thread 157 us; a binary search per four
// entries 176 us, its 21 dependent loads per thread.)
__global__ __launch_bounds__(256) void k_expand_rows(const int *__restrict__ rowptr, int m, int *__restrict__ rows)
{
    const int lane = threadIdx.x & 63;
    const int r0 = ((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6)) * 64;
    if (r0 >= m) return;
    const int nrow = min(64, m - r0);
    const int b = rowptr[min(r0 + lane, m)];
    const int last = rowptr[r0 + nrow];
    for (int j = 0; j < nrow; ++j) {
        const int s = __builtin_amdgcn_readlane(b, j);
        const int e = j + 1 < nrow ? __builtin_amdgcn_readlane(b, j + 1) : last;
        for (int k = s + lane; k < e; k += 64) rows[k] = r0 + j;
    }
}

__global__ __launch_bounds__(kRxThreads) void k_rx_count(const int *__restrict__ keys, long long nnz,
                                                         int shift, int ntiles, int *__restrict__ counts)
{
    __shared__ int h[256];
    const int t = threadIdx.x;
    h[t] = 0;
    __syncthreads();
    const long long base = (long long)blockIdx.x * kRxTile;
#pragma unroll
    for (int j = 0; j < kRxItems; ++j) {
        const long long i = base + j * kRxThreads + t;
        if (i < nnz) atomicAdd(&h[(keys[i] >> shift) & 255], 1);
    }
    __syncthreads();
    counts[(size_t)t * ntiles + blockIdx.x] = h[t];
}

__global__ __launch_bounds__(kRxThreads, 2) void k_rx_scatter(
    const int *__restrict__ kin, const int *__restrict__ rin, const double *__restrict__ vin, long long nnz,
    int shift, int ntiles, const int *__restrict__ incl, int *__restrict__ kout, int *__restrict__ rout,
    double *__restrict__ vout)
{
    __shared__ int wcnt[kRxWaves][256];
    __shared__ int run[256], lstart[256], gbase[256], wtot[kRxWaves];
    __shared__ int skey[kRxTile], srow[kRxTile];
    __shared__ double sval[kRxTile];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    run[t] = 0;
#pragma unroll
    for (int q = 0; q < kRxWaves; ++q) wcnt[q][t] = 0;
    const long long base = (long long)blockIdx.x * kRxTile;
    const int valid = (int)min((long long)kRxTile, nnz - base);
    int kk[kRxItems], rr[kRxItems], lp[kRxItems];
    double vv[kRxItems];
#pragma unroll
    for (int j = 0; j < kRxItems; ++j) {
        const int li = j * kRxThreads + t;
        if (li < valid) {
            kk[j] = kin[base + li];
            rr[j] = rin[base + li];
            vv[j] = vin[base + li];
        } else {
            kk[j] = -1;  // digit 255, ranked after every real element
            rr[j] = 0;
            vv[j] = 0.0;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRxItems; ++j) {
        const int d = (kk[j] >> shift) & 255;
        unsigned long long mm = ~0ull;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bal = __ballot((d >> b) & 1);
            mm &= ((d >> b) & 1) ? bal : ~bal;
        }
        const int rank = __popcll(mm & lt);
        if (rank == 0) wcnt[w][d] = __popcll(mm);
        __syncthreads();
        int pre = run[d];
        for (int q = 0; q < w; ++q) pre += wcnt[q][d];
        lp[j] = pre + rank;
        __syncthreads();
        int add = 0;
#pragma unroll
        for (int q = 0; q < kRxWaves; ++q) {
            add += wcnt[q][t];
            wcnt[q][t] = 0;
        }
        run[t] += add;
        __syncthreads();
    }
    if (t == 255) run[255] -= kRxTile - valid;  // padding is not part of the output
    __syncthreads();
    // exclusive scan of the tile's digit counts -> lstart
    const int c = run[t];
    const int inc = wave_incl_scan(c);
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    int woff = 0;
    for (int q = 0; q < w; ++q) woff += wtot[q];
    lstart[t] = woff + inc - c;
    gbase[t] = incl[(size_t)t * ntiles + blockIdx.x] - c;  // inclusive scan -> exclusive
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRxItems; ++j) {
        const int li = j * kRxThreads + t;
        if (li < valid) {
            const int pos = lstart[(kk[j] >> shift) & 255] + lp[j];
            skey[pos] = kk[j];
            srow[pos] = rr[j];
            sval[pos] = vv[j];
        }
    }
    __syncthreads();
    for (int li = t; li < valid; li += kRxThreads) {
        const int k = skey[li];
        const int d = (k >> shift) & 255;
        const long long g = (long long)gbase[d] + (li - lstart[d]);
        kout[g] = k;
        rout[g] = srow[li];
        vout[g] = sval[li];
    }
}

// ---- wide-digit variant (default): up to 11-bit digits, 2 passes for n <=
// 4M columns instead of 3.  Workgroup b sorts the contiguous tiles
// [b*S, (b+1)*S) in order, so (i) the count matrix is digits x workgroups,
// not digits x tiles, and (ii) a digit's output run of tile t+1 continues
// exactly where tile t's ended: the same CU appends to the same lines, which
// its XCD's L2 merges before write-back (with 2,048 digits a tile's runs are
// only ~2 entries long).  Ranking per 256-element batch: RB wave ballots give
// the in-wave rank; the first lane of each (wave, digit) group posts the
// group's size, so LDS work per element is O(waves), not O(digits).
constexpr int kRx2MaxDigits = 2048;
// scatter workgroup size: 512 threads = 8 waves, 8 entries per thread of a
// 4096-entry tile (256 threads left only 8 waves per CU at 71 KiB of LDS)
#ifndef SBLAS_R2_THREADS
#define SBLAS_R2_THREADS 512
#endif
constexpr int kR2Threads = SBLAS_R2_THREADS;

// Segments.  kSegTiles: workgroup w's contiguous tiles [w*S, (w+1)*S), counts
// indexed [digit][w].  kSegBuckets (the MSD passes): workgroup w = b*J + j
// takes part j of J of bucket b, the bucket's range read off the previous
// pass's scanned counts (bucket b = entries [Jp*b, Jp*b + Jp) of prev), and
// counts are indexed [(b*D + digit)*J + j], so one inclusive scan of them,
// bucket-major, yields the stable partition of every bucket by the digit.
constexpr int kSegTiles = 0, kSegBuckets = 1;

struct SegArgs {
    int S, nwg;               // kSegTiles
    const int *prev;          // kSegBuckets: previous pass's inclusive scan
    int Jp, J;
    int nb;                   // kSegFinal: number of buckets (grid-stride)
};

__device__ __forceinline__ void seg_range(int mode, const SegArgs &g, int wg, long long nnz, long long &s0,
                                          long long &s1)
{
    if (mode == kSegTiles) {
        s0 = (long long)wg * g.S * kRxTile;
        s1 = min(nnz, s0 + (long long)g.S * kRxTile);
        if (s0 > s1) s0 = s1;
        return;
    }
    const int b = wg / g.J, j = wg % g.J;
    const long long i0 = (long long)b * g.Jp;
    const long long bs = i0 ? g.prev[i0 - 1] : 0, be = g.prev[i0 + g.Jp - 1];
    const long long len = be - bs;
    s0 = bs + len * j / g.J;
    s1 = bs + len * (j + 1) / g.J;
}

__device__ __forceinline__ size_t seg_count_idx(int mode, const SegArgs &g, int wg, int D, int d)
{
    if (mode == kSegTiles) return (size_t)d * g.nwg + wg;
    return ((size_t)(wg / g.J) * D + d) * g.J + (wg % g.J);
}

// counts of each scatter workgroup's segment: one 1024-thread workgroup per
// segment, 16 keys in flight per thread, LDS histogram, then every digit's
// count stored plainly (no zeroing, no global atomics: with eight workgroups
// per segment merging by atomics the two count passes took 75 us each on the
// config-2 matrix, memory-side atomics being one 64-B request per lane).
constexpr int kCntThreads = 1024;
// wgrow (MSD pass A): also the row holding each segment's first entry,
// the start of the scatter's row derivation.
template <int kSeg>
__global__ __launch_bounds__(kCntThreads) void k_rx2_count(const int *__restrict__ keys, long long nnz,
                                                           int shift, int rb, SegArgs g,
                                                           int *__restrict__ counts,
                                                           const int *__restrict__ rowptr = nullptr, int m = 0,
                                                           int *__restrict__ wgrow = nullptr)
{
    // digits <= 128: one private histogram per wave (waves do not contend
    // for the same LDS words), summed at the end
    constexpr int kCW = kCntThreads / 64;
    __shared__ int h[kRx2MaxDigits > 128 * kCW ? kRx2MaxDigits : 128 * kCW];
    __shared__ int s_first;
    const int D = 1 << rb;
    const bool priv = D <= 128;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int *hw = priv ? h + wv * 128 : h;
    for (int d = threadIdx.x; d < (priv ? 128 * kCW : D); d += kCntThreads) h[d] = 0;
    const int wg = (int)blockIdx.x;
    long long p0, p1;
    seg_range(kSeg, g, wg, nnz, p0, p1);
    int lo = 0;
    if (wgrow && wv < 2) {
        // wave 0: the row holding the segment's first entry (largest r with
        // rowptr[r] <= p0); wave 1: the row of its last; wgrow[nseg + wg] =
        // the rows the segment spans beyond its first (0 when empty).  A
        // 64-ary search: each round the 64 lanes probe evenly spaced rows.
        const long long p = wv == 0 ? p0 : max(p0, p1 - 1);
        int hi = m - 1;  // rowptr[lo] <= p
        while (lo < hi) {
            const int step = (hi - lo + 63) / 64;
            const long long r = (long long)lo + (long long)(lane + 1) * step;
            const bool ok = r <= hi && rowptr[r] <= p;
            const int k = __popcll(__ballot(ok));  // ok holds for a prefix of the lanes
            lo += k * step;
            hi = min(hi, lo + step - 1);
        }
        if (wv == 0 && lane == 0) {
            wgrow[wg] = lo;
            s_first = lo;
        }
    }
    __syncthreads();  // histograms zeroed, s_first set
    if (wgrow && wv == 1 && lane == 0) wgrow[(int)gridDim.x + wg] = p1 > p0 ? lo - s_first : 0;
    // 16-B loads over the aligned body (keys arrays are 16-B aligned), single
    // keys for the head and tail
    const long long q0 = min(p1, (p0 + 3) & ~3LL), q1 = max(q0, p1 & ~3LL);
    for (long long i = p0 + threadIdx.x; i < q0; i += kCntThreads) atomicAdd(&hw[(keys[i] >> shift) & (D - 1)], 1);
    for (long long i = q1 + threadIdx.x; i < p1; i += kCntThreads) atomicAdd(&hw[(keys[i] >> shift) & (D - 1)], 1);
    const int4 *k4 = reinterpret_cast<const int4 *>(keys + q0);
    const long long n4 = (q1 - q0) >> 2;
    constexpr int kU = 8;
    for (long long i0 = 0; i0 < n4; i0 += (long long)kU * kCntThreads) {
        int4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const long long i = i0 + (long long)u * kCntThreads + threadIdx.x;
            v[u] = i < n4 ? k4[i] : make_int4(-1, -1, -1, -1);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
            if (v[u].x != -1) {
                atomicAdd(&hw[(v[u].x >> shift) & (D - 1)], 1);
                atomicAdd(&hw[(v[u].y >> shift) & (D - 1)], 1);
                atomicAdd(&hw[(v[u].z >> shift) & (D - 1)], 1);
                atomicAdd(&hw[(v[u].w >> shift) & (D - 1)], 1);
            }
    }
    __syncthreads();
    for (int dd = threadIdx.x; dd < D; dd += kCntThreads) {
        int c = h[dd];
        if (priv)
            for (int q = 1; q < kCW; ++q) c += h[q * 128 + dd];
        counts[seg_count_idx(kSeg, g, wg, D, dd)] = c;
    }
}

// Scatter: workgroup b sorts tiles [b*S, (b+1)*S) in order.  Wave w ranks
// the contiguous quarter [w*1024, (w+1)*1024) of a tile in 16 batches of 64
// with WAVE-PRIVATE digit counters (a wave's LDS operations retire in
// program order, so no barrier per batch): rank = wcnt[w][d] + in-batch rank
// from RB ballots.  Two barriers per tile then turn the per-wave counts into
// the tile's digit offsets.  The next tile's (key, row, value) are loaded
// into registers while the current one is ranked and written.
// kSegFinal (the MSD transpose's last pass): workgroup b owns bucket b of the
// previous pass whole (its entries share every column bit above `rb`), counts
// its digits itself, so its output is the contiguous run [s0, s1) in column
// order; it writes colptr for its 2^rb columns, and keys only if kout.
constexpr int kSegFinal = 2;
constexpr int kSegFinalDirect = 3;  // the same, each entry written from registers

// kDerive (the MSD transpose's pass A): the entries' rows are not read from
// an expanded array but derived per tile from rowptr.  The workgroup walks
// its tiles in order with the row rc that contains the tile's first entry
// (the first from wgrow[], written by the count pass).  Thread t holds the
// start of row rc+1+t (a window of kT rows, loaded one tile ahead); each row
// starting inside the tile marks its position in srow with atomicMax (empty
// rows share a position, the largest wins), and a prefix max over the
// positions -- per wave over its contiguous quarter, then across waves --
// is every entry's row.  Rows starting exactly at the tile's end give the
// next tile's rc.  A tile holding more than kT row starts takes more windows.
// kPkF (last pass, packed input): rows are unpacked from the staged keys, so
// no row array is staged (less LDS: more workgroups per CU); kWpe: waves per
// SIMD asked of the register allocator.
template <int kMaxD, int kSeg, int kT, bool kDerive = false, int kTile = kRxTile, bool kPkF = false,
          int kWpe = 1>
__global__ __launch_bounds__(kT, kWpe) void k_rx2_scatter(
    const int *__restrict__ kin, const int *__restrict__ rin, const double *__restrict__ vin, long long nnz,
    int shift, int rb, SegArgs sg, const int *__restrict__ incl, int *__restrict__ kout,
    int *__restrict__ rout, double *__restrict__ vout, int *__restrict__ colptr, int n, int pack,
    const int *__restrict__ rowptr = nullptr, int m = 0, const int *__restrict__ wgrow = nullptr,
    int packA = -1)
{
    constexpr bool kFinal = kSeg >= kSegFinal;
    // packA (MSD passes A and B): pass A writes ONE word per entry, the key's
    // low packA bits (all pass B and the last pass read) with the row's offset
    // from its segment's first row above them, and no row array; pass B finds
    // each entry's segment (the segments' runs inside its bucket, in LDS) and
    // adds that segment's first row.  Taken when every segment spans fewer
    // than 2^(32 - packA) rows (wgrow[nseg + s] = segment s's span, from the
    // count pass); all workgroups read the same spans, so all agree.
    constexpr bool kPA = (kSeg == kSegTiles && kDerive) || kSeg == kSegBuckets;
    constexpr int kSegMax = 512;
    __shared__ int s_segstart[kSeg == kSegBuckets ? kSegMax + 1 : 1];
    __shared__ int s_segrow[kSeg == kSegBuckets ? kSegMax : 1];
    constexpr int kW = kT / 64;  // waves
    __shared__ int wcnt[kW][kMaxD];  // per-wave counts, then per-wave starts
    __shared__ int lstart[kMaxD], gbase[kMaxD];
    __shared__ int wtot[kW];
    __shared__ int wmaxs[kW], s_next, s_more[2];  // kDerive
    __shared__ int skey[kTile], srow[kPkF ? 1 : kTile];
    __shared__ double sval[kTile];
    constexpr int kQ = kTile / kW;  // elements per wave per tile
    constexpr int kB = kQ / 64;             // batches per wave (16)
    static_assert(kB * kT == kTile, "one register slot per batch");
    static_assert(kTile == kRxTile || kSeg >= kSegFinal, "tile segments (seg_range) assume kRxTile");
    const int D = 1 << rb, dm = D - 1;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    long long s0, s1;
    seg_range(kFinal ? kSegBuckets : kSeg, sg, (int)blockIdx.x, nnz, s0, s1);
    int bk = (int)blockIdx.x;  // the last pass: current bucket (grid-stride)
    // column written to kout by the last pass: its bucket's bits and the key's
    // low rb bits (the key above them may be a packed word)
    auto colkey = [&](int k) { return kFinal ? ((bk << rb) | (k & dm)) : k; };
    bool pA = false;  // workgroup-uniform
    const int nseg = kSeg == kSegBuckets ? sg.Jp : (int)gridDim.x;
    if constexpr (kPA) {
        if (packA >= 0 && nseg <= kSegMax) {
            int v = 0;
            for (int i = t; i < nseg; i += kT) v = max(v, wgrow[nseg + i]);
#pragma unroll
            for (int off = 32; off; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
            if (lane == 0) wmaxs[w] = v;
            __syncthreads();
            int mx = 0;
#pragma unroll
            for (int q = 0; q < kW; ++q) mx = max(mx, wmaxs[q]);
            pA = packA >= 31 || mx < (1 << (32 - packA));
            __syncthreads();
        }
    }
    const unsigned kbmask = packA >= 0 && packA < 32 ? (1u << packA) - 1u : ~0u;
    int segrow0 = 0;  // pass A: the segment's first row
    int scur = 0;     // pass B: this wave's current segment
    int kk[kB], rr[kB];
    double vv[kB];
    auto rowof = [&](int j) { return (kFinal && pack >= 0) ? (int)((unsigned)kk[j] >> pack) : rr[j]; };
    auto load_tile = [&](long long base, int valid) {
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            const int li = w * kQ + j * 64 + lane;
            const bool ok = li < valid;
            const long long gi = ok ? base + li : 0;
            kk[j] = ok ? kin[gi] : -1;  // top digit, ranked after every real element
            // a packed last-pass key carries the row; it is unpacked where it is
            // used (here it would make the prefetch wait for its load)
            if (!(kFinal && pack >= 0) && !kDerive && !(kSeg == kSegBuckets && pA)) rr[j] = ok ? rin[gi] : 0;
            vv[j] = ok ? vin[gi] : 0.0;
        }
    };
    // Steps 1-5 on the tile in registers (valid entries); the tile at
    // (nbase, nvalid) is loaded into the registers between staging and
    // write-out; gbase[] then points past this tile's runs.
    int rc = 0, wv = 0;  // kDerive: row containing the tile's first entry; window
    auto derive_rows = [&](long long cbase, int valid) {
        int rw = rc, wvv = wv;
        for (int round = 0;; ++round) {
            const int r = rw + 1 + t;
            if (r < m) {
                const long long p = (long long)wvv - cbase;  // >= 1: rows after rc start past cbase
                if (p < valid) atomicMax(&srow[p], r);
                else if (p == valid) atomicMax(&s_next, r);
            }
            if (t == kT - 1) s_more[round & 1] = (r < m && (long long)wvv <= cbase + valid) ? 1 : 0;
            __syncthreads();
            if (!s_more[round & 1]) break;
            rw += kT;
            wvv = rowptr[min(rw + 1 + t, m)];
        }
        int run = -1;
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            int v = srow[w * kQ + j * 64 + lane];
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int u = __shfl_up(v, off, 64);
                if (lane >= off) v = max(v, u);
            }
            v = max(v, run);
            rr[j] = v;
            run = __builtin_amdgcn_readlane(v, 63);
        }
        if (lane == 0) wmaxs[w] = run;
        __syncthreads();
        int pre = -1, all = s_next;
#pragma unroll
        for (int q = 0; q < kW; ++q) {
            const int mq = wmaxs[q];
            if (q < w) pre = max(pre, mq);
            all = max(all, mq);
        }
#pragma unroll
        for (int j = 0; j < kB; ++j) rr[j] = max(rr[j], pre);
        rc = all;  // the next tile's first entry lies in row rc
        wv = rowptr[min(rc + 1 + t, m)];
    };
    // srow = -1 everywhere but srow[0] = rc (the row of the tile's first entry)
    auto derive_init = [&]() {
#pragma unroll
        for (int j = 0; j < kB; ++j) srow[w * kQ + j * 64 + lane] = -1;
        if (t == 0) {
            srow[0] = rc;
            s_next = rc;
        }
    };
    auto process_tile = [&](int valid, long long nbase, int nvalid, long long cbase) {
        if constexpr (kDerive) derive_rows(cbase, valid);
        int lp[kB];
        // 1. wave-private ranking
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            const int d = (kk[j] >> shift) & dm;
            unsigned long long mm = ~0ull;
            for (int b = 0; b < rb; ++b) {
                const unsigned long long bal = __ballot((d >> b) & 1);
                mm &= ((d >> b) & 1) ? bal : ~bal;
            }
            const int rank = __popcll(mm & lt);
            lp[j] = wcnt[w][d] + rank;
            if (rank == 0) wcnt[w][d] += __popcll(mm);
        }
        // padding (top digit, after every real element) is not part of the output
        if (t == kT - 1 && valid < kTile) wcnt[kW - 1][dm] -= kTile - valid;
        __syncthreads();
        // 2. digit totals, per-wave starts inside each digit, exclusive scan
        constexpr int kPer = (kMaxD + kT - 1) / kT;
        int tot[kPer];
        int sum = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int d = t * kPer + k;
            int c = 0;
            if (d < D) {
#pragma unroll
                for (int q = 0; q < kW; ++q) {
                    const int v = wcnt[q][d];
                    wcnt[q][d] = c;  // this wave's start within digit d
                    c += v;
                }
            }
            tot[k] = c;
            sum += c;
        }
        const int inc = wave_incl_scan(sum);
        if (lane == 63) wtot[w] = inc;
        __syncthreads();
        int ex = inc - sum;
        for (int q = 0; q < w; ++q) ex += wtot[q];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int d = t * kPer + k;
            if (d < D) {
                lstart[d] = ex;
#pragma unroll
                for (int q = 0; q < kW; ++q) wcnt[q][d] += ex;  // absolute tile position
            }
            ex += tot[k];
        }
        __syncthreads();
        if constexpr (kSeg == kSegFinalDirect) {
            // 3'. the last pass writes a bucket's compact run: every entry
            // straight from its registers to its final place (the run's lines
            // fill within the tile, so the L2 merges them), no LDS staging
#pragma unroll
            for (int j = 0; j < kB; ++j) {
                if (w * kQ + j * 64 + lane < valid) {
                    const int d = (kk[j] >> shift) & dm;
                    const long long g = (long long)gbase[d] + (wcnt[w][d] + lp[j] - lstart[d]);
                    if (kout) kout[g] = colkey(kk[j]);
                    rout[g] = rowof(j);
                    vout[g] = vv[j];
                }
            }
            if (nvalid > 0) load_tile(nbase, nvalid);
        } else {
            if constexpr (kSeg == kSegBuckets) {
                if (pA) {  // rows from the packed pass-A words: segment (cursor walk) + offset
#pragma unroll
                    for (int j = 0; j < kB; ++j) {
                        const long long gi = cbase + min(w * kQ + j * 64 + lane, valid - 1);
                        int sgi = scur;
                        while (gi >= s_segstart[sgi + 1]) ++sgi;
                        rr[j] = s_segrow[sgi] + (int)((unsigned)kk[j] >> packA);
                        scur = __builtin_amdgcn_readlane(sgi, 63);
                    }
                }
            }
            // 3. stage in digit order
#pragma unroll
            for (int j = 0; j < kB; ++j) {
                if (w * kQ + j * 64 + lane < valid) {
                    const int pos = wcnt[w][(kk[j] >> shift) & dm] + lp[j];
                    skey[pos] = kk[j];
                    if constexpr (!kPkF) srow[pos] = rowof(j);
                    sval[pos] = vv[j];
                }
            }
            __syncthreads();
            // 4. prefetch the next tile, write this one out as per-digit runs
            if (nvalid > 0) load_tile(nbase, nvalid);
            for (int li = t; li < valid; li += kT) {
                const int k = skey[li];
                const int d = (k >> shift) & dm;
                const long long g = (long long)gbase[d] + (li - lstart[d]);
                if (kSeg == kSegTiles && kDerive && pA) {  // pass A -> pass B: low key bits + row offset
                    kout[g] = (int)(((unsigned)k & kbmask) | ((unsigned)(srow[li] - segrow0) << packA));
                } else if (!kFinal && pack >= 0) {  // pass B -> last pass: row and the low `pack` bits in one word
                    kout[g] = (srow[li] << pack) | (k & ((1 << pack) - 1));
                } else {
                    if (kout) kout[g] = colkey(k);
                    if constexpr (kPkF) rout[g] = (int)((unsigned)k >> pack);
                    else rout[g] = srow[li];
                }
                vout[g] = sval[li];
            }
        }
        __syncthreads();
        // 5. the next tile appends after this one; counters restart
        for (int d = t; d < D; d += kT) {
            const int nxt = d < dm ? lstart[d + 1] : valid;
            gbase[d] += nxt - lstart[d];
#pragma unroll
            for (int q = 0; q < kW; ++q) wcnt[q][d] = 0;
        }
        if constexpr (kDerive) derive_init();
        __syncthreads();
    };
    long long base = s0;
    int valid = base < s1 ? (int)min((long long)kTile, s1 - base) : 0;
    if (valid > 0) load_tile(base, valid);
    if constexpr (kFinal) {
        // buckets bk = blockIdx.x, + gridDim.x, ...; each: its own digit
        // histogram -> exclusive starts -> colptr for its 2^rb columns, then
        // its tiles; the next bucket's first tile is loaded while the last
        // tile of this one is written.  A one-tile bucket counts from the
        // registers of its tile, a longer one reads its keys first.
        static_assert(kMaxD <= kT, "one digit per thread");
        if (blockIdx.x == 0 && t == 0) colptr[n] = (int)nnz;
        while (bk < sg.nb) {
            if (t < D) gbase[t] = 0;
            __syncthreads();
            if (s1 - s0 <= kTile) {
#pragma unroll
                for (int j = 0; j < kB; ++j)
                    if (w * kQ + j * 64 + lane < valid) atomicAdd(&gbase[(kk[j] >> shift) & dm], 1);
            } else {
                constexpr int kU = 8;
                for (long long i0 = s0; i0 < s1; i0 += (long long)kU * kT) {
                    int d[kU];
#pragma unroll
                    for (int u = 0; u < kU; ++u) {
                        const long long i = i0 + (long long)u * kT + t;
                        d[u] = i < s1 ? ((kin[i] >> shift) & dm) : -1;
                    }
#pragma unroll
                    for (int u = 0; u < kU; ++u)
                        if (d[u] >= 0) atomicAdd(&gbase[d[u]], 1);
                }
            }
            __syncthreads();
            {
                const int c = t < D ? gbase[t] : 0;
                const int inc = wave_incl_scan(c);
                if (lane == 63) wtot[w] = inc;
                __syncthreads();
                int ex = inc - c;
                for (int q = 0; q < w; ++q) ex += wtot[q];
                if (t < D) {
                    gbase[t] = (int)s0 + ex;
                    const long long col = ((long long)bk << rb) + t;
                    if (col < n) colptr[col] = (int)s0 + ex;
#pragma unroll
                    for (int q = 0; q < kW; ++q) wcnt[q][t] = 0;
                }
                __syncthreads();
            }
            for (;;) {  // the bucket's tiles (all values workgroup-uniform)
                long long nbase = 0, ns0 = s0, ns1 = s1;
                int nvalid = 0, nbk = bk;
                if (base + kTile < s1) {
                    nbase = base + kTile;
                    nvalid = (int)min((long long)kTile, s1 - nbase);
                } else {
                    nbk = bk + (int)gridDim.x;
                    if (nbk < sg.nb) {
                        seg_range(kSegBuckets, sg, nbk, nnz, ns0, ns1);
                        nbase = ns0;
                        nvalid = (int)min((long long)kTile, ns1 - ns0);
                    }
                }
                if (valid > 0) process_tile(valid, nbase, nvalid, base);
                else if (nvalid > 0) load_tile(nbase, nvalid);
                base = nbase;
                valid = nvalid;
                if (nbk != bk) {
                    bk = nbk;
                    s0 = ns0;
                    s1 = ns1;
                    break;
                }
            }
        }
    } else {
        for (int d = t; d < D; d += kT) {
            const size_t idx = seg_count_idx(kSeg, sg, (int)blockIdx.x, D, d);
            gbase[d] = idx ? incl[idx - 1] : 0;  // exclusive start of this workgroup's run of d
#pragma unroll
            for (int q = 0; q < kW; ++q) wcnt[q][d] = 0;
        }
        if constexpr (kDerive) {
            if (valid > 0) {
                rc = wgrow[blockIdx.x];
                segrow0 = rc;
                wv = rowptr[min(rc + 1 + t, m)];
                derive_init();
            }
        }
        if constexpr (kSeg == kSegBuckets) {
            if (pA) {  // the segments' runs inside this bucket, and their first rows
                const long long i0 = (long long)(blockIdx.x / sg.J) * nseg;
                for (int i = t; i < nseg; i += kT) {
                    s_segstart[i] = (i0 + i) ? sg.prev[i0 + i - 1] : 0;
                    s_segrow[i] = wgrow[i];
                }
                if (t == 0) s_segstart[nseg] = INT_MAX;
            }
        }
        __syncthreads();
        if constexpr (kSeg == kSegBuckets) {
            if (pA && valid > 0) {  // this wave's first entry: largest i with s_segstart[i] <= p
                const long long p = min(s0 + (long long)w * kQ, s1 - 1);
                int lo = 0, hi = nseg - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_segstart[mid] <= p) lo = mid;
                    else hi = mid - 1;
                }
                scur = lo;
            }
        }
        while (valid > 0) {  // valid: workgroup-uniform
            const long long nbase = base + kTile;
            const int nvalid = nbase < s1 ? (int)min((long long)kTile, s1 - nbase) : 0;
            process_tile(valid, nbase, nvalid, base);
            base = nbase;
            valid = nvalid;
        }
    }
}

// colptr from the sorted keys: colptr[c] = first position whose key >= c
__global__ void k_colptr_sorted(const int *__restrict__ keys, long long nnz, int n, int *__restrict__ colptr)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nnz) return;
    const int k = keys[p];
    const int prev = p == 0 ? -1 : keys[p - 1];
    for (int c = prev + 1; c <= k; ++c) colptr[c] = (int)p;
    if (p == nnz - 1)
        for (int c = k + 1; c <= n; ++c) colptr[c] = (int)nnz;
}

struct TransposeScratch {
    void *buf = nullptr;
    size_t bytes = 0;
};
static thread_local TransposeScratch g_tscratch[64];

// MSD transpose (default when n > 2^9): two stable partition passes on the
// high column bits (pass A over the whole array in fixed tile segments,
// pass B inside each pass-A bucket), then one pass per final bucket of 2^c
// columns that counts, ranks and writes the bucket's run in column order
// together with its colptr entries.  Every pass is a stable partition, so
// the composition is the stable sort by column (rows ascend in a column).
// Writes: passes A and B append per-digit runs (2^7 and 2^6 digits: few
// partially written lines per workgroup); the last pass writes one
// contiguous run per workgroup and no keys (unless colidx is asked for).
struct MsdShape {
    int c = 0, bA = 0, bB = 0;
};

// Digit shapes and pass forms other than the defaults exist for experiment
// builds only (Makefile `alt`, ALT_DEFS): -DSBLAS_TRANSPOSE_MSD_C / _MSD_A
// (final / pass-A digit bits), -DSBLAS_TRANSPOSE_LSD (the LSD passes
// everywhere), -DSBLAS_TRANSPOSE_RB8 (one-tile-per-workgroup 8-bit LSD),
// _RBMAX, _WGCU, _DERIVE, _PACKA, _PACK, _DIRECT, _FTILE, _FLEAN as below.
#ifndef SBLAS_TRANSPOSE_RBMAX
#define SBLAS_TRANSPOSE_RBMAX 8
#endif
#ifndef SBLAS_TRANSPOSE_WGCU
#define SBLAS_TRANSPOSE_WGCU 2
#endif
#ifndef SBLAS_TRANSPOSE_DERIVE
#define SBLAS_TRANSPOSE_DERIVE 1
#endif
#ifndef SBLAS_TRANSPOSE_PACKA
#define SBLAS_TRANSPOSE_PACKA 1
#endif
#ifndef SBLAS_TRANSPOSE_PACK
#define SBLAS_TRANSPOSE_PACK 1
#endif
#ifndef SBLAS_TRANSPOSE_DIRECT
#define SBLAS_TRANSPOSE_DIRECT 0
#endif
#ifndef SBLAS_TRANSPOSE_FTILE
#define SBLAS_TRANSPOSE_FTILE 0
#endif
#ifndef SBLAS_TRANSPOSE_FLEAN
#define SBLAS_TRANSPOSE_FLEAN 2
#endif

static MsdShape msd_shape(int nbits, int n, long long nnz)
{
    MsdShape m;
    // final buckets of 2^c columns: the widest whose average fits one
    // 4096-entry tile with room for the spread (<= 3072 entries), so most
    // final workgroups count from the registers of their only tile
    m.c = std::min(8, nbits);
    while (m.c > 1 && nnz / std::max<long long>(1, ((long long)n + (1LL << m.c) - 1) >> m.c) > 3072) --m.c;
#ifdef SBLAS_TRANSPOSE_MSD_C
    m.c = std::max(1, std::min(8, SBLAS_TRANSPOSE_MSD_C));
#endif
    const int high = nbits - m.c;
    m.bA = (high + 1) / 2;
#ifdef SBLAS_TRANSPOSE_MSD_A
    m.bA = std::max(1, std::min(high - 1, SBLAS_TRANSPOSE_MSD_A));
#endif
    m.bB = high - m.bA;
    return m;
}

int launch_transpose(const sblas_csr_s &A, int *colptr, int *rowidx, double *cval, hipStream_t s,
                     int *colidx)
{
    const long long nnz = A.nnz;
    const int n = A.n, m = A.m;
    if (nnz == 0) {
        SBLAS_HIP(hipMemsetAsync(colptr, 0, sizeof(int) * ((size_t)n + 1), s));
        return SBLAS_OK;
    }
    int nbits = 0;
    while (nbits < 31 && (n - 1) >> nbits) ++nbits;
    // algorithm: MSD where both high passes exist (n > 2^9), else the LSD
    // passes below (experiment builds: -DSBLAS_TRANSPOSE_LSD everywhere,
    // -DSBLAS_TRANSPOSE_RB8 the one-tile-per-workgroup 8-bit LSD path)
#ifdef SBLAS_TRANSPOSE_RB8
    constexpr int rb_env = 8;
#else
    constexpr int rb_env = 0;
#endif
#ifdef SBLAS_TRANSPOSE_LSD
    constexpr bool force_lsd = true;
#else
    constexpr bool force_lsd = false;
#endif
    const MsdShape ms = msd_shape(nbits, n, nnz);
    const bool msd = rb_env != 8 && !force_lsd && ms.bA >= 1 && ms.bB >= 1 && ms.bA <= 8 && ms.bB <= 8;
    // LSD: digits of at most SBLAS_TRANSPOSE_RBMAX bits (8: a workgroup's
    // partially written digit runs -- 2^rb per array -- must fit its share
    // of the XCD's L2 until they merge; 11-bit digits measured 0.85 ms per
    // pass against ~0.3 ms), spread evenly over the passes
    const int rbmax = std::max(1, std::min(11, SBLAS_TRANSPOSE_RBMAX));
    const bool wide = rb_env != 8;
    const int passes = wide ? std::max(1, (nbits + rbmax - 1) / rbmax) : std::max(1, (nbits + 7) / 8);
    const int rb = wide ? std::max(1, (nbits + passes - 1) / passes) : 8;
    const int ntiles = (int)((nnz + kRxTile - 1) / kRxTile);
    int ncu = 256;
    {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    }
    // tiles per workgroup: one round of resident workgroups (2 per CU for
    // <= 8-bit digits, 1 per CU above)
    const int wgcu = std::max(1, SBLAS_TRANSPOSE_WGCU);
    const int S_t = wide ? std::max(1, (ntiles + ncu * wgcu - 1) / (ncu * wgcu)) : 1;
    const int nwg = (ntiles + S_t - 1) / S_t;
    // MSD pass B: J parts per pass-A bucket, about two workgroups per CU
    const int JB = msd ? std::max(1, (ncu * wgcu) >> ms.bA) : 1;
    const long long ncntA = msd ? (long long)(1 << ms.bA) * nwg : 0;
    const long long ncntB = msd ? (long long)(1 << (ms.bA + ms.bB)) * JB : 0;
    const long long ncnt = msd ? ncntA + ncntB : (wide ? (long long)(1 << rb) * nwg : 256LL * ntiles);
    const size_t scan_ints = (size_t)(ncnt / kScanTile + 64) * 2;
    // scratch: keysA rowsA valsA | keysB rowsB valsB | counts | scan (+ outputs when null)
    const size_t z = ((size_t)nnz + 3) & ~(size_t)3;  // array stride: every array 16-B aligned
    const size_t wg_ints = ((size_t)2 * nwg + 67) & ~(size_t)3;  // MSD: segment first rows + spans
    const size_t need = z * 32 + (size_t)ncnt * 4 + scan_ints * 4 + wg_ints * 4 + (rowidx ? 0 : z * 4) +
                        (cval ? 0 : z * 8) + 256;
    TransposeScratch &S = g_tscratch[A.device & 63];
    if (S.bytes < need) {
        if (S.buf) SBLAS_HIP(hipStreamSynchronize(s));  // earlier work on s may still use it
        (void)hipFree(S.buf);
        S.buf = nullptr;
        S.bytes = 0;
        SBLAS_HIP(hipMalloc(&S.buf, need));
        S.bytes = need;
    }
    char *p = (char *)S.buf;
    double *valsA = (double *)p;
    double *valsB = valsA + z;
    int *keysA = (int *)(valsB + z);
    int *rowsA = keysA + z;
    int *keysB = rowsA + z;
    int *rowsB = keysB + z;
    int *counts = rowsB + z;
    int *scan = counts + ncnt;
    int *wgrow = scan + scan_ints;
    int *rout_final = rowidx ? rowidx : wgrow + wg_ints;
    double *vout_final = cval ? cval : (double *)(((uintptr_t)(rout_final + (rowidx ? 0 : z)) + 7) & ~(uintptr_t)7);
    // MSD pass A derives the rows from rowptr (experiment builds
    // -DSBLAS_TRANSPOSE_DERIVE=0: from an expanded row array, as the LSD
    // passes do)
    const bool derive = msd && SBLAS_TRANSPOSE_DERIVE != 0;
    if (!derive)
        hipLaunchKernelGGL(k_expand_rows, dim3((m + 255) / 256), dim3(256), 0, s, A.rowptr, m, rowsB);
    if (msd) {
        int *cntA = counts, *cntB = counts + ncntA;
        // pass A: the top bA bits, fixed tile segments, (col, row, val) -> set A
        const int shA = ms.c + ms.bB;
        const SegArgs gA{S_t, nwg, nullptr, 1, 1};
        hipLaunchKernelGGL(k_rx2_count<kSegTiles>, dim3((unsigned)nwg), dim3(kCntThreads), 0, s,
                           A.col, nnz, shA, ms.bA, gA, cntA, A.rowptr, m, derive ? wgrow : nullptr);
        SBLAS_TRY(scan_inclusive(cntA, ncntA, scan, s));
        // pass A -> pass B in one word per key (low bB + c bits + row offset in
        // the segment) when the segments' row spans allow; decided on the
        // device from the spans the count pass wrote.
        const int packA = (derive && nwg <= 512 && ms.bB + ms.c <= 24 && SBLAS_TRANSPOSE_PACKA != 0)
                              ? ms.bB + ms.c : -1;
        if (derive)
            hipLaunchKernelGGL((k_rx2_scatter<256, kSegTiles, kR2Threads, true>), dim3(nwg), dim3(kR2Threads), 0, s,
                               A.col, nullptr, A.val, nnz, shA, ms.bA, gA, cntA, keysA, rowsA, valsA, nullptr, n, -1,
                               A.rowptr, m, wgrow, packA);
        else
            hipLaunchKernelGGL((k_rx2_scatter<256, kSegTiles, kR2Threads>), dim3(nwg), dim3(kR2Threads), 0, s,
                               A.col, rowsB, A.val, nnz, shA, ms.bA, gA, cntA, keysA, rowsA, valsA, nullptr, n, -1);
        // pass B: the next bB bits inside each pass-A bucket, set A -> set B.
        // Its output keeps (row << c | low c column bits) in one word when
        // they fit (the last pass needs nothing else of the key): 12 B per
        // entry written and read instead of 16.
        int mbits = 0;
        while (mbits < 31 && (m - 1) >> mbits) ++mbits;
        const int pack = (mbits + ms.c <= 31 && SBLAS_TRANSPOSE_PACK != 0) ? ms.c : -1;
        const int nwgB = (1 << ms.bA) * JB;
        const SegArgs gB{0, 0, cntA, nwg, JB};
        hipLaunchKernelGGL(k_rx2_count<kSegBuckets>, dim3((unsigned)nwgB), dim3(kCntThreads), 0,
                           s, keysA, nnz, ms.c, ms.bB, gB, cntB);
        SBLAS_TRY(scan_inclusive(cntB, ncntB, scan, s));
        if (ms.bB <= 7)  // 128 digits: smaller count tables leave LDS for the segment tables
            hipLaunchKernelGGL((k_rx2_scatter<128, kSegBuckets, kR2Threads>), dim3(nwgB), dim3(kR2Threads), 0, s, keysA,
                               rowsA, valsA, nnz, ms.c, ms.bB, gB, cntB, keysB, rowsB, valsB, nullptr, n, pack, nullptr,
                               0, wgrow, packA);
        else
            hipLaunchKernelGGL((k_rx2_scatter<256, kSegBuckets, kR2Threads>), dim3(nwgB), dim3(kR2Threads), 0, s, keysA,
                               rowsA, valsA, nnz, ms.c, ms.bB, gB, cntB, keysB, rowsB, valsB, nullptr, n, pack, nullptr,
                               0, wgrow, packA);
        // last pass: one workgroup per pass-B bucket (2^c columns), set B -> CSC + colptr
        const int nbC = 1 << (ms.bA + ms.bB);
        // SBLAS_TRANSPOSE_DIRECT=1 (experiment builds): entries written from registers
        constexpr bool direct = SBLAS_TRANSPOSE_DIRECT == 1;
        const SegArgs gC{0, 0, cntB, JB, 1, nbC};
        // final tile: 3072 entries (6 per thread) when the buckets average <=
        // 2600 -- uniform columns then fit one tile (spread ~ sqrt(avg)) with
        // 83% of its lanes busy instead of 62% in a 4096 tile; fuller buckets
        // keep the 4096 tile (experiment builds: SBLAS_TRANSPOSE_FTILE=4096 forces it)
        const long long favg = nnz / std::max(1, nbC);
        const bool small_tile = SBLAS_TRANSPOSE_FTILE ? SBLAS_TRANSPOSE_FTILE == 3072 : favg <= 2600;
        auto kfin = direct
                        ? (small_tile ? k_rx2_scatter<256, kSegFinalDirect, kR2Threads, false, 3072>
                                      : k_rx2_scatter<256, kSegFinalDirect, kR2Threads>)
                        : (small_tile ? k_rx2_scatter<256, kSegFinal, kR2Threads, false, 3072>
                                      : k_rx2_scatter<256, kSegFinal, kR2Threads>);
        // lean last pass (packed input, <= 7 final bits, 3072 tile; default):
        // no row staging and 128-digit tables leave 42 KB of LDS, and 80
        // VGPRs, so three workgroups share a CU (config 2: 332 -> 290 us).
        // Experiment builds: SBLAS_TRANSPOSE_FLEAN=1 lean at two per CU, =0 the staged form.
        const int flean = (pack >= 0 && ms.c <= 7 && small_tile && !direct) ? SBLAS_TRANSPOSE_FLEAN : 0;
        int fgrid = std::min(nbC, ncu * wgcu);
        if (flean == 1) kfin = k_rx2_scatter<128, kSegFinal, kR2Threads, false, 3072, true, 1>;
        if (flean == 2) {
            kfin = k_rx2_scatter<128, kSegFinal, kR2Threads, false, 3072, true, 6>;
            fgrid = std::min(nbC, ncu * 3);
        }
        hipLaunchKernelGGL(kfin, dim3((unsigned)fgrid), dim3(kR2Threads), 0, s,
                           keysB, pack >= 0 ? nullptr : rowsB, valsB, nnz, 0, ms.c, gC, nullptr, colidx, rout_final,
                           vout_final, colptr, n, pack, nullptr, 0, nullptr, -1);
        SBLAS_HIP(hipGetLastError());
        return SBLAS_OK;
    }
    const int *kin = A.col, *rin = rowsB;
    const double *vin = A.val;
    for (int ps = 0; ps < passes; ++ps) {
        const int shift = 8 * ps;
        const bool last = ps == passes - 1;
        // pass ps reads set (ps even: input/B, odd: A) and writes the other
        int *ko = (ps & 1) ? keysB : keysA;
        int *ro = last ? rout_final : ((ps & 1) ? rowsB : rowsA);
        double *vo = last ? vout_final : ((ps & 1) ? valsB : valsA);
        if (wide) {
            const int sh = rb * ps;
            const SegArgs gt{S_t, nwg, nullptr, 1, 1};
            hipLaunchKernelGGL(k_rx2_count<kSegTiles>, dim3((unsigned)nwg), dim3(kCntThreads), 0, s,
                               kin, nnz, sh, rb, gt, counts);
            SBLAS_TRY(scan_inclusive(counts, ncnt, scan, s));
            if (rb <= 8)  // 71 KiB of LDS: two workgroups per CU
                hipLaunchKernelGGL((k_rx2_scatter<256, kSegTiles, kR2Threads>), dim3(nwg), dim3(kR2Threads), 0, s, kin, rin, vin,
                                   nnz, sh, rb, gt, counts, ko, ro, vo, nullptr, n, -1);
            else
                hipLaunchKernelGGL((k_rx2_scatter<kRx2MaxDigits, kSegTiles, kR2Threads>), dim3(nwg), dim3(kR2Threads), 0, s, kin,
                                   rin, vin, nnz, sh, rb, gt, counts, ko, ro, vo, nullptr, n, -1);
        } else {
            hipLaunchKernelGGL(k_rx_count, dim3(ntiles), dim3(kRxThreads), 0, s, kin, nnz, shift, ntiles, counts);
            SBLAS_TRY(scan_inclusive(counts, ncnt, scan, s));
            hipLaunchKernelGGL(k_rx_scatter, dim3(ntiles), dim3(kRxThreads), 0, s, kin, rin, vin, nnz, shift,
                               ntiles, counts, ko, ro, vo);
        }
        kin = ko;
        rin = ro;
        vin = vo;
    }
    hipLaunchKernelGGL(k_colptr_sorted, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, kin, nnz, n,
                       colptr);
    if (colidx)  // column of every CSC entry (the sorted keys)
        SBLAS_HIP(hipMemcpyAsync(colidx, kin, sizeof(int) * (size_t)nnz, hipMemcpyDeviceToDevice, s));
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

// ---- multi-device CSR -> CSC (sptrans_v1 kernal_sptrans,
// sptrans/sptrans_v1/src/sptrans_kernal.h:80-555) -------------------------
// Rows are split into g nnz-balanced blocks of whole rows; block d is
// transposed on device d % count by the single-device path above (stable:
// rows ascend within a column; its sorted keys give every entry's column).
// The pieces then travel to device 0 (peer DMA over xGMI) and one
// element-parallel kernel composes them: block d's column
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
                              int g, int n, long long nnz, const int *__restrict__ key_cat,
                              const int *__restrict__ rid_cat, const double *__restrict__ val_cat,
                              int *__restrict__ rowidx, double *__restrict__ cval)
{
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= nnz) return;
    int d = 0;
    while (d + 1 < g && start[d + 1] <= p) ++d;
    const int e = (int)(p - start[d]);
    const int c = key_cat[p];  // column of this entry (block-local CSC order)
    const int dst = base[(size_t)d * n + c] + (e - ptrs[(size_t)d * (n + 1) + c]);
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
        int *cp = nullptr, *ri = nullptr, *ck = nullptr;
        double *cv = nullptr;
        hipStream_t s = nullptr;
    };
    std::vector<Blk> B(g);
    // one stream per physical device: blocks that wrap onto the same GPU run
    // in order (they share that device's transpose scratch)
    std::vector<hipStream_t> streams((size_t)std::min(count, g), nullptr);
    int *h_ptrs = nullptr, *h_base = nullptr, *h_rid = nullptr, *h_row0 = nullptr, *h_cp = nullptr,
        *h_ri = nullptr, *h_key = nullptr;
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
            (void)hipFree(b.ck);
        }
        for (size_t p = 0; p < streams.size(); ++p)
            if (streams[p]) {
                DeviceGuard gd((int)p);
                (void)hipStreamDestroy(streams[p]);
            }
        DeviceGuard gd(0);
        for (void *p : {(void *)h_ptrs, (void *)h_base, (void *)h_rid, (void *)h_row0, (void *)h_cp,
                        (void *)h_ri, (void *)h_val, (void *)h_cv, (void *)h_start, (void *)h_key})
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
        TG(hipMalloc(&b.ck, sizeof(int) * std::max(e1 - e0, 1)));
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
        TG(hipMalloc(&h_key, sizeof(int) * std::max(nnz, 1)));
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
        const int st = launch_transpose(b.A, b.cp, b.ri, b.cv, b.s, b.ck);
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
                TG(hipMemcpyPeerAsync(h_key + start[d], 0, b.ck, b.phys, sizeof(int) * k, s0));
                TG(hipMemcpyPeerAsync(h_val + start[d], 0, b.cv, b.phys, sizeof(double) * k, s0));
            }
        }
        hipLaunchKernelGGL(k_compose_ptr, dim3((n + 1 + 255) / 256), dim3(256), 0, s0, h_ptrs, g, n, h_cp,
                           h_base);
        if (nnz && n > 0)
            hipLaunchKernelGGL(k_compose_val, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s0, h_ptrs,
                               h_base, h_start, h_row0, g, n, (long long)nnz, h_key, h_rid, h_val, h_ri, h_cv);
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
