// spmv.hip -- fp64 CSR SpMV kernels for gfx950 (MI355X).
//
// Replaces the per-device cusparseDcsrmv / cusparseDcsrmv_mp calls of
// spmv/src/dspmv_mgpu_baseline.cu:163-167 and dspmv_mgpu_v1.cu:199-210, and
// the (disabled) CSR5 library spmv/include/detail/cuda/csr5_spmv_cuda.h.
//
//  * Row split ("kernel 1"): CSR-adaptive row blocks. One 256-thread
//    workgroup per block of whole rows holding <= 2048 nnz; val/col are
//    streamed with 16-byte non-temporal loads (fully coalesced, they are read
//    once), products val*x[col] land in LDS, then a power-of-two group of
//    lanes per row (1..64, chosen from the block's row count) reduces each
//    row from LDS with wave shuffles.  Rows longer than a block are split in
//    8192-nnz chunks, one workgroup each, combined by a tiny finalize pass.
//  * CSR5-style segmented sum ("kernel 2/3"): wave64 tiles of 64 lanes x 16
//    nnz.  Values/columns are stored tile-transposed so every lane issues
//    16-byte loads and a wave reads 1 KiB contiguous per instruction; a
//    32-bit row-start mask per lane replaces CSR5's 32-lane bit-flag
//    descriptor.  Lane-local segmented sums, then a 6-step suffix segmented
//    scan across the wave joins rows that cross lanes; rows that cross tiles
//    are completed by a calibration pass (csr5_spmv_cuda.h:313-382 analogue).
//  * alpha/beta are honoured by both (the reference's CSR5 ignored them, Q4);
//    beta == 0 never reads y (BLAS/cuSPARSE convention).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <vector>

#include "sblas_internal.hpp"

namespace sblas {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v4i ld_nt_v4i(const int *p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const v4i *>(p));
}
__device__ __forceinline__ v2d ld_nt_v2d(const double *p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p));
}

// ---------------------------------------------------------------------------
// Row split
// ---------------------------------------------------------------------------
// One row block (stream or long-row chunk) of a CSR: shared by the plain
// row-split kernel and the XCD-panel kernel (which runs it on column panels).
template <bool kBeta, bool kSc1 = false>
__device__ __forceinline__ void store_y(double *p, double v)
{
    if (kSc1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

#ifndef SBLAS_RS_SEQ  // experiment builds only (Makefile `alt`): 0 = the vec4 order
#define SBLAS_RS_SEQ 1
#endif
// kSeq (default; an experiment build with SBLAS_RS_SEQ=0 selects the earlier
// form for the row-split launch): the stream block's entries are taken lane-consecutively
// -- thread t holds entries j0 + t + 256k, so one gather instruction of a
// wave covers 64 CONSECUTIVE entries and the TA merges lanes whose columns
// share an x line (a banded / stencil row's runs of neighbouring columns) --
// with 4-B / 8-B col / val loads, instead of 16-B loads of 4 consecutive
// entries per lane, whose gather instructions sample every 4th entry.
// Measured (row split, cold, `profiles/r03/rowsplit_seq/`): 27-point stencil
// 0.549 -> 0.615 of 8 TB/s, 7-point 0.577 -> 0.625, config 2 prefix columns
// 0.674 -> 0.708, random 0.208 -> 0.217.
template <bool kBeta, bool kSc1 = false, bool kSeq = true>
__device__ __forceinline__ void rowsplit_block(
    const RowBlock blk, const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x, double alpha, double beta,
    double *__restrict__ y, double *__restrict__ partial, double *__restrict__ prod,
    double *__restrict__ wsum)
{
    const int tid = threadIdx.x;

    if (blk.a >= 0) {
        // ---- stream block: rows [r0, r1), nnz <= kRsBlockNnz -------------
        const int r0 = blk.row, r1 = blk.a;
        const int j0 = rowptr[r0], j1 = rowptr[r1];
        const int base = j0 & ~3;
        const int ngroups = kSeq ? 0 : (j1 - base + 3) >> 2;
        if (kSeq && j1 > j0) {  // block-uniform
            constexpr int K = kRsBlockNnz / kRsThreads;
            static_assert(K * kRsThreads == kRsBlockNnz, "a stream block is K entries per thread");
            int c[K];
            double v[K], xv[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {  // clamped, unconditional (see below)
                const int e = min(j0 + k * kRsThreads + tid, j1 - 1);
                c[k] = __builtin_nontemporal_load(col + e);
                v[k] = __builtin_nontemporal_load(val + e);
            }
#pragma unroll
            for (int k = 0; k < K; ++k) xv[k] = x[c[k]];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int e = j0 + k * kRsThreads + tid;
                if (e < j1) prod[e - j0] = v[k] * xv[k];
            }
        }
        // Two 4-element groups per thread per pass, all loads issued before any
        // use.  Gathers are UNCONDITIONAL: the 16-B over-read window only ever
        // holds neighbouring rows' columns or the zeroed padding, so every index
        // is valid, and a per-element branch would make hipcc wait vmcnt(0)
        // after each gather (one gather in flight per lane).
        for (int g = tid; g < ngroups; g += 2 * kRsThreads) {
            const int g2 = g + kRsThreads;
            const bool has2 = g2 < ngroups;
            const int e = base + 4 * g;
            const int e2 = base + 4 * (has2 ? g2 : g);
            const v4i c = ld_nt_v4i(col + e);
            const v4i c2 = ld_nt_v4i(col + e2);
            const v2d va = ld_nt_v2d(val + e);
            const v2d vb = ld_nt_v2d(val + e + 2);
            const v2d va2 = ld_nt_v2d(val + e2);
            const v2d vb2 = ld_nt_v2d(val + e2 + 2);
            const double x0 = x[c.x], x1 = x[c.y], x2 = x[c.z], x3 = x[c.w];
            const double x4 = x[c2.x], x5 = x[c2.y], x6 = x[c2.z], x7 = x[c2.w];
            const double p[8] = {va.x * x0, va.y * x1, vb.x * x2, vb.y * x3,
                                 va2.x * x4, va2.y * x5, vb2.x * x6, vb2.y * x7};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int idx = e + k;
                if (idx >= j0 && idx < j1) prod[idx - j0] = p[k];
            }
            if (has2) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int idx = e2 + k;
                    if (idx >= j0 && idx < j1) prod[idx - j0] = p[4 + k];
                }
            }
        }
        __syncthreads();
        const int nrows = r1 - r0;
        int tpr = nrows > 0 ? kRsThreads / nrows : 64;
        tpr = tpr >= 64 ? 64 : tpr >= 32 ? 32 : tpr >= 16 ? 16 : tpr >= 8 ? 8
            : tpr >= 4 ? 4 : tpr >= 2 ? 2 : 1;
        const int grp = tid / tpr, lane = tid & (tpr - 1);
        const int ngrp = kRsThreads / tpr;
        for (int r = r0 + grp; r < r1; r += ngrp) {
            const int a = rowptr[r] - j0, b = rowptr[r + 1] - j0;
            double s = 0.0;
            for (int k = a + lane; k < b; k += tpr) s += prod[k];
            for (int off = tpr >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
            if (lane == 0) store_y<kBeta, kSc1>(&y[r], kBeta ? alpha * s + beta * y[r] : alpha * s);
        }
    } else {
        // ---- long-row chunk ------------------------------------------------
        const int r = blk.row, k = -blk.a - 1;
        const int rs = rowptr[r], re = rowptr[r + 1];
        const int j0 = rs + k * kRsLongChunk;
        const int j1 = min(re, j0 + kRsLongChunk);
        const int base = j0 & ~3;
        const int ngroups = (j1 - base + 3) >> 2;
        double s = 0.0;
        for (int g = tid; g < ngroups; g += kRsThreads) {
            const int e = base + 4 * g;
            const v4i c = ld_nt_v4i(col + e);
            const v2d va = ld_nt_v2d(val + e);
            const v2d vb = ld_nt_v2d(val + e + 2);
            const double xv[4] = {x[c.x], x[c.y], x[c.z], x[c.w]};  // unconditional
            const double v[4] = {va.x, va.y, vb.x, vb.y};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int idx = e + q;
                s += (idx >= j0 && idx < j1) ? v[q] * xv[q] : 0.0;
            }
        }
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if ((tid & 63) == 0) wsum[tid >> 6] = s;
        __syncthreads();
        if (tid == 0) {
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < kRsThreads / 64; ++w) t += wsum[w];
            if (blk.b < 0) store_y<kBeta, kSc1>(&y[r], kBeta ? alpha * t + beta * y[r] : alpha * t);
            else partial[blk.b] = t;
        }
    }
}

template <bool kBeta, bool kSeq = true>
__global__ __launch_bounds__(kRsThreads) void k_spmv_rowsplit(
    const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, const double *__restrict__ x,
    const RowBlock *__restrict__ blocks, double alpha, double beta,
    double *__restrict__ y, double *__restrict__ partial)
{
    __shared__ double prod[kRsBlockNnz + 8];
    __shared__ double wsum[kRsThreads / 64];
    rowsplit_block<kBeta, false, kSeq>(blocks[blockIdx.x], rowptr, col, val, x, alpha, beta, y, partial, prod,
                                       wsum);
}

template <bool kBeta>
__global__ void k_spmv_long_finalize(const int4 *__restrict__ long_rows, int nlong,
                                     const double *__restrict__ partial,
                                     double alpha, double beta,
                                     double *__restrict__ y)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlong) return;
    const int4 L = long_rows[i];
    double s = 0.0;
    for (int q = 0; q < L.z; ++q) s += partial[L.y + q];
    y[L.x] = kBeta ? alpha * s + beta * y[L.x] : alpha * s;
}

// Greedy CSR-adaptive blocking of rows [0, m): whole rows up to kRsBlockNnz
// nnz / kRsMaxRows rows per block; longer rows in kRsLongChunk chunks (slot
// numbers continue from `nslots`).
void make_row_blocks(const int *rp, int m, std::vector<RowBlock> &blocks,
                     std::vector<int4> &longs, int &nslots)
{
    int r = 0;
    while (r < m) {
        const int len = rp[r + 1] - rp[r];
        if (len > kRsBlockNnz) {
            const int nch = (len + kRsLongChunk - 1) / kRsLongChunk;
            if (nch == 1) {
                blocks.push_back({r, -1, -1, 0});
            } else {
                longs.push_back(make_int4(r, nslots, nch, 0));
                for (int k = 0; k < nch; ++k) blocks.push_back({r, -1 - k, nslots + k, 0});
                nslots += nch;
            }
            ++r;
            continue;
        }
        const int start = r;
        int nz = 0;
        while (r < m && r - start < kRsMaxRows) {
            const int l = rp[r + 1] - rp[r];
            if (l > kRsBlockNnz || nz + l > kRsBlockNnz) break;
            nz += l;
            ++r;
        }
        blocks.push_back({start, r, 0, 0});
    }
}

// Whether a row-oriented kernel (row split, CSR5) should run over XCD column
// panels (~4 MiB of x each, P = 4 partials added after): x outgrows an XCD's
// L2, the rows' columns are scattered (the column probe: most sampled rows
// span > n/4 of the columns, spread over the eighths) and the matrix is large
// enough to amortise the partial-y pass (`min_nnz`).  Measured on the uniform
// config 2 and its rank slices (cold spans, profiles/r05/sweep/, c5P/; plain
// / 4 panels): CSR5 567 / 287 us at N = 1, 77 / 46 (heavy) and 80 / 60
// (light rows) on configs[2]'s N = 8 ranks (5M entries), 45 / 38 on a 2.5M
// cyclic slice, 29.6 / 30.4 on 1.2M; the row split alike (573 / 310, 76 / 47,
// 79 / 58, 42 / 32, 24 / 25).  So both take panels from 2M entries.
// (Rounds 1-4 set 8M / 4M thresholds and 2 panels on short rows on the
// correlated generator, profiles/r05/gen/, whose heavy rows shared x lines.)
// The test hook `opt` ("rs_panel" / "csr5_panel", sblas_test_set_option)
// = 1 / 0 forces either form.
constexpr long long kPanelMinNnz = 2000000LL;
constexpr long long kC5WidePanelNnz = 32000000LL;  // CSR5: 2 MiB x panels from here (build_csr5_plan)
static int xcd_panels_pay(sblas_csr_s &A, hipStream_t s, const char *opt, long long min_nnz, bool *use)
{
    *use = false;
    double v = 0.0;
    if (test_option(opt, &v)) {
        *use = v == 1.0;
        return SBLAS_OK;
    }
    if ((long long)A.n * 8 <= (8LL << 20) || A.nnz < min_nnz) return SBLAS_OK;
    SBLAS_TRY(probe_columns(A, s));
    *use = A.col_scattered >= 0.5 && A.col_maxshare <= 0.25;
    return SBLAS_OK;
}

int build_rowsplit_plan(sblas_csr_s &A, hipStream_t s)
{
    if (A.rs.ready) return SBLAS_OK;
    DeviceGuard g(A.device);
    // the vec4 entry order only in experiment builds (Makefile `alt`,
    // -DSBLAS_RS_SEQ=0)
    A.rs.seq = SBLAS_RS_SEQ != 0;
    // the same row blocks per XCD column panel on large scattered matrices
    // (the panel plan, algo 4's layout; test hook "rs_panel"): decided
    // first, so a panel plan never keeps a second, unused set of row blocks
    if (!A.pn.degenerate) {
        bool use = false;
        SBLAS_TRY(xcd_panels_pay(A, s, "rs_panel", kPanelMinNnz, &use));
        if (use) {
            SBLAS_TRY(build_panel_plan(A, s));
            if (!A.pn.degenerate) {
                A.rs.panels = true;
                A.rs.ready = true;
                return SBLAS_OK;
            }
        }
    }
    std::vector<RowBlock> blocks;
    std::vector<int4> longs;
    blocks.reserve(A.nnz / kRsBlockNnz + A.m / kRsMaxRows + 16);
    int nslots = 0;
    make_row_blocks(A.h_rowptr.data(), A.m, blocks, longs, nslots);
    A.rs.nblocks = (int)blocks.size();
    A.rs.nlong = (int)longs.size();
    A.rs.nslots = nslots;
    if (A.rs.nblocks) {
        SBLAS_HIP(hipMalloc(&A.rs.blocks, sizeof(RowBlock) * blocks.size()));
        SBLAS_HIP(hipMemcpyAsync(A.rs.blocks, blocks.data(), sizeof(RowBlock) * blocks.size(),
                                 hipMemcpyHostToDevice, s));
    }
    if (A.rs.nlong) {
        SBLAS_HIP(hipMalloc(&A.rs.long_rows, sizeof(int4) * longs.size()));
        SBLAS_HIP(hipMemcpyAsync(A.rs.long_rows, longs.data(), sizeof(int4) * longs.size(),
                                 hipMemcpyHostToDevice, s));
        SBLAS_HIP(hipMalloc(&A.rs.partial, sizeof(double) * nslots));
    }
    SBLAS_HIP(hipStreamSynchronize(s));
    A.rs.ready = true;  // only once every step above has succeeded
    return SBLAS_OK;
}

// Row-split launch on raw device arrays (the out-of-core executor's chunks,
// stream.hip).
int launch_rowsplit_raw(const int *rowptr, const int *col, const double *val, const double *x,
                        const RowBlock *blocks, int nblocks, const int4 *long_rows, int nlong,
                        double *partial, double alpha, double beta, double *y, hipStream_t s)
{
    if (nblocks == 0) return SBLAS_OK;
    if (beta != 0.0) {
        SBLAS_LAUNCH(k_spmv_rowsplit<true>, dim3(nblocks), dim3(kRsThreads), 0, s, rowptr, col, val,
                           x, blocks, alpha, beta, y, partial);
        if (nlong)
            SBLAS_LAUNCH(k_spmv_long_finalize<true>, dim3((nlong + 63) / 64), dim3(64), 0, s,
                               long_rows, nlong, partial, alpha, beta, y);
    } else {
        SBLAS_LAUNCH(k_spmv_rowsplit<false>, dim3(nblocks), dim3(kRsThreads), 0, s, rowptr, col, val,
                           x, blocks, alpha, beta, y, partial);
        if (nlong)
            SBLAS_LAUNCH(k_spmv_long_finalize<false>, dim3((nlong + 63) / 64), dim3(64), 0, s,
                               long_rows, nlong, partial, alpha, beta, y);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

int launch_spmv_rowsplit(const sblas_csr_s &A, double alpha, const double *x,
                         double beta, double *y, hipStream_t s)
{
    if (!A.rs.ready) return SBLAS_ERR_INVALID;
    if (A.rs.panels) return launch_spmv_panel(A, alpha, x, beta, y, s);
    if (A.rs.nblocks == 0) return SBLAS_OK;
    const bool seq = A.rs.seq;
    if (beta != 0.0) {
        auto kern = seq ? k_spmv_rowsplit<true, true> : k_spmv_rowsplit<true, false>;
        SBLAS_LAUNCH(kern, dim3(A.rs.nblocks), dim3(kRsThreads), 0, s,
                           A.rowptr, A.col, A.val, x, A.rs.blocks, alpha, beta, y, A.rs.partial);
        if (A.rs.nlong)
            SBLAS_LAUNCH(k_spmv_long_finalize<true>, dim3((A.rs.nlong + 63) / 64), dim3(64),
                               0, s, A.rs.long_rows, A.rs.nlong, A.rs.partial, alpha, beta, y);
    } else {
        auto kern = seq ? k_spmv_rowsplit<false, true> : k_spmv_rowsplit<false, false>;
        SBLAS_LAUNCH(kern, dim3(A.rs.nblocks), dim3(kRsThreads), 0, s,
                           A.rowptr, A.col, A.val, x, A.rs.blocks, alpha, beta, y, A.rs.partial);
        if (A.rs.nlong)
            SBLAS_LAUNCH(k_spmv_long_finalize<false>, dim3((A.rs.nlong + 63) / 64), dim3(64),
                               0, s, A.rs.long_rows, A.rs.nlong, A.rs.partial, alpha, beta, y);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

// ---------------------------------------------------------------------------
// CSR5-style wave64 tiles
// ---------------------------------------------------------------------------
// Storage position of element (lane l, k) of a tile, k in [0, 16):
//   values : pairs  -> (k/2)*128 + 2l + (k&1)   (16-B loads, 1 KiB per wave)
//   columns: quads  -> (k/4)*256 + 4l + (k&3)
__device__ __forceinline__ int c5_vpos(int l, int k) { return (k >> 1) * 128 + 2 * l + (k & 1); }
__device__ __forceinline__ int c5_cpos(int l, int k) { return (k >> 2) * 256 + 4 * l + (k & 3); }

__global__ void k_c5_transpose(const int *__restrict__ col, const double *__restrict__ val,
                               long long nnz, long long total, int *__restrict__ tcol,
                               double *__restrict__ tval)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const long long t = e / kC5Tile;
    const int w = (int)(e - t * kC5Tile);
    const int l = w / kC5Sigma, k = w % kC5Sigma;
    const bool in = e < nnz;
    tval[t * kC5Tile + c5_vpos(l, k)] = in ? val[e] : 0.0;
    tcol[t * kC5Tile + c5_cpos(l, k)] = in ? col[e] : 0;
}

// One wave64 tile t of a CSR5 plan (caller: t < ntiles, wave-uniform).
// (csr5_tile_pf below is the same tile with its loads issued in phases.)
template <bool kBeta>
__device__ __forceinline__ void csr5_tile(
    long long t, const int *__restrict__ tile_row, const uint32_t *__restrict__ flags,
    const double *__restrict__ tval, const int *__restrict__ tcol,
    const int *__restrict__ seg_off, const int *__restrict__ seg_row,
    const double *__restrict__ x, long long ntiles, long long nnz, double alpha,
    double beta, double *__restrict__ y, double *__restrict__ carry)
{
    const int lane = threadIdx.x & 63;
    const double *tv = tval + t * kC5Tile;
    const int *tc = tcol + t * kC5Tile;
    const uint32_t f = flags[t * 64 + lane];
    const int trow = tile_row[t];
    const bool gap = trow < 0;  // bit31: tile contains empty rows
    const int r0 = trow & 0x7fffffff;

    double p[kC5Sigma];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        const v4i c = ld_nt_v4i(tc + q * 256 + 4 * lane);
        const v2d va = ld_nt_v2d(tv + (2 * q) * 128 + 2 * lane);
        const v2d vb = ld_nt_v2d(tv + (2 * q + 1) * 128 + 2 * lane);
        p[4 * q + 0] = va.x * x[c.x];
        p[4 * q + 1] = va.y * x[c.y];
        p[4 * q + 2] = vb.x * x[c.z];
        p[4 * q + 3] = vb.y * x[c.w];
    }
    if (t == ntiles - 1) {  // zero the padding past nnz (x[0] may be inf/nan)
        const long long e0 = t * kC5Tile + (long long)lane * kC5Sigma;
#pragma unroll
        for (int k = 0; k < kC5Sigma; ++k)
            if (e0 + k >= nnz) p[k] = 0.0;
    }

    // Exclusive prefix count of row starts over lanes -> segment index base.
    const int cnt = __popc(f);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const int segbase = incl - cnt;
    const uint32_t f0 = __shfl(f, 0, 64);
    const int first_row = (f0 & 1u) ? r0 : r0 + 1;  // row of segment 0 (no gaps)
    const int soff = gap ? seg_off[t] : 0;

    double head = 0.0, sum = 0.0;
    int seg = -1;
#pragma unroll
    for (int k = 0; k < kC5Sigma; ++k) {
        if ((f >> k) & 1u) {
            if (seg < 0) {
                head = sum;
                seg = segbase;
            } else {
                const int row = gap ? seg_row[soff + seg] : first_row + seg;
                y[row] = kBeta ? __builtin_fma(beta, y[row], alpha * sum) : alpha * sum;
                ++seg;
            }
            sum = 0.0;
        }
        sum += p[k];
    }
    const bool has = seg >= 0;
    if (!has) head = sum;

    // Suffix segmented scan: S_l = head_l + (has_l ? 0 : S_{l+1}).
    double S = head;
    bool stop = has;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double vS = __shfl_down(S, off, 64);
        const int vstop = __shfl_down((int)stop, off, 64);
        if (!stop) {
            if (lane + off < 64) {
                S += vS;
                stop = vstop != 0;
            } else {
                stop = true;
            }
        }
    }
    double Snext = __shfl_down(S, 1, 64);
    if (lane == 63) Snext = 0.0;
    if (has) {
        const int row = gap ? seg_row[soff + seg] : first_row + seg;
        const double tot = sum + Snext;
        y[row] = kBeta ? __builtin_fma(beta, y[row], alpha * tot) : alpha * tot;
    }
    if (lane == 0) carry[t] = (f0 & 1u) ? 0.0 : S;
}


// The same tile with every load of a lane issued before the first use, in
// phases the compiler may not interleave (sched_barrier):
//   1. the stream (col quads, value pairs) and the tile's flags;
//   2. the scan of row starts (shuffles, no memory), then -- gap tiles only --
//      the rows of the lane's first kC5Pre segment ends;
//   3. all 16 x gathers and the beta*y inputs of those kC5Pre rows;
//   4. products, the segmented sum and the y stores.
// The plain form lets the compiler interleave gathers with products (~8 in
// flight per lane) and loads each row end's y inside the sum loop, one
// dependent round trip per row end: on config 2's 9-entry rows (~2 row ends
// per lane) that made the light rows alone take 215 us
// (profiles/r04/split/).  Results are bit-identical to the plain form (same
// products, same summation order).
constexpr int kC5Pre = 4;
template <bool kBeta>
__device__ __forceinline__ void csr5_tile_pf(
    long long t, const int *__restrict__ tile_row, const uint32_t *__restrict__ flags,
    const double *__restrict__ tval, const int *__restrict__ tcol,
    const int *__restrict__ seg_off, const int *__restrict__ seg_row,
    const double *__restrict__ x, long long ntiles, long long nnz, double alpha,
    double beta, double *__restrict__ y, double *__restrict__ carry)
{
    const int lane = threadIdx.x & 63;
    const double *tv = tval + t * kC5Tile;
    const int *tc = tcol + t * kC5Tile;
    const uint32_t f = flags[t * 64 + lane];
    const int trow = tile_row[t];
    const bool gap = trow < 0;  // bit31: tile contains empty rows (wave-uniform)
    const int r0 = trow & 0x7fffffff;
    v4i cq[kC5Sigma / 4];
    v2d vq[kC5Sigma / 2];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        cq[q] = ld_nt_v4i(tc + q * 256 + 4 * lane);
        vq[2 * q] = ld_nt_v2d(tv + (2 * q) * 128 + 2 * lane);
        vq[2 * q + 1] = ld_nt_v2d(tv + (2 * q + 1) * 128 + 2 * lane);
    }
    const int soff = gap ? seg_off[t] : 0;
    __builtin_amdgcn_sched_barrier(0);

    // exclusive prefix count of row starts over lanes -> segment index base
    const int cnt = __popc(f);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const int segbase = incl - cnt;
    const uint32_t f0 = __shfl(f, 0, 64);
    const int first_row = (f0 & 1u) ? r0 : r0 + 1;  // row of segment 0 (no gaps)
    // rows of the lane's first kC5Pre segment ends (index clamped into the
    // lane's own segments; a lane without any reads the tile's first slot --
    // a gap tile holds at least one row start -- and ignores it)
    int qr[kC5Pre];
    const int last = cnt - 1;
    if (gap) {
#pragma unroll
        for (int j = 0; j < kC5Pre; ++j) qr[j] = seg_row[cnt > 0 ? soff + segbase + (j < last ? j : last) : soff];
    } else {
#pragma unroll
        for (int j = 0; j < kC5Pre; ++j) qr[j] = first_row + segbase + j;
    }
    __builtin_amdgcn_sched_barrier(0);

    double xv[kC5Sigma];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        xv[4 * q + 0] = x[cq[q].x];
        xv[4 * q + 1] = x[cq[q].y];
        xv[4 * q + 2] = x[cq[q].z];
        xv[4 * q + 3] = x[cq[q].w];
    }
    double qy[kC5Pre];
#pragma unroll
    for (int j = 0; j < kC5Pre; ++j) qy[j] = 0.0;
    if (kBeta) {
#pragma unroll
        for (int j = 0; j < kC5Pre; ++j)
            if (j < cnt) qy[j] = y[qr[j]];
    }
    __builtin_amdgcn_sched_barrier(0);

    double p[kC5Sigma];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        p[4 * q + 0] = vq[2 * q].x * xv[4 * q + 0];
        p[4 * q + 1] = vq[2 * q].y * xv[4 * q + 1];
        p[4 * q + 2] = vq[2 * q + 1].x * xv[4 * q + 2];
        p[4 * q + 3] = vq[2 * q + 1].y * xv[4 * q + 3];
    }
    if (t == ntiles - 1) {  // zero the padding past nnz (x[0] may be inf/nan)
        const long long e0 = t * kC5Tile + (long long)lane * kC5Sigma;
#pragma unroll
        for (int k = 0; k < kC5Sigma; ++k)
            if (e0 + k >= nnz) p[k] = 0.0;
    }
    // row ends in segment order: the prefetched ones first (shift register,
    // no dynamic register index), then loaded on the spot
    int nq = 0;
    auto next_row = [&](int sg, double &yin) {
        int row;
        if (nq < kC5Pre) {
            row = qr[0];
            yin = qy[0];
#pragma unroll
            for (int j = 0; j + 1 < kC5Pre; ++j) {
                qr[j] = qr[j + 1];
                qy[j] = qy[j + 1];
            }
        } else {
            row = gap ? seg_row[soff + sg] : first_row + sg;
            yin = kBeta ? y[row] : 0.0;
        }
        ++nq;
        return row;
    };

    double head = 0.0, sum = 0.0;
    int seg = -1;
#pragma unroll
    for (int k = 0; k < kC5Sigma; ++k) {
        if ((f >> k) & 1u) {
            if (seg < 0) {
                head = sum;
                seg = segbase;
            } else {
                double yin;
                const int row = next_row(seg, yin);
                y[row] = kBeta ? __builtin_fma(beta, yin, alpha * sum) : alpha * sum;
                ++seg;
            }
            sum = 0.0;
        }
        sum += p[k];
    }
    const bool has = seg >= 0;
    if (!has) head = sum;

    // suffix segmented scan: S_l = head_l + (has_l ? 0 : S_{l+1})
    double S = head;
    bool stop = has;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double vS = __shfl_down(S, off, 64);
        const int vstop = __shfl_down((int)stop, off, 64);
        if (!stop) {
            if (lane + off < 64) {
                S += vS;
                stop = vstop != 0;
            } else {
                stop = true;
            }
        }
    }
    double Snext = __shfl_down(S, 1, 64);
    if (lane == 63) Snext = 0.0;
    if (has) {
        double yin;
        const int row = next_row(seg, yin);
        const double tot = sum + Snext;
        y[row] = kBeta ? __builtin_fma(beta, yin, alpha * tot) : alpha * tot;
    }
    if (lane == 0) carry[t] = (f0 & 1u) ? 0.0 : S;
}

// Staged form: the lanes put their row sums into a per-wave LDS run (slot =
// the row end's index among the tile's row starts), then the wave reads the
// run and y0 and writes y with wave-wide accesses: rows [first_row, first_row
// + starts) are consecutive in a tile without empty rows (one 512-B access
// per 64 rows), and increasing, listed in seg_row, in a tile with empty rows.
// The plain form issues one scattered 8-B store (and load) per row end: a
// 9-entry-row tile ends ~114 rows spread over 16 partially active store
// instructions.  The first 128 rows' y0 are loaded before the x gathers.
// Same products and row sums as csr5_tile, and every form writes
// y = fma(beta, y0, alpha * sum) explicitly (contraction left to the
// compiler differed between forms): bit-identical
// (tests/test_spmv_gpu.py::test_csr5_forms_bit_identical).
template <bool kBeta, bool kNt>
__device__ __forceinline__ void csr5_tile_st(
    long long t, const int *__restrict__ tile_row, const uint32_t *__restrict__ flags,
    const double *__restrict__ tval, const int *__restrict__ tcol,
    const int *__restrict__ seg_off, const int *__restrict__ seg_row,
    const double *__restrict__ x, long long ntiles, long long nnz, double alpha,
    double beta, double *__restrict__ y, double *__restrict__ carry, double *__restrict__ sy)
{
    const int lane = threadIdx.x & 63;
    const double *tv = tval + t * kC5Tile;
    const int *tc = tcol + t * kC5Tile;
    const uint32_t f = flags[t * 64 + lane];
    const int trow = tile_row[t];
    const bool gap = trow < 0;  // bit31: tile contains empty rows (wave-uniform)
    const int r0 = trow & 0x7fffffff;
    v4i cq[kC5Sigma / 4];
    v2d vq[kC5Sigma / 2];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        cq[q] = ld_nt_v4i(tc + q * 256 + 4 * lane);
        vq[2 * q] = ld_nt_v2d(tv + (2 * q) * 128 + 2 * lane);
        vq[2 * q + 1] = ld_nt_v2d(tv + (2 * q + 1) * 128 + 2 * lane);
    }
    const int soff = gap ? seg_off[t] : 0;
    __builtin_amdgcn_sched_barrier(0);
    const int cnt = __popc(f);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const int segbase = incl - cnt;
    const int total = __shfl(incl, 63, 64);  // row starts in the tile = rows it writes
    const uint32_t f0 = __shfl(f, 0, 64);
    const int first_row = (f0 & 1u) ? r0 : r0 + 1;
    // rows of run slots lane and lane + 64
    int ra = 0, rb = 0;
    if (gap) {
        if (lane < total) ra = seg_row[soff + lane];
        if (lane + 64 < total) rb = seg_row[soff + 64 + lane];
    } else {
        ra = first_row + lane;
        rb = first_row + 64 + lane;
    }
    double y0a = 0.0, y0b = 0.0;
    if (kBeta) {
        if (lane < total) y0a = kNt ? __builtin_nontemporal_load(y + ra) : y[ra];
        if (lane + 64 < total) y0b = kNt ? __builtin_nontemporal_load(y + rb) : y[rb];
    }
    double xv[kC5Sigma];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        xv[4 * q + 0] = x[cq[q].x];
        xv[4 * q + 1] = x[cq[q].y];
        xv[4 * q + 2] = x[cq[q].z];
        xv[4 * q + 3] = x[cq[q].w];
    }
    __builtin_amdgcn_sched_barrier(0);
    double p[kC5Sigma];
#pragma unroll
    for (int q = 0; q < kC5Sigma / 4; ++q) {
        p[4 * q + 0] = vq[2 * q].x * xv[4 * q + 0];
        p[4 * q + 1] = vq[2 * q].y * xv[4 * q + 1];
        p[4 * q + 2] = vq[2 * q + 1].x * xv[4 * q + 2];
        p[4 * q + 3] = vq[2 * q + 1].y * xv[4 * q + 3];
    }
    if (t == ntiles - 1) {  // zero the padding past nnz (x[0] may be inf/nan)
        const long long e0 = t * kC5Tile + (long long)lane * kC5Sigma;
#pragma unroll
        for (int k = 0; k < kC5Sigma; ++k)
            if (e0 + k >= nnz) p[k] = 0.0;
    }
    double head = 0.0, sum = 0.0;
    int seg = -1;
#pragma unroll
    for (int k = 0; k < kC5Sigma; ++k) {
        if ((f >> k) & 1u) {
            if (seg < 0) {
                head = sum;
                seg = segbase;
            } else {
                sy[seg] = alpha * sum;
                ++seg;
            }
            sum = 0.0;
        }
        sum += p[k];
    }
    const bool has = seg >= 0;
    if (!has) head = sum;
    double S = head;
    bool stop = has;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double vS = __shfl_down(S, off, 64);
        const int vstop = __shfl_down((int)stop, off, 64);
        if (!stop) {
            if (lane + off < 64) {
                S += vS;
                stop = vstop != 0;
            } else {
                stop = true;
            }
        }
    }
    double Snext = __shfl_down(S, 1, 64);
    if (lane == 63) Snext = 0.0;
    if (has) sy[seg] = alpha * (sum + Snext);
    if (lane == 0) carry[t] = (f0 & 1u) ? 0.0 : S;
    // the wave's LDS writes are done before its reads (LDS keeps one wave's
    // operations in order; the wait makes the data dependence explicit)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int i = lane; i < total; i += 64) {
        const double v = sy[i];
        int row;
        double b;
        if (i < 64) {
            row = ra;
            b = y0a;
        } else if (i < 128) {
            row = rb;
            b = y0b;
        } else {
            row = gap ? seg_row[soff + i] : first_row + i;
            b = kBeta ? y[row] : 0.0;
        }
        if (kNt)
            __builtin_nontemporal_store(kBeta ? __builtin_fma(beta, b, v) : v, y + row);
        else
            y[row] = kBeta ? __builtin_fma(beta, b, v) : v;
    }
}

// The tile form: 2 (default) staged y with non-temporal y accesses; the
// experiment build (Makefile `alt`, -DSBLAS_C5_PF=f) selects 0 plain, 1
// phased loads + prefetched row ends, 3 staged y with plain accesses
#ifndef SBLAS_C5_PF
#define SBLAS_C5_PF 2
#endif
static int c5_form_env() { return std::max(0, std::min(3, SBLAS_C5_PF)); }

template <bool kBeta, int kForm = 2>
__global__ __launch_bounds__(256) void k_spmv_csr5(
    const int *__restrict__ tile_row, const uint32_t *__restrict__ flags,
    const double *__restrict__ tval, const int *__restrict__ tcol,
    const int *__restrict__ seg_off, const int *__restrict__ seg_row,
    const double *__restrict__ x, long long ntiles, long long nnz, double alpha,
    double beta, double *__restrict__ y, double *__restrict__ carry)
{
    const long long t = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (t >= ntiles) return;  // wave-uniform
    if constexpr (kForm >= 2) {
        __shared__ double s_y[4][kC5Tile + 1];  // one tile's row sums per wave
        csr5_tile_st<kBeta, kForm == 2>(t, tile_row, flags, tval, tcol, seg_off, seg_row, x, ntiles, nnz, alpha, beta,
                                        y, carry, s_y[threadIdx.x >> 6]);
    } else if constexpr (kForm == 1) {
        csr5_tile_pf<kBeta>(t, tile_row, flags, tval, tcol, seg_off, seg_row, x, ntiles, nnz, alpha, beta, y, carry);
    } else {
        csr5_tile<kBeta>(t, tile_row, flags, tval, tcol, seg_off, seg_row, x, ntiles, nnz, alpha, beta, y, carry);
    }
}

// CSR5 over XCD-affine column panels: block b runs tiles of panel b % P (the
// hardware deals blocks to the XCDs round robin, so an XCD keeps to the
// panels b % 8 selects: its x gathers stay in ~n*8/P bytes of x), writing
// the panel's alpha-scaled partial y (beta applied by the reduce).
template <int kForm>
__global__ __launch_bounds__(256) void k_spmv_csr5_panel(const Csr5Desc *__restrict__ desc, int P,
                                                         const double *__restrict__ x, double alpha)
{
    const int p = (int)(blockIdx.x % P);
    const long long t = (long long)(blockIdx.x / P) * 4 + (threadIdx.x >> 6);
    const Csr5Desc &d = desc[p];
    if (t >= d.ntiles) return;  // wave-uniform
    if constexpr (kForm >= 2) {
        __shared__ double s_y[4][kC5Tile + 1];  // one tile's row sums per wave
        csr5_tile_st<false, kForm == 2>(t, d.tile_row, d.flags, d.tval, d.tcol, d.seg_off, d.seg_row, x, d.ntiles,
                                        d.nnz, alpha, 0.0, d.y, d.carry, s_y[threadIdx.x >> 6]);
    } else {
        csr5_tile<false>(t, d.tile_row, d.flags, d.tval, d.tcol, d.seg_off, d.seg_row, x, d.ntiles, d.nnz, alpha,
                         0.0, d.y, d.carry);
    }
}

// Head runs, found once at plan build: tile t starts a run when its head
// (the part of a row that started in an earlier tile) is not the
// continuation of the previous tile's head row; head_run[t] = the number of
// consecutive tiles whose heads belong to that row (else 0).
__global__ void k_c5_headruns(const int *__restrict__ tile_row, const uint32_t *__restrict__ flags,
                              long long ntiles, int *__restrict__ head_run)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    auto has_head = [&](long long u) { return (flags[u * 64] & 1u) == 0u; };
    int L = 0;
    const int R = tile_row[t] & 0x7fffffff;
    if (has_head(t) && !(t > 0 && (tile_row[t - 1] & 0x7fffffff) == R && has_head(t - 1)))
        for (long long u = t; u < ntiles && (tile_row[u] & 0x7fffffff) == R && has_head(u); ++u) ++L;
    head_run[t] = L;
}

// Adds each head run's carries (in tile order) to its row: deterministic.
__device__ __forceinline__ void csr5_calibrate(long long t, const int *__restrict__ tile_row,
                                               const int *__restrict__ head_run,
                                               const double *__restrict__ carry, long long ntiles,
                                               double alpha, double *__restrict__ y)
{
    if (t >= ntiles) return;
    const int L = head_run[t];
    if (L == 0) return;
    const int R = tile_row[t] & 0x7fffffff;
    double s = 0.0;
    for (int u = 0; u < L; ++u) s += carry[t + u];
    y[R] += alpha * s;
}

__global__ void k_csr5_calibrate(const int *__restrict__ tile_row, const int *__restrict__ head_run,
                                 const double *__restrict__ carry, long long ntiles, double alpha,
                                 double *__restrict__ y)
{
    csr5_calibrate((long long)blockIdx.x * blockDim.x + threadIdx.x, tile_row, head_run, carry, ntiles, alpha, y);
}

// panel form: blockIdx.y = panel (the partials' empty rows were zeroed once
// at plan build and are never written; d.nempty > 0 would zero them here)
__global__ void k_csr5_calibrate_panel(const Csr5Desc *__restrict__ desc, double alpha)
{
    const Csr5Desc &d = desc[blockIdx.y];
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < d.nempty) d.y[d.empty_rows[i]] = 0.0;
    csr5_calibrate(i, d.tile_row, d.head_run, d.carry, d.ntiles, alpha, d.y);
}

template <bool kBeta>
__global__ void k_empty_rows(const int *__restrict__ rows, int n, double beta,
                             double *__restrict__ y)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = rows[i];
    y[r] = kBeta ? beta * y[r] : 0.0;
}

// ---- CSR5 tile descriptors built on the device ----------------------------
// (the reference builds its descriptors on the GPU too:
// spmv/include/detail/cuda/format_cuda.h:21-300).  Same arrays as the host
// builder below (kept as the "csr5_hostplan" test hook): row-start bits, the row of
// each tile's first element (bit 31: the tile holds empty rows), and for such
// tiles the explicit list of rows starting in the tile.
__global__ void k_c5_flags(const int *__restrict__ rp, int m, uint32_t *__restrict__ flags,
                           int *__restrict__ empty, int *__restrict__ nempty)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int a = rp[r];
    if (a == rp[r + 1]) {
        empty[atomicAdd(nempty, 1)] = r;
        return;
    }
    const long long t = a / kC5Tile;
    const int w = (int)(a - t * kC5Tile);
    atomicOr(&flags[t * 64 + w / kC5Sigma], 1u << (w % kC5Sigma));
}

// last r in [0, m) with rp[r] <= e (e < nnz: that row holds element e)
__device__ __forceinline__ int c5_row_of(const int *__restrict__ rp, int m, long long e)
{
    int lo = 0, hi = m;  // invariant rp[lo] <= e, answer in [lo, hi)
    while (hi - lo > 1) {
        const int mid = lo + (hi - lo) / 2;
        if (rp[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ void k_c5_tiles(const int *__restrict__ rp, int m, long long nnz, long long nt,
                           const uint32_t *__restrict__ flags, int *__restrict__ trow,
                           int *__restrict__ segcnt)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t == nt) trow[nt] = m;
    if (t >= nt) return;
    const long long e = t * kC5Tile;
    const long long elast = (nnz < e + kC5Tile ? nnz : e + kC5Tile) - 1;
    const int rf = c5_row_of(rp, m, e), rl = c5_row_of(rp, m, elast);
    int nstarts = 0;
    for (int l = 0; l < 64; ++l) nstarts += __popc(flags[t * 64 + l]);
    const int start0 = (int)(flags[t * 64] & 1u);
    const bool holes = nstarts != rl - rf + start0;
    trow[t] = holes ? (int)((unsigned)rf | 0x80000000u) : rf;
    segcnt[t] = holes ? nstarts : 0;
}

__global__ void k_c5_segrows(const int *__restrict__ rp, int m, long long nnz, long long nt,
                             const uint32_t *__restrict__ flags, const int *__restrict__ trow,
                             const int *__restrict__ seg_end, int *__restrict__ seg_row)
{
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt || trow[t] >= 0) return;
    const long long e = t * kC5Tile;
    const long long elast = (nnz < e + kC5Tile ? nnz : e + kC5Tile) - 1;
    const int rf = trow[t] & 0x7fffffff, rl = c5_row_of(rp, m, elast);
    int o = t ? seg_end[t - 1] : 0;
    for (int q = (flags[t * 64] & 1u) ? rf : rf + 1; q <= rl; ++q)
        if (rp[q + 1] > rp[q] && rp[q] >= e && rp[q] <= elast) seg_row[o++] = q;
}

static int build_csr5_plan_device(Csr5Plan &P, const int *rowptr, int m, long long nnz, hipStream_t s)
{
    const long long nt = P.ntiles;
    SBLAS_HIP(hipMalloc(&P.tile_row, sizeof(int) * (nt + 1)));
    SBLAS_HIP(hipMalloc(&P.flags, sizeof(uint32_t) * std::max<long long>(nt * 64, 1)));
    SBLAS_HIP(hipMalloc(&P.seg_off, sizeof(int) * (nt + 1)));
    SBLAS_HIP(hipMalloc(&P.empty_rows, sizeof(int) * (std::max(m, 1) + 1)));
    int *nempty = P.empty_rows + std::max(m, 1);  // counter word after the list
    SBLAS_HIP(hipMemsetAsync(P.flags, 0, sizeof(uint32_t) * std::max<long long>(nt * 64, 1), s));
    SBLAS_HIP(hipMemsetAsync(P.seg_off, 0, sizeof(int) * (nt + 1), s));
    SBLAS_HIP(hipMemsetAsync(nempty, 0, sizeof(int), s));
    if (m > 0)
        hipLaunchKernelGGL(k_c5_flags, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, rowptr, m,
                           P.flags, P.empty_rows, nempty);
    // seg_off[0] = 0, seg_off[1..nt] = inclusive scan of the per-tile counts
    hipLaunchKernelGGL(k_c5_tiles, dim3((unsigned)((nt + 1 + 255) / 256)), dim3(256), 0, s, rowptr, m,
                       nnz, nt, P.flags, P.tile_row, P.seg_off + 1);
    SBLAS_HIP(hipGetLastError());
    int *scratch = nullptr;
    SBLAS_HIP(hipMalloc(&scratch, sizeof(int) * (nt / 1024 + 256)));
    const int st = scan_inclusive(P.seg_off + 1, nt, scratch, s);
    int h[2] = {0, 0};
    if (st == SBLAS_OK) {
        SBLAS_HIP(hipMemcpyAsync(&h[0], P.seg_off + nt, sizeof(int), hipMemcpyDeviceToHost, s));
        SBLAS_HIP(hipMemcpyAsync(&h[1], nempty, sizeof(int), hipMemcpyDeviceToHost, s));
        SBLAS_HIP(hipStreamSynchronize(s));
    }
    (void)hipFree(scratch);
    SBLAS_TRY(st);
    P.nempty = h[1];
    SBLAS_HIP(hipMalloc(&P.seg_row, sizeof(int) * std::max(h[0], 1)));
    if (h[0] > 0)
        hipLaunchKernelGGL(k_c5_segrows, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, rowptr, m,
                           nnz, nt, P.flags, P.tile_row, P.seg_off + 1, P.seg_row);
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

template <bool kBeta>
__global__ void k_panel_reduce(const double *__restrict__ ypart, int P, long long m, double beta,
                               double *__restrict__ y);

// the device builder over raw CSR arrays (the whole matrix or one panel)
static int build_csr5_core(Csr5Plan &P, const int *rowptr, const int *col, const double *val, int m,
                           long long nnz, hipStream_t s)
{
    P.ntiles = (nnz + kC5Tile - 1) / kC5Tile;
    SBLAS_TRY(build_csr5_plan_device(P, rowptr, m, nnz, s));
    const long long nt = P.ntiles, total = nt * kC5Tile;
    SBLAS_HIP(hipMalloc(&P.tval, sizeof(double) * std::max<long long>(total, 1)));
    SBLAS_HIP(hipMalloc(&P.tcol, sizeof(int) * std::max<long long>(total, 1)));
    SBLAS_HIP(hipMalloc(&P.carry, sizeof(double) * std::max<long long>(nt, 1)));
    SBLAS_HIP(hipMalloc(&P.head_run, sizeof(int) * std::max<long long>(nt, 1)));
    if (total) {
        hipLaunchKernelGGL(k_c5_transpose, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, col, val, nnz,
                           total, P.tcol, P.tval);
        SBLAS_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_c5_headruns, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, P.tile_row, P.flags, nt,
                           P.head_run);
        SBLAS_HIP(hipGetLastError());
    }
    SBLAS_HIP(hipStreamSynchronize(s));
    P.ready = true;
    return SBLAS_OK;
}

static void free_csr5_arrays(Csr5Plan &P)
{
    (void)hipFree(P.tile_row);
    (void)hipFree(P.flags);
    (void)hipFree(P.tval);
    (void)hipFree(P.tcol);
    (void)hipFree(P.seg_off);
    (void)hipFree(P.seg_row);
    (void)hipFree(P.empty_rows);
    (void)hipFree(P.carry);
    (void)hipFree(P.head_run);
    for (Csr5Plan &Q : P.panels) free_csr5_arrays(Q);
    (void)hipFree(P.desc);
    (void)hipFree(P.ypart);
}

// A's columns cut into P panels of W columns: a panel-local CSR each
// (rowptr [P][m+1]; col / val panel-major from base[p], each panel 16-B
// aligned).  The caller owns (and frees) rowptr / col / val.
struct PanelCsr {
    int P = 0;
    long long W = 0;
    int *rowptr = nullptr;
    int *col = nullptr;
    double *val = nullptr;
    std::vector<int> hrp;         // host copy of rowptr
    std::vector<long long> base;  // panel p's first element in col / val
};

static int split_panels(const sblas_csr_s &A, int P, hipStream_t s, PanelCsr &o);
static void free_panel_csr(PanelCsr &o);
static int default_panels(const sblas_csr_s &A);

// CSR5 over XCD column panels (XCD-affine x gathers): the columns cut into P
// panels of their own (split_panels; not the row-split panel plan, whose
// panel count is the row split's), one tile plan per non-empty panel, the
// panel CSR freed once the tiles are built.  Each panel's empty rows get no
// segment, so their partials are zeroed once here and never written.
static int build_csr5_panels(sblas_csr_s &A, int Preq, hipStream_t s)
{
    Csr5Plan &P = A.c5;
    const long long m = A.m;
    PanelCsr pc;
    int st = split_panels(A, Preq, s, pc);
    std::vector<int> live;
    for (int p = 0; st == SBLAS_OK && p < pc.P; ++p)
        if (pc.hrp[(size_t)p * (m + 1) + m] > 0) live.push_back(p);
    if (st == SBLAS_OK && live.size() < 2) st = SBLAS_ERR_UNSUPPORTED;
    const int PL = (int)live.size();
    if (st == SBLAS_OK) {
        P.panels.assign((size_t)PL, Csr5Plan{});
        if (hipMalloc(&P.ypart, sizeof(double) * std::max<long long>(PL * m, 1)) != hipSuccess ||
            hipMemsetAsync(P.ypart, 0, sizeof(double) * std::max<long long>(PL * m, 1), s) != hipSuccess) {
            set_error("csr5 panels: %s", hipGetErrorString(hipGetLastError()));
            st = SBLAS_ERR_HIP;
        }
    }
    std::vector<Csr5Desc> hd((size_t)std::max(PL, 0));
    for (int q = 0; st == SBLAS_OK && q < PL; ++q) {
        const int p = live[q];
        const int nz = pc.hrp[(size_t)p * (m + 1) + m];
        Csr5Plan &S = P.panels[(size_t)q];
        st = build_csr5_core(S, pc.rowptr + (size_t)p * (m + 1), pc.col + pc.base[p], pc.val + pc.base[p], (int)m, nz,
                             s);
        hd[(size_t)q] = Csr5Desc{S.tile_row, S.flags,    S.tval, S.tcol, S.seg_off, S.seg_row, S.empty_rows,
                                 P.ypart + (size_t)q * m, S.carry, S.ntiles, (long long)nz, 0, 0, S.head_run};
        P.maxtiles = std::max(P.maxtiles, S.ntiles);
    }
    if (st == SBLAS_OK && hipStreamSynchronize(s) != hipSuccess) st = SBLAS_ERR_HIP;
    free_panel_csr(pc);
    if (st != SBLAS_OK) return st;
    SBLAS_HIP(hipMalloc(&P.desc, sizeof(Csr5Desc) * PL));
    SBLAS_HIP(hipMemcpy(P.desc, hd.data(), sizeof(Csr5Desc) * PL, hipMemcpyHostToDevice));
    P.P = PL;
    P.ready = true;
    return SBLAS_OK;
}

int build_csr5_plan(sblas_csr_s &A, hipStream_t s)
{
    if (A.c5.ready) return SBLAS_OK;
    DeviceGuard g(A.device);
    Csr5Plan &P = A.c5;
    P.form = c5_form_env();
    // test hook "csr5_hostplan": the host-built descriptors (the device
    // builder's cross-check, tests/test_spmv_gpu.py)
    double hv = 0.0;
    const bool hostplan = test_option("csr5_hostplan", &hv) && hv != 0.0;
    // Tiles per XCD column panel (each XCD's gathers in a slice of x) when x
    // outgrows an XCD's L2, the rows' columns are scattered (the probe: most
    // sampled rows span > n/4 of the columns, spread over the eighths) and
    // the matrix is large enough to amortise the panels' partial-y pass.
    // P = default_panels (4 on config 2) whatever the row length: on the
    // uniform config 2 4 panels beat 2 and 8 on short rows (N = 8 light rank
    // 60 vs 68 / 67 us) and are within 4-8% of 8 on 96-entry rows
    // (profiles/r05/c5P/).  Test hooks "csr5_panel" (1 / 0 forces either
    // form) and "panels" (the count).  From 32M entries the panels halve to
    // ~2 MiB of x (P = 8, one per XCD): the x re-fetch the panel's entry
    // stream forces through a 4 MiB L2 grows with the entries, the partial
    // y (16 B per row and panel) with the rows -- config 2 at N = 1 (39.75M
    // entries, 2M rows): 284.6-285.1 us at P = 4, 273.7-274.6 at P = 8
    // (profiles/r06/panels/); the N = 8 light slice keeps P = 4.
    int npanels = default_panels(A);
    double popt = 0.0;
    if (A.nnz >= kC5WidePanelNnz && !test_option("panels", &popt)) npanels = std::min(8, 2 * npanels);
    bool panels = false;
    SBLAS_TRY(xcd_panels_pay(A, s, "csr5_panel", kPanelMinNnz, &panels));
    if (panels && npanels >= 2 && !hostplan) {
        const int rc = build_csr5_panels(A, npanels, s);
        if (rc == SBLAS_OK) return SBLAS_OK;
        free_csr5_arrays(P);
        A.c5 = Csr5Plan{};
        if (rc != SBLAS_ERR_UNSUPPORTED) return rc;
    }
    if (!hostplan) return build_csr5_core(P, A.rowptr, A.col, A.val, A.m, A.nnz, s);
    const long long nnz = A.nnz;
    const std::vector<int> &rp = A.h_rowptr;
    P.ntiles = (nnz + kC5Tile - 1) / kC5Tile;
    const long long nt = P.ntiles;
    std::vector<uint32_t> flags((size_t)nt * 64, 0u);
    std::vector<int> empty;
    for (int r = 0; r < A.m; ++r) {
        const int a = rp[r], b = rp[r + 1];
        if (a == b) {
            empty.push_back(r);
            continue;
        }
        const long long t = a / kC5Tile;
        const int w = (int)(a - t * kC5Tile);
        flags[(size_t)t * 64 + w / kC5Sigma] |= 1u << (w % kC5Sigma);
    }
    // tile_row: row holding the tile's first element (last r with rp[r] <= e)
    std::vector<int> trow((size_t)nt + 1, A.m);
    std::vector<int> seg_off((size_t)nt + 1, 0);
    std::vector<int> seg_row;
    int r = 0;
    for (long long t = 0; t < nt; ++t) {
        const long long e = t * kC5Tile;
        while (r < A.m && rp[r + 1] <= e) ++r;
        const int rfirst = r;
        // last row of tile
        const long long elast = std::min(nnz, e + kC5Tile) - 1;
        int rl = r;
        while (rl < A.m && rp[rl + 1] <= elast) ++rl;
        int nstarts = 0;
        for (int l = 0; l < 64; ++l) nstarts += __builtin_popcount(flags[(size_t)t * 64 + l]);
        const bool start0 = flags[(size_t)t * 64] & 1u;
        const int expected = rl - rfirst + (start0 ? 1 : 0);
        trow[t] = rfirst;
        seg_off[t] = (int)seg_row.size();
        if (nstarts != expected) {
            trow[t] = rfirst | (int)0x80000000u;
            for (int q = (start0 ? rfirst : rfirst + 1); q <= rl; ++q)
                if (rp[q + 1] > rp[q] && rp[q] >= e && rp[q] <= elast) seg_row.push_back(q);
        }
    }
    seg_off[nt] = (int)seg_row.size();
    P.nempty = (int)empty.size();

    SBLAS_HIP(hipMalloc(&P.tile_row, sizeof(int) * (nt + 1)));
    SBLAS_HIP(hipMalloc(&P.flags, sizeof(uint32_t) * std::max<long long>(nt * 64, 1)));
    SBLAS_HIP(hipMalloc(&P.tval, sizeof(double) * std::max<long long>(nt * kC5Tile, 1)));
    SBLAS_HIP(hipMalloc(&P.tcol, sizeof(int) * std::max<long long>(nt * kC5Tile, 1)));
    SBLAS_HIP(hipMalloc(&P.seg_off, sizeof(int) * (nt + 1)));
    SBLAS_HIP(hipMalloc(&P.seg_row, sizeof(int) * std::max<size_t>(seg_row.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.empty_rows, sizeof(int) * std::max<size_t>(empty.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.carry, sizeof(double) * std::max<long long>(nt, 1)));
    SBLAS_HIP(hipMalloc(&P.head_run, sizeof(int) * std::max<long long>(nt, 1)));
    SBLAS_HIP(hipMemcpyAsync(P.tile_row, trow.data(), sizeof(int) * (nt + 1), hipMemcpyHostToDevice, s));
    if (nt) SBLAS_HIP(hipMemcpyAsync(P.flags, flags.data(), sizeof(uint32_t) * nt * 64, hipMemcpyHostToDevice, s));
    SBLAS_HIP(hipMemcpyAsync(P.seg_off, seg_off.data(), sizeof(int) * (nt + 1), hipMemcpyHostToDevice, s));
    if (!seg_row.empty())
        SBLAS_HIP(hipMemcpyAsync(P.seg_row, seg_row.data(), sizeof(int) * seg_row.size(), hipMemcpyHostToDevice, s));
    if (!empty.empty())
        SBLAS_HIP(hipMemcpyAsync(P.empty_rows, empty.data(), sizeof(int) * empty.size(), hipMemcpyHostToDevice, s));
    const long long total = nt * kC5Tile;
    if (total) {
        hipLaunchKernelGGL(k_c5_transpose, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                           A.col, A.val, nnz, total, P.tcol, P.tval);
        SBLAS_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_c5_headruns, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, P.tile_row, P.flags, nt,
                           P.head_run);
        SBLAS_HIP(hipGetLastError());
    }
    SBLAS_HIP(hipStreamSynchronize(s));
    P.ready = true;
    return SBLAS_OK;
}

int launch_spmv_csr5(const sblas_csr_s &A, double alpha, const double *x,
                     double beta, double *y, hipStream_t s)
{
    const Csr5Plan &P = A.c5;
    if (!P.ready) return SBLAS_ERR_INVALID;
    if (P.P > 0) {  // XCD-affine panels
        if (A.m == 0) return SBLAS_OK;
        const long long grid = (P.maxtiles + 3) / 4 * P.P;
        if (grid > 0)
            SBLAS_LAUNCH((P.form == 2   ? k_spmv_csr5_panel<2>
                          : P.form == 3 ? k_spmv_csr5_panel<3>
                                        : k_spmv_csr5_panel<0>),
                         dim3((unsigned)grid), dim3(256), 0, s, P.desc, P.P, x, alpha);
        const long long mc = P.maxtiles;
        if (mc > 0)
            SBLAS_LAUNCH(k_csr5_calibrate_panel, dim3((unsigned)((mc + 255) / 256), (unsigned)P.P), dim3(256), 0, s,
                         P.desc, alpha);
        const unsigned rb = (unsigned)((A.m + 255) / 256);
        if (beta != 0.0)
            SBLAS_LAUNCH(k_panel_reduce<true>, dim3(rb), dim3(256), 0, s, P.ypart, P.P, (long long)A.m, beta, y);
        else
            SBLAS_LAUNCH(k_panel_reduce<false>, dim3(rb), dim3(256), 0, s, P.ypart, P.P, (long long)A.m, beta, y);
        SBLAS_HIP(hipGetLastError());
        return SBLAS_OK;
    }
    if (P.ntiles) {
        const unsigned nb = (unsigned)((P.ntiles + 3) / 4);
        const int form = P.form;
        if (beta != 0.0)
            SBLAS_LAUNCH((form == 2   ? k_spmv_csr5<true, 2>
                          : form == 3 ? k_spmv_csr5<true, 3>
                          : form == 1 ? k_spmv_csr5<true, 1>
                                      : k_spmv_csr5<true, 0>),
                         dim3(nb), dim3(256), 0, s, P.tile_row, P.flags, P.tval, P.tcol, P.seg_off, P.seg_row, x,
                         P.ntiles, A.nnz, alpha, beta, y, P.carry);
        else
            SBLAS_LAUNCH((form == 2   ? k_spmv_csr5<false, 2>
                          : form == 3 ? k_spmv_csr5<false, 3>
                          : form == 1 ? k_spmv_csr5<false, 1>
                                      : k_spmv_csr5<false, 0>),
                         dim3(nb), dim3(256), 0, s, P.tile_row, P.flags, P.tval, P.tcol, P.seg_off, P.seg_row, x,
                         P.ntiles, A.nnz, alpha, beta, y, P.carry);
        SBLAS_LAUNCH(k_csr5_calibrate, dim3((unsigned)((P.ntiles + 255) / 256)), dim3(256),
                           0, s, P.tile_row, P.head_run, P.carry, P.ntiles, alpha, y);
    }
    if (P.nempty) {
        if (beta != 0.0)
            SBLAS_LAUNCH(k_empty_rows<true>, dim3((P.nempty + 255) / 256), dim3(256), 0, s,
                               P.empty_rows, P.nempty, beta, y);
        else
            SBLAS_LAUNCH(k_empty_rows<false>, dim3((P.nempty + 255) / 256), dim3(256), 0, s,
                               P.empty_rows, P.nempty, beta, y);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}


// ---------------------------------------------------------------------------
// XCD-affine column panels (algo 4)
// ---------------------------------------------------------------------------
// Config 2's columns are uniform over n: with one launch over all of A every
// XCD gathers from all of x (16 MB, 4x its 4 MB L2) and ~55% of gathers miss
// to the Infinity Cache at 64-B line granularity.  Splitting A into P = 8
// column panels and dealing panel p's row blocks to workgroups with
// blockIdx % 8 == p keeps each XCD on one ~2 MB slice of x (round-robin
// dispatch; a different placement is only slower, never wrong).
template <bool kSc1>
__global__ __launch_bounds__(kRsThreads) void k_spmv_panel(const PanelDesc *__restrict__ desc,
                                                           int P, const double *__restrict__ x,
                                                           double alpha)
{
    __shared__ double prod[kRsBlockNnz + 8];
    __shared__ double wsum[kRsThreads / 64];
    const int p = blockIdx.x % P;
    const int lb = blockIdx.x / P;
    const PanelDesc d = desc[p];
    if (lb >= d.nblocks) return;
    rowsplit_block<false, kSc1>(d.blocks[lb], d.rowptr, d.col, d.val, x, alpha, 0.0, d.out,
                                d.partial, prod, wsum);
}

__global__ void k_panel_long_finalize(const int4 *__restrict__ long_rows, int nlong,
                                      const double *__restrict__ partial, double alpha,
                                      double *__restrict__ ypart, long long m)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlong) return;
    const int4 L = long_rows[i];
    double s = 0.0;
    for (int q = 0; q < L.z; ++q) s += partial[L.y + q];
    ypart[(long long)L.w * m + L.x] = alpha * s;
}

template <bool kBeta>
__global__ void k_panel_reduce(const double *__restrict__ ypart, int P, long long m, double beta,
                               double *__restrict__ y)
{
    const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    double s = 0.0;
    for (int p = 0; p < P; ++p) s += __builtin_nontemporal_load(ypart + (long long)p * m + r);
    y[r] = kBeta ? s + beta * y[r] : s;
}

// thread per row: counts of the row's entries per panel -> rowptr[p][r+1]
// Rows of >= kPanelLongRow entries are split by a wave each (the _long
// kernels below): one thread walking a power-law hub row of 62k entries P
// times made the split of an R-MAT graph take 73 ms.
constexpr int kPanelLongRow = 256;

__global__ void k_panel_count(const int *__restrict__ rowptr, const int *__restrict__ col, int m,
                              long long W, int P, int lmin, int *__restrict__ prp)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    if (rowptr[r + 1] - rowptr[r] >= lmin) return;  // k_panel_count_long
    for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) {
        const int p = (int)(col[j] / W);
        prp[(long long)p * (m + 1) + r + 1]++;
    }
}

// thread per row: stable scatter of the row's entries into the panels
__global__ void k_panel_scatter(const int *__restrict__ rowptr, const int *__restrict__ col,
                                const double *__restrict__ val, int m, long long W, int P, int lmin,
                                const int *__restrict__ prp, const long long *__restrict__ base,
                                int *__restrict__ pcol, double *__restrict__ pval)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const int a = rowptr[r], b = rowptr[r + 1];
    if (b - a >= lmin) return;  // k_panel_scatter_long
    for (int p = 0; p < P; ++p) {
        long long o = base[p] + prp[(long long)p * (m + 1) + r];
        for (int j = a; j < b; ++j) {
            const int c = col[j];
            if ((int)(c / W) == p) {
                pcol[o] = c;
                pval[o] = val[j];
                ++o;
            }
        }
    }
}

// a wave per long row (rows[i]): per 64 entries, one ballot per panel counts
// (and, in the scatter, ranks) the entries of that panel: the same stable
// order as the thread-per-row kernels
__global__ __launch_bounds__(256) void k_panel_count_long(const int *__restrict__ rowptr,
                                                          const int *__restrict__ col, int m, long long W,
                                                          int P, const int *__restrict__ rows, int nrows,
                                                          int *__restrict__ prp)
{
    const int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= nrows) return;  // wave-uniform
    const int r = rows[w];
    const int a = rowptr[r], b = rowptr[r + 1];
    for (int p = 0; p < P; ++p) {
        int cnt = 0;
        for (int j0 = a; j0 < b; j0 += 64) {
            const int j = j0 + lane;
            const bool in = j < b && (int)(col[j] / W) == p;
            cnt += __popcll(__ballot(in));
        }
        if (lane == 0) prp[(long long)p * (m + 1) + r + 1] = cnt;
    }
}

__global__ __launch_bounds__(256) void k_panel_scatter_long(const int *__restrict__ rowptr,
                                                            const int *__restrict__ col,
                                                            const double *__restrict__ val, int m, long long W,
                                                            int P, const int *__restrict__ rows, int nrows,
                                                            const int *__restrict__ prp,
                                                            const long long *__restrict__ base,
                                                            int *__restrict__ pcol, double *__restrict__ pval)
{
    const int w = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= nrows) return;  // wave-uniform
    const int r = rows[w];
    const int a = rowptr[r], b = rowptr[r + 1];
    const unsigned long long below = (1ULL << lane) - 1ULL;
    for (int p = 0; p < P; ++p) {
        long long o = base[p] + prp[(long long)p * (m + 1) + r];
        for (int j0 = a; j0 < b; j0 += 64) {
            const int j = j0 + lane;
            const int c = j < b ? col[j] : 0;
            const bool in = j < b && (int)(c / W) == p;
            const unsigned long long mask = __ballot(in);
            if (in) {
                const long long d = o + __popcll(mask & below);
                pcol[d] = c;
                pval[d] = val[j];
            }
            o += __popcll(mask);
        }
    }
}

static int split_panels(const sblas_csr_s &A, int P, hipStream_t s, PanelCsr &o)
{
    o.P = P;
    o.W = ((long long)A.n + P - 1) / P;
    const long long m = A.m;
    SBLAS_HIP(hipMalloc(&o.rowptr, sizeof(int) * P * (m + 1)));
    SBLAS_HIP(hipMemsetAsync(o.rowptr, 0, sizeof(int) * P * (m + 1), s));
    const long long cap = ((A.nnz + 3) & ~3LL) + 4 * P + 4;
    SBLAS_HIP(hipMalloc(&o.col, sizeof(int) * cap));
    SBLAS_HIP(hipMalloc(&o.val, sizeof(double) * cap));
    SBLAS_HIP(hipMemsetAsync(o.col, 0, sizeof(int) * cap, s));
    SBLAS_HIP(hipMemsetAsync(o.val, 0, sizeof(double) * cap, s));
    // rows split by a wave each (host rowptr: A.h_rowptr)
    std::vector<int> hlong;
    const bool have_h = (long long)A.h_rowptr.size() > m;
    const int lmin = have_h ? kPanelLongRow : INT_MAX;  // no host copy: every row thread-per-row
    for (long long r = 0; have_h && r < m; ++r)
        if (A.h_rowptr[r + 1] - A.h_rowptr[r] >= lmin) hlong.push_back((int)r);
    int *dlong = nullptr;
    const int nlong = (int)hlong.size();
    if (nlong) {
        SBLAS_HIP(hipMalloc(&dlong, sizeof(int) * nlong));
        SBLAS_HIP(hipMemcpy(dlong, hlong.data(), sizeof(int) * nlong, hipMemcpyHostToDevice));
    }
    if (m > 0) {
        hipLaunchKernelGGL(k_panel_count, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s,
                           A.rowptr, A.col, (int)m, o.W, P, lmin, o.rowptr);
        if (nlong)
            hipLaunchKernelGGL(k_panel_count_long, dim3((unsigned)((nlong + 3) / 4)), dim3(256), 0, s, A.rowptr,
                               A.col, (int)m, o.W, P, dlong, nlong, o.rowptr);
        int *scratch = nullptr;
        SBLAS_HIP(hipMalloc(&scratch, sizeof(int) * ((m + 1) / 1024 + 256)));
        for (int p = 0; p < P; ++p) SBLAS_TRY(scan_inclusive(o.rowptr + p * (m + 1), m + 1, scratch, s));
        SBLAS_HIP(hipStreamSynchronize(s));
        (void)hipFree(scratch);
    }
    o.hrp.assign((size_t)P * (m + 1), 0);
    SBLAS_HIP(hipMemcpy(o.hrp.data(), o.rowptr, sizeof(int) * o.hrp.size(), hipMemcpyDeviceToHost));
    o.base.assign(P, 0);
    long long acc = 0;
    for (int p = 0; p < P; ++p) {
        o.base[p] = acc;
        acc += o.hrp[(size_t)p * (m + 1) + m];
        acc = (acc + 3) & ~3LL;
    }
    long long *dbase = nullptr;
    SBLAS_HIP(hipMalloc(&dbase, sizeof(long long) * P));
    SBLAS_HIP(hipMemcpy(dbase, o.base.data(), sizeof(long long) * P, hipMemcpyHostToDevice));
    if (m > 0)
        hipLaunchKernelGGL(k_panel_scatter, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s,
                           A.rowptr, A.col, A.val, (int)m, o.W, P, lmin, o.rowptr, dbase, o.col, o.val);
    if (m > 0 && nlong)
        hipLaunchKernelGGL(k_panel_scatter_long, dim3((unsigned)((nlong + 3) / 4)), dim3(256), 0, s, A.rowptr,
                           A.col, A.val, (int)m, o.W, P, dlong, nlong, o.rowptr, dbase, o.col, o.val);
    SBLAS_HIP(hipStreamSynchronize(s));
    (void)hipFree(dbase);
    (void)hipFree(dlong);
    return SBLAS_OK;
}

static void free_panel_csr(PanelCsr &o)
{
    (void)hipFree(o.rowptr);
    (void)hipFree(o.col);
    (void)hipFree(o.val);
    o.rowptr = nullptr;
    o.col = nullptr;
    o.val = nullptr;
}

// ~4 MiB of x per panel (one XCD's L2), at most one panel per XCD (config 2:
// P = 4 beats 8, fewer partial-y bytes); the test hook "panels" overrides
static int default_panels(const sblas_csr_s &A)
{
    int P = (int)std::min<long long>(8, std::max<long long>(1, ((long long)A.n * 8 + (4 << 20) - 1) >> 22));
    double v = 0.0;
    if (test_option("panels", &v)) P = std::max(1, std::min(64, (int)v));
    if (A.n < P) P = std::max(1, A.n);
    return P;
}

int build_panel_plan(sblas_csr_s &A, hipStream_t s)
{
    if (A.pn.ready) return SBLAS_OK;
    DeviceGuard g(A.device);
    PanelPlan &Q = A.pn;
    const int P = default_panels(A);
    const long long m = A.m;
    PanelCsr pc;
    {
        const int st = split_panels(A, P, s, pc);
        if (st != SBLAS_OK) {
            free_panel_csr(pc);
            return st;
        }
    }
    Q.P = P;
    Q.W = pc.W;
    Q.rowptr = pc.rowptr;
    Q.col = pc.col;
    Q.val = pc.val;
    SBLAS_HIP(hipMalloc(&Q.ypart, sizeof(double) * std::max<long long>(P * m, 1)));
    const std::vector<int> &hrp = pc.hrp;
    const std::vector<long long> &base = pc.base;
    // Only non-empty panels take part.  One non-empty panel (all columns in
    // one x slice, e.g. the prefix layout) is plain row split: use it.
    std::vector<int> live;
    for (int p = 0; p < P; ++p)
        if (hrp[(size_t)p * (m + 1) + m] > 0) live.push_back(p);
    if (live.size() <= 1) {
        (void)hipFree(Q.rowptr);
        (void)hipFree(Q.col);
        (void)hipFree(Q.val);
        (void)hipFree(Q.ypart);
        Q.rowptr = nullptr;
        Q.col = nullptr;
        Q.val = nullptr;
        Q.ypart = nullptr;
        Q.P = 1;
        Q.degenerate = true;
        SBLAS_TRY(build_rowsplit_plan(A, s));
        Q.ready = true;
        return SBLAS_OK;
    }
    const int PL = (int)live.size();
    // per-panel row blocks, padded to a common count for the interleaved grid
    std::vector<std::vector<RowBlock>> pb(PL);
    std::vector<int4> longs;
    int nslots = 0;
    for (int q = 0; q < PL; ++q) {
        std::vector<int4> pl;
        make_row_blocks(hrp.data() + (size_t)live[q] * (m + 1), (int)m, pb[q], pl, nslots);
        for (auto &L : pl) longs.push_back(make_int4(L.x, L.y, L.z, q));
        Q.maxblocks = std::max<int>(Q.maxblocks, (int)pb[q].size());
    }
    std::vector<RowBlock> all((size_t)PL * Q.maxblocks, RowBlock{0, 0, 0, 0});
    for (int q = 0; q < PL; ++q)
        std::copy(pb[q].begin(), pb[q].end(), all.begin() + (size_t)q * Q.maxblocks);
    SBLAS_HIP(hipMalloc(&Q.blocks, sizeof(RowBlock) * std::max<size_t>(all.size(), 1)));
    if (!all.empty())
        SBLAS_HIP(hipMemcpy(Q.blocks, all.data(), sizeof(RowBlock) * all.size(), hipMemcpyHostToDevice));
    Q.nlong = (int)longs.size();
    SBLAS_HIP(hipMalloc(&Q.partial, sizeof(double) * std::max(nslots, 1)));
    if (Q.nlong) {
        SBLAS_HIP(hipMalloc(&Q.long_rows, sizeof(int4) * longs.size()));
        SBLAS_HIP(hipMemcpy(Q.long_rows, longs.data(), sizeof(int4) * longs.size(), hipMemcpyHostToDevice));
    }
    std::vector<PanelDesc> hd(PL);
    for (int q = 0; q < PL; ++q) {
        const int p = live[q];
        hd[q].rowptr = Q.rowptr + (size_t)p * (m + 1);
        hd[q].col = Q.col + base[p];
        hd[q].val = Q.val + base[p];
        hd[q].blocks = Q.blocks + (size_t)q * Q.maxblocks;
        hd[q].out = Q.ypart + (size_t)q * m;
        hd[q].partial = Q.partial;
        hd[q].nblocks = (int)pb[q].size();
        hd[q].pad = 0;
    }
    Q.P = PL;
    SBLAS_HIP(hipMalloc(&Q.desc, sizeof(PanelDesc) * PL));
    SBLAS_HIP(hipMemcpy(Q.desc, hd.data(), sizeof(PanelDesc) * PL, hipMemcpyHostToDevice));
    Q.ready = true;
    return SBLAS_OK;
}

int launch_spmv_panel(const sblas_csr_s &A, double alpha, const double *x, double beta,
                      double *y, hipStream_t s)
{
    const PanelPlan &Q = A.pn;
    if (!Q.ready) return SBLAS_ERR_INVALID;
    if (Q.degenerate) return launch_spmv_rowsplit(A, alpha, x, beta, y, s);
    if (A.m == 0) return SBLAS_OK;
    const long long grid = (long long)Q.maxblocks * Q.P;
    // agent-scope stores of the partials: experiment builds only (Makefile
    // `alt`, -DSBLAS_PANEL_SC1=1)
#ifndef SBLAS_PANEL_SC1
#define SBLAS_PANEL_SC1 0
#endif
    constexpr bool sc1 = SBLAS_PANEL_SC1 != 0;
    if (grid > 0) {
        if (sc1)
            SBLAS_LAUNCH(k_spmv_panel<true>, dim3((unsigned)grid), dim3(kRsThreads), 0, s,
                               Q.desc, Q.P, x, alpha);
        else
            SBLAS_LAUNCH(k_spmv_panel<false>, dim3((unsigned)grid), dim3(kRsThreads), 0, s,
                               Q.desc, Q.P, x, alpha);
    }
    if (Q.nlong)
        SBLAS_LAUNCH(k_panel_long_finalize, dim3((Q.nlong + 63) / 64), dim3(64), 0, s,
                           Q.long_rows, Q.nlong, Q.partial, alpha, Q.ypart, (long long)A.m);
    const unsigned rb = (unsigned)((A.m + 255) / 256);
    if (beta != 0.0)
        SBLAS_LAUNCH(k_panel_reduce<true>, dim3(rb), dim3(256), 0, s, Q.ypart, Q.P,
                           (long long)A.m, beta, y);
    else
        SBLAS_LAUNCH(k_panel_reduce<false>, dim3(rb), dim3(256), 0, s, Q.ypart, Q.P,
                           (long long)A.m, beta, y);
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

void free_plans(sblas_csr_s &A)
{
    DeviceGuard g(A.device);
    (void)hipFree(A.rs.blocks);
    (void)hipFree(A.rs.long_rows);
    (void)hipFree(A.rs.partial);
    A.rs = RsPlan{};
    free_csr5_arrays(A.c5);
    A.c5 = Csr5Plan{};
    PanelPlan &Q = A.pn;
    (void)hipFree(Q.rowptr);
    (void)hipFree(Q.col);
    (void)hipFree(Q.val);
    (void)hipFree(Q.blocks);
    (void)hipFree(Q.desc);
    (void)hipFree(Q.ypart);
    (void)hipFree(Q.partial);
    (void)hipFree(Q.long_rows);
    A.pn = PanelPlan{};
    free_xsort_plan(A);
    free_spmm_plan(A);
}

}  // namespace sblas
