// sblas_internal.hpp -- shared internals of libsblas (HIP host + kernels).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/sblas.h"

namespace sblas {

void set_error(const char *fmt, ...);

// Kernel-span timing of one library call (sblas_spmv_timed): while `stop` is
// set, SBLAS_LAUNCH launches through hipExtLaunchKernelGGL so the runtime
// stamps `start` as the call's FIRST kernel begins and `stop` as each kernel
// ends (the last one wins): the call's device span without the dispatch and
// event-record gaps that stream events around the call include.
struct LaunchTimer {
    hipEvent_t start = nullptr, stop = nullptr;
    bool pending_start = false;
};
LaunchTimer &launch_timer();
#define SBLAS_LAUNCH(kern, grid, block, shmem, stream, ...)                                        \
    do {                                                                                          \
        ::sblas::LaunchTimer &lt_ = ::sblas::launch_timer();                                      \
        if (lt_.stop) {                                                                           \
            hipExtLaunchKernelGGL(kern, grid, block, shmem, stream,                              \
                                  lt_.pending_start ? lt_.start : nullptr, lt_.stop, 0, __VA_ARGS__); \
            lt_.pending_start = false;                                                            \
        } else {                                                                                  \
            hipLaunchKernelGGL(kern, grid, block, shmem, stream, __VA_ARGS__);                    \
        }                                                                                         \
    } while (0)

#define SBLAS_HIP(expr)                                                        \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            ::sblas::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,    \
                               hipGetErrorString(e_));                         \
            return SBLAS_ERR_HIP;                                              \
        }                                                                      \
    } while (0)

#define SBLAS_TRY(expr)                                                        \
    do {                                                                       \
        int s_ = (expr);                                                       \
        if (s_ != SBLAS_OK) return s_;                                         \
    } while (0)

// Row-split (CSR-adaptive) tuning. One 256-thread workgroup per row block.
constexpr int kRsThreads = 256;
#ifndef SBLAS_RS_BLOCK_NNZ  // experiment builds only (Makefile `alt`)
#define SBLAS_RS_BLOCK_NNZ 2048
#endif
constexpr int kRsBlockNnz = SBLAS_RS_BLOCK_NNZ;  // LDS product stream capacity (16 KiB f64)
constexpr int kRsMaxRows = 1024;    // rows per stream block
constexpr int kRsLongChunk = 8192;  // nnz per workgroup for long rows

// Row block descriptor (16 B): stream block when a > row (a = end row);
// long-row chunk when a < 0 (chunk k = -a-1, b = partial slot or -1).
struct RowBlock {
    int row;
    int a;
    int b;
    int c;
};

// CSR5-style tiles: 64 lanes x kC5Sigma nnz per tile (one wave per tile).
constexpr int kC5Lanes = 64;
constexpr int kC5Sigma = 16;
constexpr int kC5Tile = kC5Lanes * kC5Sigma;

struct Csr5Plan {
    long long ntiles = 0;
    int *tile_row = nullptr;       // [ntiles+1] row of tile's first element; bit31: tile has empty rows
    uint32_t *flags = nullptr;     // [ntiles*64] per-lane row-start bits (bit k: element k starts a row)
    double *tval = nullptr;        // [ntiles*kC5Tile] tile-transposed values
    int *tcol = nullptr;           // [ntiles*kC5Tile] tile-transposed columns
    int *seg_off = nullptr;        // [ntiles+1] offset into seg_row for tiles with empty rows
    int *seg_row = nullptr;        // explicit row of each row start for flagged tiles
    int *empty_rows = nullptr;     // rows with no entries (y = beta*y)
    int nempty = 0;
    double *carry = nullptr;       // [ntiles] tile head partial sums
    int *head_run = nullptr;       // [ntiles] > 0: tile t starts a run of that many tiles whose heads
                                   // continue one row (calibrated together), else 0
    bool ready = false;
    int form = 2;                  // tile form (spmv.hip c5_form_env; alternatives in experiment builds)
    // XCD-affine form (spmv.hip "CSR5 over column panels"): one tile plan per
    // column panel of the panel plan, panel p's tiles dealt to the XCDs with
    // blockIdx % P == p, alpha-scaled partial y per panel, then a reduce.
    int P = 0;                     // 0: plain CSR5 (this plan's own tiles)
    std::vector<Csr5Plan> panels;  // host-side sub-plans (device arrays each)
    struct Csr5Desc *desc = nullptr;  // device [P]
    long long maxtiles = 0;
    double *ypart = nullptr;       // [P][m]
};

// Device-side view of one CSR5 tile plan (the panel form's per-panel plans).
struct Csr5Desc {
    const int *tile_row;
    const uint32_t *flags;
    const double *tval;
    const int *tcol;
    const int *seg_off;
    const int *seg_row;
    const int *empty_rows;
    double *y;        // this panel's partial y
    double *carry;
    long long ntiles;
    long long nnz;
    int nempty;  // empty rows zeroed per call (0: the partial's empty rows stay zero from the plan build)
    int pad;
    const int *head_run;
};

// XCD-panel plan: A split into P column panels (x panel ~2 MiB), each a CSR
// with its own rowptr; one launch interleaves the panels' row blocks so that
// blockIdx % P selects the panel (P = 8 = #XCDs: each XCD's L2 then serves
// one x panel).  Panels write alpha-scaled partial y; a reduce adds them.
struct PanelDesc {
    const int *rowptr;
    const int *col;
    const double *val;
    const RowBlock *blocks;
    double *out;      // ypart + p*m
    double *partial;  // long-row chunk partials
    int nblocks;
    int pad;
};

struct PanelPlan {
    int P = 0;
    long long W = 0;
    int maxblocks = 0;
    int *rowptr = nullptr;      // [P][m+1] panel-local
    int *col = nullptr;         // panel-major, padded
    double *val = nullptr;
    RowBlock *blocks = nullptr; // [P][maxblocks]
    PanelDesc *desc = nullptr;  // device [P]
    double *ypart = nullptr;    // [P][m]
    double *partial = nullptr;  // long-row slots, all panels
    int4 *long_rows = nullptr;  // {row, slot, nchunks, panel}
    int nlong = 0;
    bool degenerate = false;    // <= 1 non-empty panel: plain row split
    bool ready = false;
};

// SpMM plan: 16-row blocks whose column union is dense enough run on MFMA
// (v_mfma_f64_16x16x4f64 over a dense 16 x |U| A tile); other rows take the
// row-wave FMA kernel.
struct SpmmPlan {
    int nmfma = 0;             // MFMA blocks
    int *mblock = nullptr;     // [nmfma] 16-row block index
    int *mchunk = nullptr;     // [nmfma+1] offsets in 4-column chunks
    int *ucol = nullptr;       // [4*chunks] union columns (padded)
    double *atile = nullptr;   // [chunks*64] A fragments, lane-major
    int nsparse = 0;           // rows handled by the row-wave kernel
    long long sparse_nnz = 0;  // their nonzeros
    int *srows = nullptr;
    // Column-sorted C-tile form (few rows, tall B; spmm.hip build_spmm_plan):
    // columns of A cut into slabs of 2^ct_wlog columns, slab s owned by XCD
    // s % 8 and its slabs split into ct_ns contiguous sets; rows into ct_nrb
    // blocks of ct_R.  Entries of (XCD, set, row block) sorted by (column,
    // row) with packed keys (XCD-local column << ct_rbits | local row).  A
    // workgroup accumulates one (row block x 16 C columns) tile in LDS and
    // writes it to its (XCD, set) partial; a reduce adds the partials.
    int ct_ns = 0, ct_nrb = 0, ct_R = 0, ct_rbits = 0, ct_wlog = 0;
    bool ct_direct = false;              // keys hold the global column
    bool ct_slots = false;               // units are column-run slots of <= 2 entries
    unsigned *ct_key2 = nullptr;         // slots: second entry's local row, ~0 if none
    double *ct_val2 = nullptr;
    unsigned *ct_key = nullptr;
    double *ct_val = nullptr;
    long long *ct_off = nullptr;         // [8*ns*nrb + 1] entry offsets
    double fill_thresh = 0.08;  // MFMA tile when a 16-row block fills >= 8% of its column union
    bool ready = false;
};

// Column-sorted XCD-group plan (algo 5, xsort.hip).  Columns are cut into
// G = 8q groups of Wg <= 2^18 columns (XCD k serves groups [kq, (k+1)q)), rows
// into ranges of <= kXsRows rows.  Block (range i, group g) holds the range's
// entries of group g sorted by (column, row) as packed keys
// (col - g*Wg) << 14 | (row - row0) plus values, padded to whole 256-entry
// chunks stored lane-transposed, so the lanes of one gather instruction share
// x lines.  A narrow range is one sub-item (walks all groups, XCD-staggered,
// and writes y); a wide range is 8 sub-items, one per XCD, each writing an
// alpha-free partial that a reduce pass adds in XCD order.  A work item pairs
// two sub-items (one per half of the workgroup).
struct XsRange {
    int row0;
    int nrows;
    int wide;
    int widx;         // wide: index among the wide ranges, else -1
    long long pbase;  // wide: offset of the range's [8][nrows] partials
};

struct XsArgs {
    const uint32_t *key;
    const double *val;
    const long long *xrec;  // per (slot, team): sub, row0|nrows<<32, pbase, widx, G+1 block offsets
    int *qhead;             // [8] claim heads of this launch (start past the static items)
    int *qreset;            // the other parity's heads, re-armed to qstat by block 0
    int qstat[8];           // items per queue taken statically (block b: queue b%8, index b/8)
    int dynamic;            // items beyond the static share exist (claims needed)
    double *partial;
    int qlen[8];
    int qstride;
    int G, q, Wg;
    int kstride, vstride;   // chunk strides in 16-B units (keys, values)
};

struct XsPlan {
    int G = 0, q = 0, Wg = 0;
    int nranges = 0, nwide = 0, nitems = 0, grid = 0;
    XsRange *wranges = nullptr;  // [nwide] the wide ranges' records (k_xsort_reduce)
    uint32_t *key = nullptr;     // owns the chunk storage (keys and values, interleaved per chunk)
    double *val = nullptr;       // values inside it
    int kstride = 64, vstride = 128;
    long long *xrec = nullptr;   // item records (see XsArgs)
    int *qhead = nullptr;        // [2][16]: claim heads per launch parity
    mutable int parity = 0;      // flips every launch (stream-ordered launches)
    double *partial = nullptr;
    int qlen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int qstat[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int dynamic = 0;
    int qstride = 0;
    long long nchunks = 0;       // 256-entry chunks (blocks padded to whole chunks)
    bool solo = false;           // narrow ranges are items of their own (16,384 LDS rows)
    int maxc = 0;                // most chunks of one item (both sub-items)
    bool ready = false;
};

struct RsPlan {
    int nblocks = 0;
    RowBlock *blocks = nullptr;
    int nlong = 0;                 // multi-chunk long rows
    int4 *long_rows = nullptr;     // {row, first_slot, nchunks, 0}
    double *partial = nullptr;     // [nslots]
    int nslots = 0;
    bool ready = false;
    bool panels = false;           // run as the panel plan (XCD column panels, spmv.hip xcd_panels_pay)
    bool seq = true;               // consecutive entries per thread (experiment build SBLAS_RS_SEQ=0: vec4 order)
};

}  // namespace sblas

namespace sblas {
// SBLAS_DETERMINISTIC=1 (read once): new handles default to repeatable
// (bitwise) SpMV results (sblas_csr_set_deterministic).
bool deterministic_default();
}  // namespace sblas

struct sblas_csr_s {
    int device = 0;
    int m = 0, n = 0;
    long long nnz = 0;
    int *rowptr = nullptr;   // [m+1] int32 local
    int *col = nullptr;      // [nnz + pad]
    double *val = nullptr;   // [nnz + pad]
    sblas::RsPlan rs;
    sblas::Csr5Plan c5;
    sblas::PanelPlan pn;
    sblas::SpmmPlan mm;
    sblas::XsPlan xs;
    std::vector<int> h_rowptr;  // host copy (analysis)
    // SpMM per-call scratch, owned by the handle so that distinct handles
    // never share it (row-major copy of a column-major B; C-tile partials).
    // Grown on demand; one SpMM per handle in flight (as for sblas_spmv).
    mutable double *spmm_bt = nullptr;
    mutable size_t spmm_bt_bytes = 0;
    mutable double *spmm_part = nullptr;
    mutable size_t spmm_part_bytes = 0;
    long long plan_bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // device bytes per algorithm's plan
    int auto_algo = 0;          // SBLAS_SPMV_AUTO's choice (capi.hip pick_algo), 0 = not yet
    bool deterministic = sblas::deterministic_default();  // bitwise-repeatable launches (xsort's ordered form)
    double col_adjacency = -1;  // its locality probe
    double col_maxshare = -1;   // its largest eighth-of-the-columns share of the sampled entries
    double col_scattered = -1;  // share of sampled rows whose columns span > n/4
};

namespace sblas {

// Kernel launchers (defined in the .hip files).
int launch_spmv_rowsplit(const sblas_csr_s &A, double alpha, const double *x,
                         double beta, double *y, hipStream_t s);
int build_rowsplit_plan(sblas_csr_s &A, hipStream_t s);
int launch_spmv_csr5(const sblas_csr_s &A, double alpha, const double *x,
                     double beta, double *y, hipStream_t s);
int build_csr5_plan(sblas_csr_s &A, hipStream_t s);
// the column-locality probe (capi.hip): fills col_adjacency / col_maxshare once
int probe_columns(sblas_csr_s &A, hipStream_t s);
void free_plans(sblas_csr_s &A);

int launch_spmv_panel(const sblas_csr_s &A, double alpha, const double *x,
                      double beta, double *y, hipStream_t s);
int build_panel_plan(sblas_csr_s &A, hipStream_t s);
int scan_inclusive(int *a, long long len, int *scratch, hipStream_t s);

int launch_spmv_xsort(const sblas_csr_s &A, double alpha, const double *x,
                      double beta, double *y, hipStream_t s);
int build_xsort_plan(sblas_csr_s &A, hipStream_t s);
void free_xsort_plan(sblas_csr_s &A);

int build_spmm_plan(sblas_csr_s &A, int ncols, hipStream_t s);  // C width of the first call
void free_spmm_plan(sblas_csr_s &A);
int launch_spmm(const sblas_csr_s &A, int n, double alpha, const double *B,
                int ldb, int b_layout, double beta, double *C, int ldc,
                hipStream_t s);
int launch_transpose(const sblas_csr_s &A, int *colptr, int *rowidx,
                     double *cval, hipStream_t s, int *colidx = nullptr);
void make_row_blocks(const int *rp, int m, std::vector<RowBlock> &blocks,
                     std::vector<int4> &longs, int &nslots);
int launch_rowsplit_raw(const int *rowptr, const int *col, const double *val, const double *x,
                        const RowBlock *blocks, int nblocks, const int4 *long_rows, int nlong,
                        double *partial, double alpha, double beta, double *y, hipStream_t s);

// Scoped device switch.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Process-wide peer access (ctx.hip).  Peer access is per process, so every
// user (the loopback all-reduce of a context, a trsv_mgpu handle) takes a
// reference on the (a -> b) link: the first acquire enables it (a link
// already enabled by someone outside the library is used and never
// disabled), the last release disables what the library enabled.  acquire
// returns SBLAS_ERR_UNSUPPORTED when the pair has no peer path (or the test
// hook sblas_test_deny_peer_access is set), SBLAS_ERR_HIP when enabling fails.
int peer_acquire(int a, int b, const char *who);
void peer_release(int a, int b);
bool peer_denied();  // the test hook's state

// Test hooks (capi.hip): a planner override set by sblas_test_set_option;
// false when unset.  Names: "xs_cap", "xs_allwide", "xs_solo" (xsort
// planner), "spmm_ctile", "spmm_mfma_fill" (SpMM plan form), "rs_panel",
// "csr5_panel", "panels" (XCD-panel forms).
bool test_option(const char *name, double *value);

// Host helpers shared by capi / refapi (host_utils.cpp).
int row_of_index(int m, const long long *rowptr, long long idx);
int resolve_device(int ordinal, int *phys);  // wraps ordinals on few GPUs
sblas_ctx bound_ctx();                       // ctx.hip: sblas_ctx_bind's context (or null)

}  // namespace sblas
