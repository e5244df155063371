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
//  * columns are cut into G = 8q groups of <= 2^18 columns; XCD k serves groups
//    [kq, (k+1)q) (x slice <= 2 MiB, L2-resident);
//  * inside a block (row range x group) the entries are sorted by column, and
//    lanes read consecutive entries, so the lanes of one gather instruction
//    land on few x lines (the TA merges them) -- measured 2x on the gather.
// Row sums then arrive in column order, so they accumulate into per-row LDS
// slots with ds_add_f64.  The summation ORDER within a row therefore depends
// on wave timing: results are within the fp64 error bound of the sequential
// row sum (tests) but not bitwise reproducible from run to run, unlike the
// row-split/CSR5/panel kernels.
//
// Work items: a narrow range (few nonzeros) is one item -- one workgroup walks
// all G groups, starting at its XCD's first group, and writes y; a wide range
// is G items, one per group, each writing a partial for its rows, which a
// reduce pass adds in group order.  Items sit in one queue per XCD; a
// persistent grid claims from its own XCD's queue (XCC_ID hardware register)
// and steals from the others when it runs dry.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <utility>
#include <vector>

#include "sblas_internal.hpp"

namespace sblas {

constexpr int kXsThreads = 1024;  // default workgroup (SBLAS_XS_THREADS=512 for experiments)
constexpr int kXsRows = 16384;     // LDS row accumulators per workgroup (128 KiB)
constexpr int kXsRowBits = 14;     // packed key: local row in the low 14 bits
constexpr int kXsColBits = 18;     //             group-local column above
constexpr int kXsUnroll = 8;       // entries per lane in flight
static_assert(kXsRowBits + kXsColBits == 32, "packed key is 32 bits");
static_assert(kXsRows <= (1 << kXsRowBits), "local row must fit the key");

// XCC_ID hardware register (gfx940+: HW_REG_XCC_ID = 20, bits [3:0]).
__device__ __forceinline__ int xs_xcc_id()
{
    return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7;
}

__device__ __forceinline__ int xs_claim(const XsArgs &a, int xcc)
{
    for (int k = 0; k < 8; ++k) {
        const int qq = (xcc + k) & 7;
        if (__hip_atomic_load(&a.qhead[qq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= a.qlen[qq])
            continue;
        const int idx = atomicAdd(&a.qhead[qq], 1);
        if (idx < a.qlen[qq]) return a.qitems[qq * a.qstride + idx];
    }
    return -1;
}

// One work item's entries [s0, s1): consecutive column-group blocks whose
// offsets are bnd[0..ng] (bnd[0] = s0, bnd[ng] = s1) for groups gb, gb+1, ...
// (a wide item is one block, a narrow item all G blocks of its range, walked
// as ONE stream so the pipeline never drains between groups).  Lanes read
// consecutive entries; each lane tracks the group of its (increasing)
// entries and turns it into the x offset of the group.
// Software pipeline with ping-pong registers and an even, workgroup-uniform
// trip count (no mid-loop exit, so nothing can be sunk below the adds):
//   gathers(A) | loads(B) | adds(A) | gathers(B) | loads(A') | adds(B)
// sched_barrier pins that issue order; waiting for the gathers (vmcnt counts
// in order) then leaves the next batch's key/value loads in flight.  Lanes
// past s1 load the last entry (one line per wave) and add an exact +0.0
// (a select, not a product: the clamped x may be inf/nan).
// kMode (timing experiments only, SBLAS_XS_MODE): 0 = the product kernel,
// bit 0 = plain LDS stores instead of ds_add_f64, bit 1 = gathers read x[0].
template <int kMode, int NT>
__device__ __forceinline__ void xs_stream(const uint32_t *__restrict__ key,
                                          const double *__restrict__ val, long long s0,
                                          long long s1, const long long *bnd, int gb, int Wg,
                                          const double *__restrict__ x, double *acc)
{
    if (s1 <= s0) return;  // workgroup-uniform
    constexpr int U = kXsUnroll;
    constexpr long long S = (long long)U * NT;
    int gi = 0;              // lane's current group (relative to gb)
    long long nb = bnd[1];   // its end
    auto load = [&](long long eb, uint32_t *kk, double *vv, int *xo) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long eu = eb + (long long)u * NT;
            const long long ei = eu < s1 ? eu : s1 - 1;
            kk[u] = __builtin_nontemporal_load(key + ei);
            vv[u] = __builtin_nontemporal_load(val + ei);
            while (ei >= nb) nb = bnd[++gi + 1];
            xo[u] = (gb + gi) * Wg;
        }
    };
    auto gather = [&](const uint32_t *kk, const int *xo, double *xx) {
#pragma unroll
        for (int u = 0; u < U; ++u) xx[u] = x[(kMode & 2) ? 0 : xo[u] + (int)(kk[u] >> kXsRowBits)];
    };
    auto accumulate = [&](long long eb, const uint32_t *kk, const double *vv, const double *xx) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double p = eb + (long long)u * NT < s1 ? vv[u] * xx[u] : 0.0;
            if (kMode & 1) acc[kk[u] & ((1u << kXsRowBits) - 1)] = p;
            else atomicAdd(&acc[kk[u] & ((1u << kXsRowBits) - 1)], p);
        }
    };
    uint32_t ka[U], kb[U];
    double va[U], vb[U], xa[U], xb[U];
    int oa[U], ob[U];
    const long long nit = (s1 - s0 + S - 1) / S;
    long long e = s0 + threadIdx.x;
    load(e, ka, va, oa);
    for (long long it = 0; it < nit; it += 2) {
        gather(ka, oa, xa);
        __builtin_amdgcn_sched_barrier(0);
        load(e + S, kb, vb, ob);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(e, ka, va, xa);
        __builtin_amdgcn_sched_barrier(0);
        gather(kb, ob, xb);
        __builtin_amdgcn_sched_barrier(0);
        load(e + 2 * S, ka, va, oa);
        __builtin_amdgcn_sched_barrier(0);
        accumulate(e + S, kb, vb, xb);
        e += 2 * S;
    }
}

template <bool kBeta, int kMode, int NT>
__global__ __launch_bounds__(NT) void k_spmv_xsort(const XsArgs a, const double *__restrict__ x,
                                                   double alpha, double beta,
                                                   double *__restrict__ y)
{
    __shared__ double acc[kXsRows];
    __shared__ long long s_bnd[256];
    __shared__ int s_item;
    const int xcc = a.use_xcc ? xs_xcc_id() : (int)(blockIdx.x & 7);
    if (threadIdx.x == 0) s_item = xs_claim(a, xcc);
    for (;;) {
        __syncthreads();
        const int item = s_item;
        if (item < 0) return;  // workgroup-uniform
        // item = range << 8 | slot: slot k+1 = wide item of XCD k (its q
        // groups [kq, kq+q), partial slot k); slot 0 = narrow item (all G
        // groups, starting at this XCD's first group and wrapping)
        const int ri = item >> 8, k1 = item & 255;
        const XsRange R = a.ranges[ri];
        const long long *bo = a.blk + (long long)ri * a.G;
        const int g0 = k1 ? (k1 - 1) * a.q : xcc * a.q;
        const int ng = k1 ? a.q : a.G;
        for (int r = threadIdx.x; r < R.nrows; r += NT) acc[r] = 0.0;
        // s_bnd[j] = start of group (g0 + j) % G in a wrapped walk: segment 1
        // is groups [g0, G) (bounds s_bnd[0..G-g0]), segment 2 groups [0, g0)
        const int n1 = k1 ? ng : a.G - g0;
        for (int j = threadIdx.x; j <= n1; j += NT) s_bnd[j] = bo[g0 + j];
        if (!k1)
            for (int j = threadIdx.x; j <= g0; j += NT) s_bnd[128 + j] = bo[j];
        __syncthreads();
        // claim the next item now; its result is consumed after the stream,
        // so the atomic's latency hides behind the stream's own loads
        int pre = 0;
        long long t0 = 0;
        if (threadIdx.x == 0) {
            pre = atomicAdd(&a.qhead[xcc], 1);
            if (a.trace) t0 = (long long)__builtin_amdgcn_s_memrealtime();
        }
        xs_stream<kMode, NT>(a.key, a.val, s_bnd[0], s_bnd[n1], s_bnd, g0, a.Wg, x, acc);
        if (!k1 && g0 > 0)
            xs_stream<kMode, NT>(a.key, a.val, s_bnd[128], s_bnd[128 + g0], s_bnd + 128, 0, a.Wg, x,
                                 acc);
        if (threadIdx.x == 0) {
            if (a.trace) {  // debugging aid (SBLAS_XS_TRACE): per-item timeline
                const long long t1 = (long long)__builtin_amdgcn_s_memrealtime();
                const long long slot = 1 + 4LL * atomicAdd((unsigned long long *)a.trace, 1ULL);
                a.trace[slot] = item;
                const long long cnt = k1 ? s_bnd[n1] - s_bnd[0] : bo[a.G] - bo[0];
                a.trace[slot + 1] = (cnt << 20) | ((long long)blockIdx.x << 4) | xcc;
                a.trace[slot + 2] = t0;
                a.trace[slot + 3] = t1;
            }
            s_item = pre < a.qlen[xcc] ? a.qitems[xcc * a.qstride + pre] : xs_claim(a, xcc);
        }
        __syncthreads();
        if (k1) {
            double *out = a.partial + R.pbase + (long long)(k1 - 1) * R.nrows;
            for (int r = threadIdx.x; r < R.nrows; r += NT) out[r] = acc[r];
        } else {
            double *yr = y + R.row0;
            for (int r = threadIdx.x; r < R.nrows; r += NT)
                yr[r] = kBeta ? alpha * acc[r] + beta * yr[r] : alpha * acc[r];
        }
        // (the barrier at the loop top orders these reads of acc before the
        // next item's zeroing)
    }
}

// Wide ranges: y = alpha * sum_k partial[k] (+ beta*y), XCD slots in order.
template <bool kBeta>
__global__ __launch_bounds__(256) void k_xsort_reduce(const XsRange *__restrict__ ranges,
                                                      const int *__restrict__ wide, int G,
                                                      const double *__restrict__ partial,
                                                      double alpha, double beta,
                                                      double *__restrict__ y)
{
    const XsRange R = ranges[wide[blockIdx.y]];
    for (int r = blockIdx.x * 256 + threadIdx.x; r < R.nrows; r += gridDim.x * 256) {
        const double *p = partial + R.pbase + r;
        double s = 0.0;
        for (int g = 0; g < G; ++g) s += p[(long long)g * R.nrows];
        double *yr = y + R.row0 + r;
        *yr = kBeta ? alpha * s + beta * *yr : alpha * s;
    }
}

void free_xsort_plan(sblas_csr_s &A)
{
    XsPlan &P = A.xs;
    (void)hipFree(P.ranges);
    (void)hipFree(P.wide);
    (void)hipFree(P.blk);
    (void)hipFree(P.key);
    (void)hipFree(P.val);
    (void)hipFree(P.qitems);
    (void)hipFree(P.qhead);
    (void)hipFree(P.partial);
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

    // column groups: G = 8q groups of Wg <= 2^18 columns and ~1 MiB of x
    // (an XCD's current group plus the A stream must fit its 4 MiB L2)
    const long long ng = ((long long)std::max(n, 1) + (1LL << kXsColBits) - 1) >> kXsColBits;
    const long long nmib = ((long long)std::max(n, 1) * 8 + (1LL << 20) - 1) >> 20;
    P.q = (int)std::max<long long>({1LL, (ng + 7) / 8, (nmib + 7) / 8});
    if (const char *e = getenv("SBLAS_XS_Q"))  // experiments: override, >= the 2^18 bound
        P.q = (int)std::max<long long>({1LL, (ng + 7) / 8, (long long)atoi(e)});
    P.G = 8 * P.q;
    if (P.G > 127) {
        set_error("xsort: n = %d needs %d column groups (> 127)", n, P.G);
        return SBLAS_ERR_UNSUPPORTED;
    }
    P.Wg = (int)std::max<long long>(1, ((long long)std::max(n, 1) + P.G - 1) / P.G);
    const int G = P.G, Wg = P.Wg;

    // resident workgroups -> work per item
    int dev = 0, ncu = 0, per_cu = 0;
    SBLAS_HIP(hipGetDevice(&dev));
    SBLAS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    P.nt = getenv("SBLAS_XS_THREADS") && atoi(getenv("SBLAS_XS_THREADS")) == 512 ? 512 : kXsThreads;
    if (P.nt == 512)
        SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spmv_xsort<true, 0, 512>, 512, 0));
    else
        SBLAS_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spmv_xsort<true, 0, kXsThreads>,
                                                                kXsThreads, 0));
    const int resident = std::max(1, ncu * std::max(per_cu, 1));
    // about kper items per resident workgroup (claimed dynamically)
    int kper = 1;
    if (const char *e = getenv("SBLAS_XS_K")) kper = std::max(1, atoi(e));
    long long wstar = std::max<long long>(1, (nnz + (long long)resident * kper - 1) / ((long long)resident * kper));
    if (const char *e = getenv("SBLAS_XS_WSTAR")) wstar = std::max(1LL, atoll(e));
    const bool all_wide = getenv("SBLAS_XS_ALLWIDE") && atoi(getenv("SBLAS_XS_ALLWIDE")) != 0;
    const bool nosort = getenv("SBLAS_XS_NOSORT") && atoi(getenv("SBLAS_XS_NOSORT")) != 0;
    int rows_cap = kXsRows;
    if (const char *e = getenv("SBLAS_XS_ROWS")) rows_cap = std::max(1, std::min(kXsRows, atoi(e)));

    // Row ranges: a candidate range takes <= rows_cap rows while one of its
    // 8 wide items costs <= cap; it becomes wide or is re-cut into narrow
    // ranges of cost <= cap (below).
    std::vector<XsRange> ranges;
    // Cost model (work units ~ one streamed entry): an item's time is its
    // entries plus lambda per distinct x line its gathers touch; with
    // uniform columns a block of c entries over L lines touches
    // L*(1 - exp(-c/L)) lines.  A narrow item spreads its entries over all of
    // x (G*Lg lines), a wide item's 1/8 share over its XCD's q groups.
    // lambda = 1.7 was fitted on config 2's item timeline (SBLAS_XS_TRACE:
    // narrow items ran at 0.58x the entries/us of wide ones).
    double lam = 1.7;
    if (const char *e = getenv("SBLAS_XS_LAMBDA")) lam = atof(e);
    const double Lg = std::max(1.0, Wg / 16.0);  // 128-B lines of one group's x slice
    auto narrow_cost = [&](double c) { return c + lam * G * Lg * (1.0 - std::exp(-c / (G * Lg))); };
    auto wide_cost = [&](double c) {
        const double ci = c / 8.0;
        return ci + lam * P.q * Lg * (1.0 - std::exp(-ci / (P.q * Lg)));
    };
    auto build_ranges = [&](double cap) {
        ranges.clear();
        // extend [r, ...) while cost(entries) <= cap and rows <= rows_cap
        auto cut = [&](int r, int rend, bool wide, long long &cnt) {
            const int start = r;
            cnt = 0;
            while (r < rend && r - start < rows_cap) {
                const long long len = rp[r + 1] - rp[r];
                const double c = (double)(cnt + len);
                if (r > start && (wide ? wide_cost(c) : narrow_cost(c)) > cap) break;
                cnt += len;
                ++r;
            }
            return r;
        };
        int r = 0;
        while (r < m) {
            long long cnt;
            const int e = cut(r, m, true, cnt);
            // WIDE (8 items, one per XCD, + 8 partials per row) when it holds
            // more than one narrow item's work and its rows average >= 16
            // entries (the partials then cost <= 8 B per entry)
            const bool wide = cnt > 0 && (all_wide || (narrow_cost((double)cnt) > cap &&
                                                       cnt >= 16LL * (e - r)));
            if (wide) {
                XsRange R{};
                R.row0 = r;
                R.nrows = e - r;
                R.wide = 1;
                ranges.push_back(R);
            } else {
                for (int q0 = r; q0 < e;) {
                    long long c2;
                    const int q1 = cut(q0, e, false, c2);
                    XsRange R{};
                    R.row0 = q0;
                    R.nrows = q1 - q0;
                    R.wide = 0;
                    ranges.push_back(R);
                    q0 = q1;
                }
            }
            r = e;
        }
    };
    auto count_items = [&]() {
        long long c = 0;
        for (const XsRange &R : ranges) c += R.wide ? 8 : 1;
        return c;
    };
    // grow the item cost until the items fit the resident grid (a second
    // round for a few items would double the kernel's tail)
    const long long slots = (long long)resident * kper;
    double cap = (double)wstar;
    if (!getenv("SBLAS_XS_WSTAR")) cap = narrow_cost((double)nnz) / (double)slots;
    for (int it = 0; it < 200; ++it) {
        build_ranges(cap);
        if (count_items() <= slots || getenv("SBLAS_XS_WSTAR")) break;
        cap *= 1.02;
    }
    const int I = (int)ranges.size();
    if ((long long)I >= (1LL << 23)) {
        set_error("xsort: %d row ranges (> 2^23)", I);
        return SBLAS_ERR_UNSUPPORTED;
    }

    // host copies of the CSR entries
    std::vector<int> hcol((size_t)nnz);
    std::vector<double> hval((size_t)nnz);
    if (nnz) {
        SBLAS_HIP(hipMemcpy(hcol.data(), A.col, sizeof(int) * nnz, hipMemcpyDeviceToHost));
        SBLAS_HIP(hipMemcpy(hval.data(), A.val, sizeof(double) * nnz, hipMemcpyDeviceToHost));
    }

    // pass 1: entries per (range, group)
    std::vector<long long> blk((size_t)I * G + 1, 0);
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < I; ++i) {
        long long *c = blk.data() + (size_t)i * G + 1;
        for (int e = rp[ranges[i].row0]; e < rp[ranges[i].row0 + ranges[i].nrows]; ++e)
            ++c[hcol[e] / Wg];
    }
    for (size_t k = 1; k < blk.size(); ++k) blk[k] += blk[k - 1];

    // pass 2: fill each block and sort it by (column, row)
    std::vector<uint32_t> hkey((size_t)nnz);
    std::vector<double> hv((size_t)nnz);
    bool bad = false;
#pragma omp parallel
    {
        std::vector<long long> pos(G);
        std::vector<std::pair<uint32_t, double>> tmp;
#pragma omp for schedule(dynamic, 16) reduction(|| : bad)
        for (int i = 0; i < I; ++i) {
            const XsRange &R = ranges[i];
            for (int g = 0; g < G; ++g) pos[g] = blk[(size_t)i * G + g];
            for (int r = R.row0; r < R.row0 + R.nrows; ++r) {
                for (int e = rp[r]; e < rp[r + 1]; ++e) {
                    const int c = hcol[e];
                    const int g = c / Wg;
                    const uint32_t cp = (uint32_t)(c - g * Wg), lr = (uint32_t)(r - R.row0);
                    if (c < 0 || c >= n || cp >= (1u << kXsColBits) || lr >= (uint32_t)kXsRows) bad = true;
                    const long long o = pos[g]++;
                    hkey[o] = (cp << kXsRowBits) | lr;
                    hv[o] = hval[e];
                }
            }
            for (int g = 0; g < G; ++g) {
                const long long b0 = blk[(size_t)i * G + g], b1 = blk[(size_t)i * G + g + 1];
                tmp.resize((size_t)(b1 - b0));
                for (long long o = b0; o < b1; ++o) tmp[o - b0] = {hkey[o], hv[o]};
                if (!nosort) std::stable_sort(tmp.begin(), tmp.end(),
                                 [](const std::pair<uint32_t, double> &a,
                                    const std::pair<uint32_t, double> &b) { return a.first < b.first; });
                for (long long o = b0; o < b1; ++o) {
                    hkey[o] = tmp[o - b0].first;
                    hv[o] = tmp[o - b0].second;
                }
            }
        }
    }
    if (bad) {
        set_error("xsort: column index out of [0, n) or key overflow");
        return SBLAS_ERR_INVALID;
    }

    // items, wide partial slots, XCD queues
    std::vector<int> wide;
    std::vector<std::vector<int>> q(8);
    long long pbase = 0;
    int nnarrow = 0;
    for (int i = 0; i < I; ++i) {
        XsRange &R = ranges[i];
        if (R.wide) {
            R.pbase = pbase;
            pbase += 8LL * R.nrows;
            wide.push_back(i);
            for (int k = 0; k < 8; ++k) q[k].push_back((i << 8) | (k + 1));
        } else {
            q[nnarrow++ % 8].push_back(i << 8);
        }
    }
    P.nranges = I;
    P.nwide = (int)wide.size();
    P.qstride = 1;
    P.nitems = 0;
    for (int k = 0; k < 8; ++k) {
        P.qlen[k] = (int)q[k].size();
        P.qstride = std::max(P.qstride, P.qlen[k]);
        P.nitems += P.qlen[k];
    }
    P.grid = std::min(P.nitems, resident);
    std::vector<int> qflat((size_t)8 * P.qstride, -1);
    for (int k = 0; k < 8; ++k) std::copy(q[k].begin(), q[k].end(), qflat.begin() + (size_t)k * P.qstride);

    SBLAS_HIP(hipMalloc(&P.ranges, sizeof(XsRange) * std::max(I, 1)));
    SBLAS_HIP(hipMalloc(&P.wide, sizeof(int) * std::max<size_t>(wide.size(), 1)));
    SBLAS_HIP(hipMalloc(&P.blk, sizeof(long long) * blk.size()));
    SBLAS_HIP(hipMalloc(&P.key, sizeof(uint32_t) * std::max<long long>(nnz, 1)));
    SBLAS_HIP(hipMalloc(&P.val, sizeof(double) * std::max<long long>(nnz, 1)));
    SBLAS_HIP(hipMalloc(&P.qitems, sizeof(int) * qflat.size()));
    SBLAS_HIP(hipMalloc(&P.qhead, sizeof(int) * 8));
    SBLAS_HIP(hipMalloc(&P.partial, sizeof(double) * std::max<long long>(pbase, 1)));
    if (I) SBLAS_HIP(hipMemcpy(P.ranges, ranges.data(), sizeof(XsRange) * I, hipMemcpyHostToDevice));
    if (!wide.empty())
        SBLAS_HIP(hipMemcpy(P.wide, wide.data(), sizeof(int) * wide.size(), hipMemcpyHostToDevice));
    SBLAS_HIP(hipMemcpy(P.blk, blk.data(), sizeof(long long) * blk.size(), hipMemcpyHostToDevice));
    if (nnz) {
        SBLAS_HIP(hipMemcpy(P.key, hkey.data(), sizeof(uint32_t) * nnz, hipMemcpyHostToDevice));
        SBLAS_HIP(hipMemcpy(P.val, hv.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
    }
    SBLAS_HIP(hipMemcpy(P.qitems, qflat.data(), sizeof(int) * qflat.size(), hipMemcpyHostToDevice));
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
    XsArgs a{};
    a.ranges = P.ranges;
    a.blk = P.blk;
    a.key = P.key;
    a.val = P.val;
    a.qitems = P.qitems;
    a.qhead = P.qhead;
    a.partial = P.partial;
    for (int k = 0; k < 8; ++k) a.qlen[k] = P.qlen[k];
    a.qstride = P.qstride;
    a.G = P.G;
    a.q = P.q;
    a.Wg = P.Wg;
    a.use_xcc = use_xcc;
    static const int mode = [] {
        const char *e = getenv("SBLAS_XS_MODE");
        return e ? atoi(e) : 0;
    }();
    SBLAS_HIP(hipMemsetAsync(P.qhead, 0, sizeof(int) * 8, s));
    using K = void (*)(const XsArgs, const double *, double, double, double *);
    K kern;
    if (P.nt == 512)
        kern = beta != 0.0 ? k_spmv_xsort<true, 0, 512> : k_spmv_xsort<false, 0, 512>;
    else if (mode == 1)
        kern = beta != 0.0 ? k_spmv_xsort<true, 1, kXsThreads> : k_spmv_xsort<false, 1, kXsThreads>;
    else if (mode == 2)
        kern = beta != 0.0 ? k_spmv_xsort<true, 2, kXsThreads> : k_spmv_xsort<false, 2, kXsThreads>;
    else if (mode == 3)
        kern = beta != 0.0 ? k_spmv_xsort<true, 3, kXsThreads> : k_spmv_xsort<false, 3, kXsThreads>;
    else
        kern = beta != 0.0 ? k_spmv_xsort<true, 0, kXsThreads> : k_spmv_xsort<false, 0, kXsThreads>;
    static const char *trace_path = getenv("SBLAS_XS_TRACE");
    std::vector<long long> htrace;
    if (trace_path) {
        const size_t len = 1 + 4 * (size_t)P.nitems;
        SBLAS_HIP(hipMalloc(&a.trace, sizeof(long long) * len));
        SBLAS_HIP(hipMemsetAsync(a.trace, 0, sizeof(long long) * len, s));
        htrace.resize(len);
    }
    hipLaunchKernelGGL(kern, dim3(P.grid), dim3(P.nt), 0, s, a, x, alpha, beta, y);
    if (trace_path) {  // debugging aid: append {item, block<<8|xcc, t0, t1} rows
        SBLAS_HIP(hipMemcpyAsync(htrace.data(), a.trace, sizeof(long long) * htrace.size(),
                                 hipMemcpyDeviceToHost, s));
        SBLAS_HIP(hipStreamSynchronize(s));
        (void)hipFree(a.trace);
        if (FILE *f = fopen(trace_path, "a")) {
            fprintf(f, "# launch items=%d grid=%d\n", P.nitems, P.grid);
            for (long long i = 0; i < htrace[0]; ++i)
                fprintf(f, "%lld %lld %lld %lld\n", htrace[1 + 4 * i], htrace[2 + 4 * i],
                        htrace[3 + 4 * i], htrace[4 + 4 * i]);
            fclose(f);
        }
    }
    if (P.nwide) {
        const dim3 grid((kXsRows + 255) / 256, (unsigned)P.nwide);
        if (beta != 0.0)
            hipLaunchKernelGGL(k_xsort_reduce<true>, grid, dim3(256), 0, s, P.ranges, P.wide, 8,
                               P.partial, alpha, beta, y);
        else
            hipLaunchKernelGGL(k_xsort_reduce<false>, grid, dim3(256), 0, s, P.ranges, P.wide, 8,
                               P.partial, alpha, beta, y);
    }
    SBLAS_HIP(hipGetLastError());
    return SBLAS_OK;
}

}  // namespace sblas
