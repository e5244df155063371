// sptrsv.hip -- sync-free sparse triangular solve for gfx950.
//
// Replaces sptrsv_syncfree_cuda_analyser / _executor
// (sptrsv/sptrsv_v1/src/sptrsv_syncfree_cuda.h:10-167).
//
// Forward progress on CDNA: there is no independent thread scheduling and
// dispatch order is not a contract, so a wave must never wait on work that
// has not been handed to a running wave.  Both executors therefore take
// their columns/rows from a monotone ticket (one device-scope atomicAdd):
// everything a waiting wave depends on was ticketed earlier, by a wave that
// is already resident, and the earliest unfinished item can always proceed.
// Every spin is bounded (timeout word -> SBLAS_ERR_HIP instead of a hang).
//
// Cross-workgroup visibility (MI355X: per-XCD L2s, per-CU L1):
//   * push (algo 0, the reference's CSC scatter): left_sum updates are
//     device-scope fp64 atomic adds (performed at the memory side), then
//     `s_waitcnt vmcnt(0)`, then the in-degree counters are bumped; the
//     consumer polls its counter with an sc1 (L1-bypassing) load and reads
//     left_sum with an sc1 load -- no L2 write-back fence per column.
//   * pull (algo 1, CSR): x itself is the ready flag -- x is pre-filled with
//     a signalling-NaN pattern no arithmetic can produce, x_i is published by
//     one 8-byte sc1 store and consumed by one sc1 load.  No float atomics:
//     sums are deterministic.  One LANE per row; lanes never block inside an
//     iteration, so rows that depend on rows of the same wave resolve across
//     iterations.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include <hip/hip_runtime.h>

#include "sblas_internal.hpp"

struct sblas_trsv_s {
    int device = 0;
    int n = 0, nnz = 0;
    int substitution = 0;
    // CSC (input layout; push executor)
    int *colptr = nullptr, *rowidx = nullptr;
    double *val = nullptr;
    int *in_degree = nullptr;  // per row: entries in the row (incl. diagonal)
    // CSR (pull executor): built lazily with the device transpose
    int *rrowptr = nullptr, *rcol = nullptr;
    double *rval = nullptr;
    // scratch
    int *done = nullptr;       // push: arrivals per row; pull: ready flags
    double *left = nullptr;    // push: left sums
    double *left_rhs = nullptr;  // SpTRSM push: left sums n x rhs (grown on demand)
    size_t left_rhs_cap = 0;
    unsigned *ctl = nullptr;   // [0] ticket, [kAbort] timeout flag (kCtlBytes block)
    int nlevels = -1;
    int auto_algo = 0;         // sblas_trsv_solve algo 4: the pull executor's ticket order (1 or 3)
    int pull_threads = 0;      // fixed at create (0: by ticket order, pull_threads())
    // level-set executor (algo 2), built on its first solve: rows in level
    // order (stable by row), the CSR rows copied into that order, level
    // pointers, and the launch schedule (runs of narrow levels -> one
    // workgroup with barriers; each wide level -> one grid launch)
    int *lrow = nullptr, *lrp = nullptr, *lcol = nullptr;
    double *lval = nullptr;
    int *lptr_d = nullptr;
    unsigned *larrive = nullptr;            // grid barrier: arrival epoch per workgroup
    std::vector<int> lptr;                  // host copy [nlevels + 1]
    std::vector<std::pair<int, int>> lsched;  // (first level, end level); end < 0: wide level
};

namespace sblas {

constexpr unsigned kSpinLimit = 1u << 25;  // ~1 s of polling per wave
// control block: ticket counter at word 0, abort/timeout word on its own
// 128-B line (word 32) -- polling it next to the hot ticket atomics is slow
constexpr int kAbort = 32;
// multi-device blocks: first-start / last-exit timestamps (s_memrealtime,
// 100 MHz) as 64-bit words on a third line, so a test can see that blocks
// sharing a GPU overlap in time; start is kept as (~0 - t) under atomicMax
constexpr int kTStart64 = 32, kTEnd64 = 33;
constexpr int kCtlBytes = 384;

__device__ __forceinline__ void stamp_start(unsigned *ctl)
{
    if (threadIdx.x == 0)
        atomicMax((unsigned long long *)ctl + kTStart64,
                  ~0ULL - (unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void stamp_end(unsigned *ctl)
{
    atomicMax((unsigned long long *)ctl + kTEnd64, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

__device__ __forceinline__ int ld_sc1_i32(const int *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1_f64(const double *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_trsv_indegree(const int *__restrict__ rowidx, int nnz, int *__restrict__ deg)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nnz) atomicAdd(&deg[rowidx[e]], 1);
}

// ---- push: one wave per column, reference dataflow -----------------------
__global__ __launch_bounds__(256) void k_trsv_push(
    const int *__restrict__ colptr, const int *__restrict__ rowidx,
    const double *__restrict__ val, const int *__restrict__ in_degree, int n,
    int backward, const double *__restrict__ b, double *__restrict__ x, int *done,
    double *left, unsigned *ctl)
{
    const int lane = threadIdx.x & 63;
    for (;;) {
        int t = 0;
        if (lane == 0) t = ld_sc1_i32((const int *)&ctl[kAbort]) ? n : (int)atomicAdd(&ctl[0], 1u);
        t = __shfl(t, 0, 64);
        if (t >= n) return;
        const int i = backward ? n - 1 - t : t;
        const int a = colptr[i], e = colptr[i + 1];
        const int dpos = backward ? e - 1 : a;
        const double diag = val[dpos];
        const int need = in_degree[i] - 1;
        // wait for all left contributions (one lane polls)
        int bail = 0;
        if (lane == 0) {
            unsigned spins = 0;
            while (ld_sc1_i32(&done[i]) != need) {
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 1023u) == 0) {
                    if (spins > kSpinLimit) atomicOr(&ctl[kAbort], 1u);
                    if (ld_sc1_i32((const int *)&ctl[kAbort])) {
                        bail = 1;
                        break;
                    }
                }
            }
        }
        if (__shfl(bail, 0, 64)) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double xi = 0.0;
        if (lane == 0) {
            xi = (b[i] - ld_sc1_f64(&left[i])) / diag;
            x[i] = xi;
        }
        xi = __shfl(xi, 0, 64);
        const int lo = backward ? a : a + 1, hi = backward ? e - 1 : e;
        for (int j = lo + lane; j < hi; j += 64)
            (void)__hip_atomic_fetch_add(&left[rowidx[j]], xi * val[j], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int j = lo + lane; j < hi; j += 64)
            (void)__hip_atomic_fetch_add(&done[rowidx[j]], 1, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- pull: one lane per row over CSR, x itself is the ready flag -----------
// x is pre-filled with a signalling-NaN bit pattern that no arithmetic result
// can equal (IEEE operations return quiet NaNs), so one 8-byte sc1 store
// publishes x_i and one sc1 load both tests and fetches it.  Each lane loads
// up to 8 of its row's dependencies at once and consumes the ready prefix in
// column order (fixed summation order -> deterministic).
// Row layout: forward (lower) = off-diagonals ascending, diagonal LAST;
// backward (upper, rows processed from n-1 down) = diagonal FIRST.
constexpr unsigned long long kXPending = 0x7FF4DEADBEEF5A5AULL;

__global__ void k_fill_pending(unsigned long long *__restrict__ x, long long n)
{
    const long long stride = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        x[i] = kXPending;
}

static void fill_pending(unsigned long long *x, long long n, hipStream_t s)
{
    if (n <= 0) return;
    const long long blocks = std::min<long long>((n + 255) / 256, 1 << 16);
    hipLaunchKernelGGL(k_fill_pending, dim3((unsigned)blocks), dim3(256), 0, s, x, n);
}

__device__ __forceinline__ unsigned long long ld_sc1_u64(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Poll back-off of a wave whose lanes all still wait (SBLAS_TRSV_SLEEP):
// slp >= 0 sleeps slp x 64 clocks after every poll; slp < 0 doubles the
// sleep after each poll on which no lane of the wave advanced, up to 2^-slp,
// and drops it back to one on progress.  Every polling lane is an L2 request
// the producers also need, so fewer polls can shorten the chain.
__device__ __forceinline__ void trsv_backoff(int units)
{
    // s_sleep takes an immediate: whole 8-unit steps, then the remainder
    for (; units >= 8; units -= 8) __builtin_amdgcn_s_sleep(8);
    if (units & 4) __builtin_amdgcn_s_sleep(4);
    if (units & 2) __builtin_amdgcn_s_sleep(2);
    if (units & 1) __builtin_amdgcn_s_sleep(1);
}

// kLevel (algo 3): tickets walk the level-ordered CSR of the level-set
// analysis (position t holds row lrow[t]; rows of one level are contiguous),
// so the 64 rows of a wave belong to one level and become ready together
// instead of a wave waiting on its latest level.  Same sums, same order.
template <bool kLevel>
__global__ __launch_bounds__(256) void k_trsv_pull(
    const int *__restrict__ rowptr, const int *__restrict__ col,
    const double *__restrict__ val, int n, int backward, const double *__restrict__ b,
    unsigned long long *xbits, unsigned *ctl, const int *__restrict__ lrow, int slp)
{
    constexpr int kBatch = 8;
    const int lane = threadIdx.x & 63;
    const int slp_cap = slp < 0 ? 1 << min(-slp, 10) : slp;
    // spin limit of ~1 s of polling at a fixed back-off; the adaptive one
    // mixes short and long sleeps (a wave whose other lanes advance keeps
    // sleeping short), so it keeps 1/8 of the count: >= ~2 s, <= ~2 min
    const unsigned spin_lim = kSpinLimit / (unsigned)(slp < 0 ? 8 : max(slp_cap, 1));
    for (;;) {
        int t0 = 0;
        if (lane == 0) t0 = ld_sc1_i32((const int *)&ctl[kAbort]) ? n : (int)atomicAdd(&ctl[0], 64u);
        t0 = __shfl(t0, 0, 64);
        if (t0 >= n) return;  // done, or another wave timed out: the solve is void
        const int t = t0 + lane;
        const bool live = t < n;
        const int i = live ? (kLevel ? lrow[t] : (backward ? n - 1 - t : t)) : 0;
        const int ri = kLevel ? t : i;  // CSR row index of this row
        int j = 0, jend = 0;
        double diag = 1.0, sum = 0.0;
        if (live) {
            const int a = rowptr[ri], e = rowptr[ri + 1];
            if (backward) {
                diag = val[a];
                j = a + 1;
                jend = e;
            } else {
                diag = val[e - 1];
                j = a;
                jend = e - 1;
            }
        }
        bool pending = live;
        unsigned spins = 0;
        int cur = 1;  // adaptive back-off (slp < 0), wave-uniform
        // current dependency cached in registers: a spin costs ONE sc1 load
        int cj = (live && j < jend) ? col[j] : 0;
        double vj = (live && j < jend) ? val[j] : 0.0;
        while (__any(pending)) {
            bool adv = false;
            if (pending && j < jend) {
                const unsigned long long x0 = ld_sc1_u64(xbits + cj);
                if (x0 != kXPending) {
                    adv = true;
                    sum += vj * __longlong_as_double((long long)x0);
                    ++j;
                    if (j < jend) {  // ready: batch the next dependencies
                        int cc[kBatch - 1];
                        double vv[kBatch - 1];
                        unsigned long long xb[kBatch - 1];
#pragma unroll
                        for (int k = 0; k < kBatch - 1; ++k) {  // clamped, unconditional
                            const int jj = min(j + k, jend - 1);
                            cc[k] = col[jj];
                            vv[k] = val[jj];
                        }
#pragma unroll
                        for (int k = 0; k < kBatch - 1; ++k) xb[k] = ld_sc1_u64(xbits + cc[k]);
                        bool open = true;
#pragma unroll
                        for (int k = 0; k < kBatch - 1; ++k) {
                            if (open && j < jend) {
                                if (xb[k] == kXPending) {
                                    open = false;
                                } else {
                                    sum += vv[k] * __longlong_as_double((long long)xb[k]);
                                    ++j;
                                }
                            }
                        }
                        if (j < jend) {
                            cj = col[j];
                            vj = val[j];
                        }
                    }
                }
            }
            if (pending && j == jend) {
                const double xi = (b[i] - sum) / diag;
                __hip_atomic_store(xbits + i, (unsigned long long)__double_as_longlong(xi),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                pending = false;
                adv = true;
            }
            if (__any(pending)) {
                // a timeout voids the whole solve (every wave exits)
                if (slp < 0) {
                    cur = __any(adv) ? 1 : min(2 * cur, slp_cap);
                    trsv_backoff(cur);
                } else {
                    trsv_backoff(slp_cap);
                }
                if ((++spins & 1023u) == 0) {
                    if (spins > spin_lim) {
                        if (lane == 0) atomicOr(&ctl[kAbort], 1u);
                        return;
                    }
                    if (ld_sc1_i32((const int *)&ctl[kAbort])) return;
                }
            }
        }
    }
}

// ---- multi-device pull (replaces sptrsv_v3's NVSHMEM gets) ----
// Rows are split into g blocks of the solve order (o = i forward, n-1-i
// backward).  Device d solves its block and keeps a FULL-length x in
// fine-grained memory; dependencies always have a smaller order index, so
// they come from blocks <= d.  A producer publishes x_i with one system-scope
// store into its own x and into the x of every LATER block (xGMI peer writes
// when the blocks sit on other GPUs); consumers poll only local memory.
struct TrsvPart {
    const int *rowptr;   // local CSR of the block's rows (solve order)
    const int *col;      // global column indices
    const double *val;
    const double *b;     // local b (solve order)
    unsigned long long *const *xs;  // [g] x arrays (peer pointers); xs[d] = own
    int g, d, o0, nloc, n, backward;
};

__device__ __forceinline__ unsigned long long ld_sys_u64(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_trsv_pull_part(const TrsvPart P, unsigned *ctl)
{
    constexpr int kBatch = 8;
    const int lane = threadIdx.x & 63;
    unsigned long long *xl = P.xs[P.d];
    stamp_start(ctl);
    for (;;) {
        int t0 = 0;
        if (lane == 0) t0 = ld_sc1_i32((const int *)&ctl[kAbort]) ? P.nloc : (int)atomicAdd(&ctl[0], 64u);
        t0 = __shfl(t0, 0, 64);
        if (t0 >= P.nloc) {
            if (lane == 0) stamp_end(ctl);
            return;
        }
        const int t = t0 + lane;
        const bool live = t < P.nloc;
        const int o = P.o0 + (live ? t : 0);
        const int i = P.backward ? P.n - 1 - o : o;
        int j = 0, jend = 0;
        double diag = 1.0, sum = 0.0;
        if (live) {
            const int a = P.rowptr[t], e = P.rowptr[t + 1];
            if (P.backward) {
                diag = P.val[a];
                j = a + 1;
                jend = e;
            } else {
                diag = P.val[e - 1];
                j = a;
                jend = e - 1;
            }
        }
        bool pending = live;
        unsigned spins = 0;
        int cj = (live && j < jend) ? P.col[j] : 0;
        double vj = (live && j < jend) ? P.val[j] : 0.0;
        while (__any(pending)) {
            if (pending && j < jend) {
                const unsigned long long x0 = ld_sys_u64(xl + cj);
                if (x0 != kXPending) {
                    sum += vj * __longlong_as_double((long long)x0);
                    ++j;
                    if (j < jend) {
                        int cc[kBatch - 1];
                        double vv[kBatch - 1];
                        unsigned long long xb[kBatch - 1];
#pragma unroll
                        for (int k = 0; k < kBatch - 1; ++k) {
                            const int jj = min(j + k, jend - 1);
                            cc[k] = P.col[jj];
                            vv[k] = P.val[jj];
                        }
#pragma unroll
                        for (int k = 0; k < kBatch - 1; ++k) xb[k] = ld_sys_u64(xl + cc[k]);
                        bool open = true;
#pragma unroll
                        for (int k = 0; k < kBatch - 1; ++k) {
                            if (open && j < jend) {
                                if (xb[k] == kXPending) {
                                    open = false;
                                } else {
                                    sum += vv[k] * __longlong_as_double((long long)xb[k]);
                                    ++j;
                                }
                            }
                        }
                        if (j < jend) {
                            cj = P.col[j];
                            vj = P.val[j];
                        }
                    }
                }
            }
            if (pending && j == jend) {
                const double xi = (P.b[t] - sum) / diag;
                const unsigned long long bits = (unsigned long long)__double_as_longlong(xi);
                for (int q = P.d; q < P.g; ++q)  // own copy, then every later block's
                    __hip_atomic_store(P.xs[q] + i, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                pending = false;
            }
            if (__any(pending)) {
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 1023u) == 0) {
                    if (spins > kSpinLimit) {
                        if (lane == 0) atomicOr(&ctl[kAbort], 1u);
                        return;
                    }
                    if (ld_sc1_i32((const int *)&ctl[kAbort])) return;
                }
            }
        }
    }
}

// ---- SpTRSM: rhs > 1 (sptrsm_syncfree_cuda_executor, sptrsv_v1/src/
// sptrsv_syncfree_cuda.h:170-282; x and b are n x rhs row-major,
// x[i*rhs + k]).  Pull form: RP lanes per row (power of two <= 64) span the
// right-hand sides, 64/RP rows per wave from the monotone ticket; every x
// element is its own ready flag (sentinel), so each lane waits only for the
// element it reads and no fences are needed.  rhs > 64 runs in chunks of 64.
// Works single-device (by_row: CSR indexed by row, xs = {x}) and per block of
// the multi-device split (CSR/b indexed by local solve order, xs = peers).
struct TrsmArgs {
    const int *rowptr, *col;
    const double *val, *b;
    unsigned long long *xown;             // this block's x (polled)
    unsigned long long *const *xs;        // [g] peers' x (only q > d used); null if g == 1
    int g, d, o0, nloc, n, rhs, backward, by_row;
    const int *lrow;                      // level order (algo 3): ticket t is row lrow[t], CSR row t; else null
    int slp;                              // poll back-off (k_trsv_pull's SBLAS_TRSV_SLEEP units)
};

// RP lanes per row, each lane V right-hand sides RP apart (a pass covers
// RP x V of them), R = 64 / RP rows per wave step: V > 1 puts V independent
// polls in flight per lane and R x V rows on one ticket claim -- one claim
// per row at rhs 64 (V = 1) capped the solve at the single counter's ~85 M
// claims/s.  kSys: x polled at system scope (peer devices
// publish into it, g > 1); one device polls at agent scope (L2).  After a
// ready dependency the next kBatch - 1 are loaded together, as in
// k_trsv_pull.  Per column the same sums in the same order for every (RP, V).
template <int RP, int V, bool kSys>
__global__ __launch_bounds__(256) void k_trsm_pull(const TrsmArgs P, unsigned *ctl)
{
    constexpr int kBatch = V >= 4 ? 2 : 8 / V;
    constexpr int R = 64 / RP;
    const int lane = threadIdx.x & 63;
    const int slot = lane / RP, kl = lane % RP;
    const unsigned long long *xl = P.xown;
    // poll back-off as k_trsv_pull's (slp >= 0 fixed, < 0 adaptive)
    const int slp_cap = P.slp < 0 ? 1 << min(-P.slp, 10) : P.slp;
    const unsigned spin_lim = kSpinLimit / (unsigned)(P.slp < 0 ? 8 : max(slp_cap, 1));
    stamp_start(ctl);
    for (;;) {
        int t0 = 0;
        if (lane == 0) t0 = ld_sc1_i32((const int *)&ctl[kAbort]) ? P.nloc : (int)atomicAdd(&ctl[0], (unsigned)R);
        t0 = __shfl(t0, 0, 64);
        if (t0 >= P.nloc) {
            if (lane == 0) stamp_end(ctl);
            return;
        }
        const int t = t0 + slot;
        const bool live = t < P.nloc;
        const int o = P.o0 + (live ? t : 0);
        const int i = P.lrow ? (live ? P.lrow[t] : 0) : (P.backward ? P.n - 1 - o : o);
        const int ri = P.lrow ? (live ? t : 0) : (P.by_row ? i : (live ? t : 0));
        const int bi = P.lrow ? i : ri;  // b's row
        int j0 = 0, jend = 0;
        double diag = 1.0;
        if (live) {
            const int a = P.rowptr[ri], e = P.rowptr[ri + 1];
            if (P.backward) {
                diag = P.val[a];
                j0 = a + 1;
                jend = e;
            } else {
                diag = P.val[e - 1];
                j0 = a;
                jend = e - 1;
            }
        }
        for (int kc = 0; kc < P.rhs; kc += RP * V) {
            // this lane's columns k0 + v*RP, v < nv: each load instruction reads RP
            // consecutive columns of a row (one line at RP = 16), not RP strided groups
            const int k0 = kc + kl;
            const int rem = P.rhs - k0;
            const int nv = (live && rem > 0) ? min(V, (rem + RP - 1) / RP) : 0;
            bool pending = nv > 0;
            int j = j0;
            double sum[V];
#pragma unroll
            for (int v = 0; v < V; ++v) sum[v] = 0.0;
            unsigned spins = 0;
            int cur = 1;  // adaptive back-off, wave-uniform
            int cj = (pending && j < jend) ? P.col[j] : 0;
            double vj = (pending && j < jend) ? P.val[j] : 0.0;
            // x row c, this lane's columns (out-of-range columns read as 0: ready)
            auto ldrow = [&](int c, unsigned long long(&xv)[V]) {
                const unsigned long long *p = xl + (size_t)c * P.rhs + k0;
#pragma unroll
                for (int v = 0; v < V; ++v)
                    xv[v] = v < nv ? (kSys ? ld_sys_u64(p + v * RP) : ld_sc1_u64(p + v * RP)) : 0ull;
            };
            auto ready = [&](const unsigned long long(&xv)[V]) {
                bool r = true;
#pragma unroll
                for (int v = 0; v < V; ++v) r &= xv[v] != kXPending;
                return r;
            };
            auto acc = [&](double a, const unsigned long long(&xv)[V]) {
#pragma unroll
                for (int v = 0; v < V; ++v) sum[v] += a * __longlong_as_double((long long)xv[v]);
            };
            while (__any(pending)) {
                bool adv = false;
                if (pending && j < jend) {
                    unsigned long long xv[V];
                    ldrow(cj, xv);
                    if (ready(xv)) {
                        adv = true;
                        acc(vj, xv);
                        if (++j < jend) {  // ready: batch the next dependencies
                            int cc[kBatch - 1];
                            double vv[kBatch - 1];
                            unsigned long long xb[kBatch - 1][V];
#pragma unroll
                            for (int u = 0; u < kBatch - 1; ++u) {  // clamped, unconditional
                                const int jj = min(j + u, jend - 1);
                                cc[u] = P.col[jj];
                                vv[u] = P.val[jj];
                            }
#pragma unroll
                            for (int u = 0; u < kBatch - 1; ++u) ldrow(cc[u], xb[u]);
                            bool open = true;
#pragma unroll
                            for (int u = 0; u < kBatch - 1; ++u) {
                                if (open && j < jend) {
                                    if (!ready(xb[u])) {
                                        open = false;
                                    } else {
                                        acc(vv[u], xb[u]);
                                        ++j;
                                    }
                                }
                            }
                            if (j < jend) {
                                cj = P.col[j];
                                vj = P.val[j];
                            }
                        }
                    }
                }
                if (pending && j == jend) {
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        if (v >= nv) break;
                        const double xi = (P.b[(size_t)bi * P.rhs + k0 + v * RP] - sum[v]) / diag;
                        const unsigned long long bits = (unsigned long long)__double_as_longlong(xi);
                        const size_t at = (size_t)i * P.rhs + k0 + v * RP;
                        if (kSys)
                            __hip_atomic_store(P.xown + at, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        else
                            __hip_atomic_store(P.xown + at, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        for (int q = P.d + 1; q < P.g; ++q)
                            __hip_atomic_store(P.xs[q] + at, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    pending = false;
                    adv = true;
                }
                if (__any(pending)) {
                    if (P.slp < 0) {
                        cur = __any(adv) ? 1 : min(2 * cur, slp_cap);
                        trsv_backoff(cur);
                    } else {
                        trsv_backoff(slp_cap);
                    }
                    if ((++spins & 1023u) == 0) {
                        if (spins > spin_lim) {
                            if (lane == 0) atomicOr(&ctl[kAbort], 1u);
                            return;
                        }
                        if (ld_sc1_i32((const int *)&ctl[kAbort])) return;
                    }
                }
            }
        }
    }
}

// Right-hand sides per lane for pass width c (rhs rounded up to a power of
// two, <= 64).  Measured (r03_trsm_v3, ms; config-5 stand-in natural order /
// 27-point 100^3 stencil level order):
//   rhs   V=1          V=2          V=4          V=8
//    4    4.22 / 3.01  3.21 / 3.50  4.95 / 8.19  4.95 / 8.19
//    8    8.21 / 3.14  4.29 / 3.30  4.61 / 5.68  8.29 / 19.2
//   16   16.2  / 3.81  8.25 / 3.51  6.48 / 5.10  7.58 / 13.2
//   32   32.2  / 6.32  16.3 / 3.85  10.2 / 5.01  10.2 / 8.54
//   64   64.3  / 11.8  32.6 / 6.38  17.2 / 4.94  16.0 / 7.94
// Natural order is bound by the ticket counter (~85 M claims/s, one claim
// per 64 / RP rows) up to V = 4: wider lanes, fewer claims.  In level order a
// wave's rows are independent rows of one level and longer per-lane rows
// lengthen every level.  An experiment build (Makefile `alt`,
// -DSBLAS_TRSM_V=v) fixes V.
static int trsm_cols_per_lane(int c, bool level)
{
#ifdef SBLAS_TRSM_V
    (void)c;
    (void)level;
    return SBLAS_TRSM_V >= 8 ? 8 : SBLAS_TRSM_V >= 4 ? 4 : SBLAS_TRSM_V >= 2 ? 2 : 1;
#endif
    if (level) return c <= 8 ? 1 : c <= 32 ? 2 : 4;
    return c <= 8 ? 2 : c <= 32 ? 4 : 8;
}

template <int V, bool kSys>
static void launch_trsm_v(int rp, const TrsmArgs &P, unsigned *ctl, int grid, hipStream_t s)
{
    switch (rp) {
    case 1: hipLaunchKernelGGL((k_trsm_pull<1, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    case 2: hipLaunchKernelGGL((k_trsm_pull<2, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    case 4: hipLaunchKernelGGL((k_trsm_pull<4, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    case 8: hipLaunchKernelGGL((k_trsm_pull<8, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    case 16: hipLaunchKernelGGL((k_trsm_pull<16, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    case 32: hipLaunchKernelGGL((k_trsm_pull<32, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    default: hipLaunchKernelGGL((k_trsm_pull<64, V, kSys>), dim3(grid), dim3(256), 0, s, P, ctl); break;
    }
}

template <bool kSys>
static void launch_trsm_t(const TrsmArgs &P, unsigned *ctl, int grid, hipStream_t s)
{
    int c = 1;  // pass width: right-hand sides rounded up to a power of two, <= 64
    while (c < P.rhs && c < 64) c *= 2;
    const int v = std::min(trsm_cols_per_lane(c, P.lrow != nullptr), c);
    const int rp = c / v;
    if (v == 8) launch_trsm_v<8, kSys>(rp, P, ctl, grid, s);
    else if (v == 4) launch_trsm_v<4, kSys>(rp, P, ctl, grid, s);
    else if (v == 2) launch_trsm_v<2, kSys>(rp, P, ctl, grid, s);
    else launch_trsm_v<1, kSys>(rp, P, ctl, grid, s);
}

static void launch_trsm(const TrsmArgs &P, unsigned *ctl, int grid, hipStream_t s)
{
    if (P.g > 1) launch_trsm_t<true>(P, ctl, grid, s);
    else launch_trsm_t<false>(P, ctl, grid, s);
}

// ---- SpTRSM push: the reference's dataflow with its lane mappings ---------
// sptrsm_syncfree_cuda_executor (sptrsv_v1/src/sptrsv_syncfree_cuda.h:170-282):
// one wave per column (monotone ticket, as k_trsv_push), the column's
// contributions scattered into left sums n x rhs with fp64 atomics, then the
// in-degree counters bumped.  The lane mapping is the reference's `opt`:
//   kOptNnz  (OPT_WARP_NNZ, 1): lanes over the column's entries, each lane
//            loops over the rhs;
//   kOptRhs  (OPT_WARP_RHS, 2): lanes over the rhs, entries in sequence;
//   kOptAuto (OPT_WARP_AUTO, 3): per column, the rhs mapping when
//            (len <= rhs || rhs > 16) && len < 2048, else the nnz mapping.
// Counters are bumped once per entry after all rhs of the entry have landed
// (s_waitcnt vmcnt(0) orders the atomics, as in k_trsv_push).  Sums are added
// in arrival order: within the fp64 bound, exact on integer systems.
constexpr int kOptNnz = 1, kOptRhs = 2, kOptAuto = 3;

template <int kOpt>
__global__ __launch_bounds__(256) void k_trsm_push(
    const int *__restrict__ colptr, const int *__restrict__ rowidx,
    const double *__restrict__ val, const int *__restrict__ in_degree, int n, int backward,
    int rhs, const double *__restrict__ b, double *x, int *done, double *left, unsigned *ctl)
{
    const int lane = threadIdx.x & 63;
    for (;;) {
        int t = 0;
        if (lane == 0) t = ld_sc1_i32((const int *)&ctl[kAbort]) ? n : (int)atomicAdd(&ctl[0], 1u);
        t = __shfl(t, 0, 64);
        if (t >= n) return;
        const int i = backward ? n - 1 - t : t;
        const int a = colptr[i], e = colptr[i + 1];
        const double diag = val[backward ? e - 1 : a];
        const int need = in_degree[i] - 1;
        int bail = 0;
        if (lane == 0) {
            unsigned spins = 0;
            while (ld_sc1_i32(&done[i]) != need) {
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 1023u) == 0) {
                    if (spins > kSpinLimit) atomicOr(&ctl[kAbort], 1u);
                    if (ld_sc1_i32((const int *)&ctl[kAbort])) {
                        bail = 1;
                        break;
                    }
                }
            }
        }
        if (__shfl(bail, 0, 64)) return;
        const int lo = backward ? a : a + 1, hi = backward ? e - 1 : e;
        const int len = hi - lo;
        const bool by_rhs = kOpt == kOptRhs ||
                            (kOpt == kOptAuto && (len <= rhs || rhs > 16) && len < 2048);
        const size_t xi = (size_t)i * rhs;
        for (int kc = 0; kc < rhs; kc += 64) {
            const int k = kc + lane;
            if (k >= rhs) break;
            const double xk = (b[xi + k] - ld_sc1_f64(&left[xi + k])) / diag;
            __hip_atomic_store(&x[xi + k], xk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (by_rhs)
                for (int j = lo; j < hi; ++j)
                    (void)__hip_atomic_fetch_add(&left[(size_t)rowidx[j] * rhs + k], xk * val[j],
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!by_rhs)
            for (int j = lo + lane; j < hi; j += 64) {
                const size_t r = (size_t)rowidx[j] * rhs;
                const double v = val[j];
                for (int k = 0; k < rhs; ++k)
                    (void)__hip_atomic_fetch_add(&left[r + k], ld_sc1_f64(&x[xi + k]) * v,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int j = lo + lane; j < hi; j += 64)
            (void)__hip_atomic_fetch_add(&done[rowidx[j]], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---- level-set executor (algo 2; findlevel.h:71-147's level sets) --------
// Rows are solved level by level: every row of level l depends only on rows
// of levels < l, so no ready flags are needed -- a level boundary is a kernel
// boundary (wide levels) or a workgroup barrier (a run of narrow levels in
// one workgroup).  Sums in CSR column order, as the pull executor: the two
// give bit-identical x.  The comparison baseline for the sync-free
// executors: one synchronisation per level, whatever the dependencies.
__device__ __forceinline__ void level_row(const int *__restrict__ lrp, const int *__restrict__ lcol,
                                          const double *__restrict__ lval, const int *__restrict__ lrow,
                                          int k, int backward, const double *__restrict__ b, double *x)
{
    const int i = lrow[k];
    const int a = lrp[k], e = lrp[k + 1];
    const double diag = backward ? lval[a] : lval[e - 1];
    const int j0 = backward ? a + 1 : a, j1 = backward ? e : e - 1;
    double sum = 0.0;
    for (int j = j0; j < j1; ++j) sum += lval[j] * ld_sc1_f64(x + lcol[j]);
    __hip_atomic_store(x + i, (b[i] - sum) / diag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_trsv_level(const int *__restrict__ lrp, const int *__restrict__ lcol,
                                                    const double *__restrict__ lval, const int *__restrict__ lrow,
                                                    int p0, int p1, int backward, const double *__restrict__ b,
                                                    double *x)
{
    const int k = p0 + (int)(blockIdx.x * 256 + threadIdx.x);
    if (k < p1) level_row(lrp, lcol, lval, lrow, k, backward, b, x);
}

constexpr int kLevelWG = 1024;         // threads of the narrow-run workgroup
constexpr int kLevelNarrow = 2 * kLevelWG;  // a level with <= this many rows is narrow
constexpr int kLevelMaxWG = 1024;           // grid-barrier workgroups (arrival words)

__global__ __launch_bounds__(kLevelWG) void k_trsv_level_run(
    const int *__restrict__ lrp, const int *__restrict__ lcol, const double *__restrict__ lval,
    const int *__restrict__ lrow, const int *__restrict__ lptr, int l0, int l1, int backward,
    const double *__restrict__ b, double *x)
{
    for (int l = l0; l < l1; ++l) {
        for (int k = lptr[l] + (int)threadIdx.x; k < lptr[l + 1]; k += kLevelWG)
            level_row(lrp, lcol, lval, lrow, k, backward, b, x);
        // this level's x stores (agent scope) complete before any wave reads them
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// A run of wide levels in ONE launch: a persistent grid (every workgroup
// resident) strides over each level's rows, then meets at a grid barrier.
// The barrier avoids one hot counter (256 RMWs on one address serialise at
// the memory side: ~19 us per level, measured): workgroup w stores its
// arrival epoch into its own word arrive[w]; workgroup 0's first wave reads
// all of them (64 per load) and then publishes the epoch in a release word
// that everyone polls.  Plain agent-scope (sc1) loads/stores, no fences: x
// itself travels through agent-scope stores and sc1 loads, and every wave's
// x stores drained (vmcnt(0)) before its workgroup's barrier.  Bounded
// spins; the abort word voids the solve as in the sync-free executors.
__global__ __launch_bounds__(1024) void k_trsv_level_grid(
    const int *__restrict__ lrp, const int *__restrict__ lcol, const double *__restrict__ lval,
    const int *__restrict__ lrow, const int *__restrict__ lptr, int l0, int l1, int backward,
    const double *__restrict__ b, double *x, unsigned *ctl, unsigned *arrive)
{
    const unsigned nwg = gridDim.x;
    unsigned *release = &ctl[1];
    for (int l = l0; l < l1; ++l) {
        const int p1 = lptr[l + 1];
        for (int k = lptr[l] + (int)(blockIdx.x * blockDim.x + threadIdx.x); k < p1;
             k += (int)(nwg * blockDim.x))
            level_row(lrp, lcol, lval, lrow, k, backward, b, x);
        if (l + 1 == l1) break;
        const unsigned epoch = (unsigned)(l - l0 + 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(&arrive[blockIdx.x], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool bail = false;
        if (blockIdx.x == 0 && threadIdx.x < 64) {  // the master wave gathers every arrival
            unsigned spins = 0;
            for (;;) {
                bool all = true;
                for (unsigned w = threadIdx.x; w < nwg; w += 64)
                    all &= __hip_atomic_load(&arrive[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
                if (__all(all)) break;
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 255u) == 0 &&
                    (spins > kSpinLimit || __hip_atomic_load(&ctl[kAbort], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                    bail = true;
                    break;
                }
            }
            if (threadIdx.x == 0) {
                if (bail) atomicOr(&ctl[kAbort], 1u);
                else __hip_atomic_store(release, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (threadIdx.x == 0) {
            unsigned spins = 0;
            while (__hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 1023u) == 0 &&
                    (spins > kSpinLimit || __hip_atomic_load(&ctl[kAbort], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                    atomicOr(&ctl[kAbort], 1u);
                    break;
                }
            }
        }
        __syncthreads();
        if (__hip_atomic_load(&ctl[kAbort], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
}

// Threads per pull workgroup (one workgroup per CU, grid_for): the waves
// spinning on a CU.  Every pending lane polls, and the polls share the
// memory path with the producers' stores and loads, so fewer waves shorten
// each dependency hop -- as long as enough rows are in flight to cover a
// level.  Config-5 stand-in (natural order, 985 levels): 1 / 2 / 3 / 4 waves
// per CU 2.44 / 2.12 / 2.24 / 2.45 ms; level order (a ticket holds 64 rows of
// one level): 27-point 100^3 1.79 / 1.92 / 1.99 / 2.03 ms, 7-point 0.81 /
// 0.85 / 0.87 / 0.89 ms (profiles/r05/trsv_waves/).  An experiment build
// (-DSBLAS_TRSV_THREADS = 64 / 128 / 192 / 256) overrides.  The multi-device blocks keep 256: four
// blocks sharing one GPU ran 4.7 ms at 4 waves per CU and 6.2 at 2 (each
// block then has a quarter of the grid), and one block per GPU is unmeasured
// here.
#ifndef SBLAS_TRSV_THREADS
#define SBLAS_TRSV_THREADS 0
#endif
static int pull_threads_env()  // fixed when a handle is created
{
    constexpr int t = SBLAS_TRSV_THREADS;
    return t == 64 || t == 128 || t == 192 || t == 256 ? t : 0;
}
static int pull_threads(bool level_order, int forced)
{
    return forced ? forced : level_order ? 64 : 128;
}

static int grid_for(int dev)
{
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 1024;
    // one workgroup per CU (the pull executors' pull_threads() threads each,
    // the push executor's 256).  More spinning waves is slower: every polling
    // lane costs an L2 request the producers need (config 5, pull: 1/CU 2.44
    // ms, 2/CU 2.99 ms, 4/CU 4.92 ms at 256 threads; 8/CU starves the chain).
    return p.multiProcessorCount;
}

}  // namespace sblas

using namespace sblas;

extern "C" {

int sblas_trsv_create(sblas_trsv *out, int device, int n, int nnz, const int *d_colptr,
                      const int *d_rowidx, const double *d_val, int substitution, void *stream)
{
    if (!out || n < 0 || nnz < n || (substitution != 0 && substitution != 1)) return SBLAS_ERR_INVALID;
    int phys;
    SBLAS_TRY(resolve_device(device, &phys));
    DeviceGuard g(phys);
    hipStream_t s = (hipStream_t)stream;
    auto *T = new sblas_trsv_s();
    T->device = phys;
    T->n = n;
    T->nnz = nnz;
    T->substitution = substitution;
    T->pull_threads = pull_threads_env();
    auto fail = [&](hipError_t e) {
        set_error("sblas_trsv_create: %s", hipGetErrorString(e));
        sblas_trsv_destroy(T);
        return SBLAS_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipMalloc(&T->colptr, sizeof(int) * ((size_t)n + 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->rowidx, sizeof(int) * std::max(nnz, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->val, sizeof(double) * std::max(nnz, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->in_degree, sizeof(int) * std::max(n, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->done, sizeof(int) * std::max(n, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->left, sizeof(double) * std::max(n, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->ctl, kCtlBytes)) != hipSuccess) return fail(e);
    if ((e = hipMemcpyAsync(T->colptr, d_colptr, sizeof(int) * ((size_t)n + 1), hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(e);
    if (nnz) {
        if ((e = hipMemcpyAsync(T->rowidx, d_rowidx, sizeof(int) * nnz, hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(e);
        if ((e = hipMemcpyAsync(T->val, d_val, sizeof(double) * nnz, hipMemcpyDeviceToDevice, s)) != hipSuccess) return fail(e);
    }
    if ((e = hipMemsetAsync(T->in_degree, 0, sizeof(int) * std::max(n, 1), s)) != hipSuccess) return fail(e);
    if (nnz) hipLaunchKernelGGL(k_trsv_indegree, dim3((nnz + 255) / 256), dim3(256), 0, s, T->rowidx, nnz, T->in_degree);
    if ((e = hipGetLastError()) != hipSuccess) return fail(e);
    // CSR copy for the pull executor: transpose of the CSC (= CSC of L^T).
    sblas_csr_s csc;
    csc.device = phys;
    csc.m = n;  // "rows" of the CSC-as-CSR are L's columns
    csc.n = n;
    csc.nnz = nnz;
    csc.rowptr = T->colptr;
    csc.col = T->rowidx;
    csc.val = T->val;
    if ((e = hipMalloc(&T->rrowptr, sizeof(int) * ((size_t)n + 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->rcol, sizeof(int) * std::max(nnz, 1))) != hipSuccess) return fail(e);
    if ((e = hipMalloc(&T->rval, sizeof(double) * std::max(nnz, 1))) != hipSuccess) return fail(e);
    int st = launch_transpose(csc, T->rrowptr, T->rcol, T->rval, s);
    csc.rowptr = nullptr;
    csc.col = nullptr;
    csc.val = nullptr;
    if (st != SBLAS_OK) {
        sblas_trsv_destroy(T);
        return st;
    }
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return fail(e);
    *out = T;
    return SBLAS_OK;
}

// level sets of the solve (rows of level l depend only on levels < l), as
// findlevel.h:71-147 computes them: level(i) = 1 + max level of i's
// dependencies, walking columns in solve order
static void host_levels(const sblas_trsv_s *T, const std::vector<int> &cp, const std::vector<int> &ri,
                        std::vector<int> &lev, int &nl)
{
    lev.assign((size_t)T->n, 0);
    nl = 0;
    for (int k = 0; k < T->n; ++k) {
        const int i = T->substitution ? T->n - 1 - k : k;
        const int li = lev[(size_t)i];
        nl = std::max(nl, li + 1);
        for (int j = cp[(size_t)i]; j < cp[(size_t)i + 1]; ++j)
            if (ri[(size_t)j] != i) lev[(size_t)ri[(size_t)j]] = std::max(lev[(size_t)ri[(size_t)j]], li + 1);
    }
}

static int build_levelset(sblas_trsv_s *T, hipStream_t s)
{
    if (T->lrow) return SBLAS_OK;
    const int n = T->n, nnz = T->nnz;
    std::vector<int> cp((size_t)n + 1), ri((size_t)nnz);
    SBLAS_HIP(hipStreamSynchronize(s));
    SBLAS_HIP(hipMemcpy(cp.data(), T->colptr, sizeof(int) * cp.size(), hipMemcpyDeviceToHost));
    if (nnz) SBLAS_HIP(hipMemcpy(ri.data(), T->rowidx, sizeof(int) * ri.size(), hipMemcpyDeviceToHost));
    std::vector<int> lev;
    int nl = 0;
    host_levels(T, cp, ri, lev, nl);
    T->nlevels = nl;
    // counting sort of the rows by level (stable: ascending row in a level)
    T->lptr.assign((size_t)nl + 1, 0);
    for (int i = 0; i < n; ++i) T->lptr[(size_t)lev[(size_t)i] + 1]++;
    for (int l = 0; l < nl; ++l) T->lptr[(size_t)l + 1] += T->lptr[(size_t)l];
    std::vector<int> lrow((size_t)std::max(n, 1)), next(T->lptr.begin(), T->lptr.end() - 1);
    for (int i = 0; i < n; ++i) lrow[(size_t)next[(size_t)lev[(size_t)i]]++] = i;
    // CSR rows (the pull executor's device CSR) copied into level order
    std::vector<int> rrp((size_t)n + 1), rc((size_t)std::max(nnz, 1));
    std::vector<double> rv((size_t)std::max(nnz, 1));
    SBLAS_HIP(hipMemcpy(rrp.data(), T->rrowptr, sizeof(int) * rrp.size(), hipMemcpyDeviceToHost));
    if (nnz) {
        SBLAS_HIP(hipMemcpy(rc.data(), T->rcol, sizeof(int) * nnz, hipMemcpyDeviceToHost));
        SBLAS_HIP(hipMemcpy(rv.data(), T->rval, sizeof(double) * nnz, hipMemcpyDeviceToHost));
    }
    std::vector<int> lrp((size_t)n + 1, 0), lc((size_t)std::max(nnz, 1));
    std::vector<double> lv((size_t)std::max(nnz, 1));
    for (int k = 0; k < n; ++k) {
        const int i = lrow[(size_t)k];
        const int len = rrp[(size_t)i + 1] - rrp[(size_t)i];
        std::copy(rc.begin() + rrp[(size_t)i], rc.begin() + rrp[(size_t)i + 1], lc.begin() + lrp[(size_t)k]);
        std::copy(rv.begin() + rrp[(size_t)i], rv.begin() + rrp[(size_t)i + 1], lv.begin() + lrp[(size_t)k]);
        lrp[(size_t)k + 1] = lrp[(size_t)k] + len;
    }
    // schedule: maximal runs of narrow levels (one workgroup, workgroup
    // barriers) and of wide levels (persistent grid, grid barriers), encoded
    // (l0, l1) narrow / (l0, -l1) wide
    T->lsched.clear();
    auto narrow = [&](int l) { return T->lptr[(size_t)l + 1] - T->lptr[(size_t)l] <= kLevelNarrow; };
    for (int l = 0; l < nl;) {
        const bool nw = narrow(l);
        int e = l;
        while (e < nl && narrow(e) == nw) ++e;
        T->lsched.push_back({l, nw ? e : -e});
        l = e;
    }
    SBLAS_HIP(hipMalloc(&T->lrow, sizeof(int) * lrow.size()));
    SBLAS_HIP(hipMalloc(&T->lrp, sizeof(int) * lrp.size()));
    SBLAS_HIP(hipMalloc(&T->lcol, sizeof(int) * lc.size()));
    SBLAS_HIP(hipMalloc(&T->lval, sizeof(double) * lv.size()));
    SBLAS_HIP(hipMalloc(&T->lptr_d, sizeof(int) * T->lptr.size()));
    SBLAS_HIP(hipMalloc(&T->larrive, sizeof(unsigned) * kLevelMaxWG));
    SBLAS_HIP(hipMemcpy(T->lrow, lrow.data(), sizeof(int) * lrow.size(), hipMemcpyHostToDevice));
    SBLAS_HIP(hipMemcpy(T->lrp, lrp.data(), sizeof(int) * lrp.size(), hipMemcpyHostToDevice));
    SBLAS_HIP(hipMemcpy(T->lcol, lc.data(), sizeof(int) * lc.size(), hipMemcpyHostToDevice));
    SBLAS_HIP(hipMemcpy(T->lval, lv.data(), sizeof(double) * lv.size(), hipMemcpyHostToDevice));
    SBLAS_HIP(hipMemcpy(T->lptr_d, T->lptr.data(), sizeof(int) * T->lptr.size(), hipMemcpyHostToDevice));
    return SBLAS_OK;
}

static int solve_levelset(sblas_trsv_s *T, const double *b, double *x, hipStream_t s)
{
    SBLAS_TRY(build_levelset(T, s));
    SBLAS_HIP(hipMemsetAsync(T->ctl, 0, kCtlBytes, s));
    int ncu = 0;
    SBLAS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, T->device));
#ifndef SBLAS_TRSV_LEVEL_LAUNCH  // experiment builds: one launch per wide level
#define SBLAS_TRSV_LEVEL_LAUNCH 0
#endif
    constexpr int per_level = SBLAS_TRSV_LEVEL_LAUNCH;
    for (const auto &seg : T->lsched) {
        if (seg.second < 0 && per_level) {
            for (int l = seg.first; l < -seg.second; ++l) {
                const int p0 = T->lptr[(size_t)l], p1 = T->lptr[(size_t)l + 1];
                hipLaunchKernelGGL(k_trsv_level, dim3((unsigned)((p1 - p0 + 255) / 256)), dim3(256), 0, s, T->lrp,
                                   T->lcol, T->lval, T->lrow, p0, p1, T->substitution, b, x);
            }
        } else if (seg.second < 0) {
            // one 1024-thread workgroup per CU: all resident (the barrier's premise)
            const int nwg = std::max(1, std::min(ncu, kLevelMaxWG));
            SBLAS_HIP(hipMemsetAsync(T->ctl, 0, 8, s));
            SBLAS_HIP(hipMemsetAsync(T->larrive, 0, sizeof(unsigned) * kLevelMaxWG, s));
            hipLaunchKernelGGL(k_trsv_level_grid, dim3((unsigned)nwg), dim3(1024), 0, s, T->lrp, T->lcol, T->lval,
                               T->lrow, T->lptr_d, seg.first, -seg.second, T->substitution, b, x, T->ctl,
                               T->larrive);
        } else {
            hipLaunchKernelGGL(k_trsv_level_run, dim3(1), dim3(kLevelWG), 0, s, T->lrp, T->lcol, T->lval, T->lrow,
                               T->lptr_d, seg.first, seg.second, T->substitution, b, x);
        }
    }
    SBLAS_HIP(hipGetLastError());
    unsigned h[kCtlBytes / 4] = {0};
    SBLAS_HIP(hipMemcpyAsync(h, T->ctl, kCtlBytes, hipMemcpyDeviceToHost, s));
    SBLAS_HIP(hipStreamSynchronize(s));
    if (h[kAbort]) {
        set_error("sptrsv level-set: grid barrier spin limit exceeded");
        return SBLAS_ERR_HIP;
    }
    return SBLAS_OK;
}

// Rows (sampled, <= 65,536 spread over the solve order) with a dependency
// inside their own 64-row ticket of the natural order: such a row waits on a
// lane of its own wave, so a chain runs through every lane of the wave (a
// stencil's row i - 1), one global store -> poll round trip per lane.
// cnt = {rows with a local dependency, rows sampled}.
__global__ void k_trsv_local_deps(const int *__restrict__ rowptr, const int *__restrict__ col, int n,
                                  int backward, int S, unsigned long long *cnt)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned local = 0, tot = 0;
    if (t < S) {
        const int o = (int)((long long)t * n / S);  // solve order
        const int i = backward ? n - 1 - o : o;
        const int a = rowptr[i], b = rowptr[i + 1];
        bool hit = false;
        for (int e = a; e < b && e < a + 64; ++e) {
            const int j = col[e];
            if (j == i) continue;
            const int oj = backward ? n - 1 - j : j;
            hit |= (oj >> 6) == (o >> 6);
        }
        local = hit;
        tot = 1;
    }
    for (int off = 32; off > 0; off >>= 1) {
        local += __shfl_down(local, off, 64);
        tot += __shfl_down(tot, off, 64);
    }
    if ((threadIdx.x & 63) == 0 && tot) {
        atomicAdd(&cnt[0], (unsigned long long)local);
        atomicAdd(&cnt[1], (unsigned long long)tot);
    }
}

// algo 4: the pull executor in natural order (1) unless at least a quarter
// of the rows depend on a row of their own wave, then in level order (3):
// lower triangles of 3-D stencils 2.3-4x faster in level order, the banded
// random config-5 stand-in 1.4x slower
static int trsv_pick(sblas_trsv_s *T, hipStream_t s)
{
    if (T->auto_algo) return T->auto_algo;
    const int S = std::min(T->n, 65536);
    unsigned long long *d = nullptr, h[2] = {0, 0};
    // errors come back negative (callers read a positive return as the choice)
    hipError_t e = hipMalloc(&d, sizeof(h));
    if (e != hipSuccess) {
        set_error("sblas_trsv_solve (auto): hipMalloc: %s", hipGetErrorString(e));
        return -SBLAS_ERR_HIP;
    }
    e = hipMemsetAsync(d, 0, sizeof(h), s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_trsv_local_deps, dim3((S + 255) / 256), dim3(256), 0, s, T->rrowptr, T->rcol, T->n,
                           T->substitution, S, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    if (e != hipSuccess) {
        set_error("sblas_trsv_solve (auto): %s", hipGetErrorString(e));
        return -SBLAS_ERR_HIP;
    }
    T->auto_algo = (h[1] && 4 * h[0] >= h[1]) ? 3 : 1;
    return T->auto_algo;
}

int sblas_trsv_pick(sblas_trsv T, void *stream, int *algo)
{
    if (!T || !algo) return SBLAS_ERR_INVALID;
    if (T->n == 0) {
        *algo = 1;
        return SBLAS_OK;
    }
    DeviceGuard g(T->device);
    const int a = trsv_pick(T, (hipStream_t)stream);
    if (a < 0) return -a;
    *algo = a;
    return SBLAS_OK;
}

int sblas_trsv_solve(sblas_trsv T, int algo, const double *d_b, double *d_x, void *stream)
{
    if (!T || !d_b || !d_x || algo < 0 || algo > 4) return SBLAS_ERR_INVALID;
    if (T->n == 0) return SBLAS_OK;
    DeviceGuard g(T->device);
    hipStream_t s = (hipStream_t)stream;
    if (algo == 4) {
        const int a = trsv_pick(T, s);
        if (a < 0) return -a;
        algo = a;
    }
    if (algo == 2) return solve_levelset(T, d_b, d_x, s);
    if (algo == 3) SBLAS_TRY(build_levelset(T, s));
    SBLAS_HIP(hipMemsetAsync(T->ctl, 0, kCtlBytes, s));
    const int grid = grid_for(T->device);
    // poll back-off of the pull executors (k_trsv_pull header): natural order
    // one s_sleep(1) per poll; level order the adaptive back-off up to 64
    // units (-6: 27-point 100^3 2.25 -> 2.03 ms, 7-point 0.97 -> 0.88 ms; -8
    // and deeper lose; profiles/r03/sptrsv_sleep/)
    const int slp = algo == 3 ? -6 : 1;
    const int pth = pull_threads(algo == 3, T->pull_threads);
    if (algo == 3) {  // sync-free pull, tickets in level order
        fill_pending((unsigned long long *)d_x, T->n, s);
        hipLaunchKernelGGL(k_trsv_pull<true>, dim3(grid), dim3(pth), 0, s, T->lrp, T->lcol, T->lval, T->n,
                           T->substitution, d_b, (unsigned long long *)d_x, T->ctl, T->lrow, slp);
    } else if (algo == 0) {
        SBLAS_HIP(hipMemsetAsync(T->done, 0, sizeof(int) * T->n, s));
        SBLAS_HIP(hipMemsetAsync(T->left, 0, sizeof(double) * T->n, s));
        hipLaunchKernelGGL(k_trsv_push, dim3(grid), dim3(256), 0, s, T->colptr, T->rowidx, T->val,
                           T->in_degree, T->n, T->substitution, d_b, d_x, T->done, T->left, T->ctl);
    } else {
        fill_pending((unsigned long long *)d_x, T->n, s);
        hipLaunchKernelGGL(k_trsv_pull<false>, dim3(grid), dim3(pth), 0, s, T->rrowptr, T->rcol, T->rval,
                           T->n, T->substitution, d_b, (unsigned long long *)d_x, T->ctl, nullptr, slp);
    }
    SBLAS_HIP(hipGetLastError());
    unsigned h[kCtlBytes / 4] = {0};
    SBLAS_HIP(hipMemcpyAsync(h, T->ctl, kCtlBytes, hipMemcpyDeviceToHost, s));
    SBLAS_HIP(hipStreamSynchronize(s));
    if (h[kAbort]) {
        set_error("sptrsv: spin limit exceeded (matrix not triangular or missing diagonal?)");
        return SBLAS_ERR_HIP;
    }
    return SBLAS_OK;
}

// SpTRSM pull: tickets in natural order, or in level order (level = true:
// the rows of a ticket independent, as algo 3 of sblas_trsv_solve)
static int trsm_pull(sblas_trsv_s *T, bool level, int rhs, const double *d_b, double *d_x, hipStream_t s)
{
    if (level) SBLAS_TRY(build_levelset(T, s));
    SBLAS_HIP(hipMemsetAsync(T->ctl, 0, kCtlBytes, s));
    fill_pending((unsigned long long *)d_x, (long long)T->n * rhs, s);
    TrsmArgs P{level ? T->lrp : T->rrowptr, level ? T->lcol : T->rcol, level ? T->lval : T->rval, d_b,
               (unsigned long long *)d_x, nullptr, 1, 0, 0, T->n, T->n, rhs, T->substitution, 1,
               level ? T->lrow : nullptr, level ? -6 : 1};
    // workgroups per CU (x grid_for's): natural order at rhs >= 16 gains from
    // more rows in flight (config 5: rhs 16 / 32 / 64 at 1 -> 2 -> 4 per CU:
    // 6.50 / 10.2 / 16.1 -> 4.63 / 8.55 / 10.4 -> 4.86 / 8.53 / 9.26 ms); level
    // order loses (27-point stencil rhs 64: 4.93 / 5.12 / 5.32 ms;
    // profiles/r03/sptrsm/trsm_grid2/).
    const int mult = level || rhs < 16 ? 1 : rhs <= 32 ? 2 : 4;
    const int grid = grid_for(T->device) * mult;
    launch_trsm(P, T->ctl, grid, s);
    SBLAS_HIP(hipGetLastError());
    unsigned h[kCtlBytes / 4] = {0};
    SBLAS_HIP(hipMemcpyAsync(h, T->ctl, kCtlBytes, hipMemcpyDeviceToHost, s));
    SBLAS_HIP(hipStreamSynchronize(s));
    if (h[kAbort]) {
        set_error("sptrsm: spin limit exceeded (matrix not triangular or missing diagonal?)");
        return SBLAS_ERR_HIP;
    }
    return SBLAS_OK;
}

int sblas_trsv_solve_rhs(sblas_trsv T, int rhs, const double *d_b, double *d_x, void *stream)
{
    if (!T || !d_b || !d_x || rhs <= 0) return SBLAS_ERR_INVALID;
    if (rhs == 1) return sblas_trsv_solve(T, 1, d_b, d_x, stream);
    if (T->n == 0) return SBLAS_OK;
    DeviceGuard g(T->device);
    return trsm_pull(T, false, rhs, d_b, d_x, (hipStream_t)stream);
}

int sblas_trsv_solve_rhs_opt(sblas_trsv T, int algo, int opt, int rhs, const double *d_b,
                             double *d_x, void *stream)
{
    if (!T || !d_b || !d_x || rhs <= 0 || algo < 0 || algo > 4 || algo == 2) return SBLAS_ERR_INVALID;
    if (algo == 1) return sblas_trsv_solve_rhs(T, rhs, d_b, d_x, stream);
    if (algo != 0 && rhs == 1) return sblas_trsv_solve(T, algo, d_b, d_x, stream);
    if (algo == 0 && (opt < kOptNnz || opt > kOptAuto)) return SBLAS_ERR_INVALID;
    if (T->n == 0) return SBLAS_OK;
    DeviceGuard g(T->device);
    hipStream_t s = (hipStream_t)stream;
    if (algo == 4) {
        const int a = trsv_pick(T, s);
        if (a < 0) return -a;
        algo = a;
    }
    if (algo != 0) return trsm_pull(T, algo == 3, rhs, d_b, d_x, s);
    const size_t need = (size_t)T->n * rhs;
    if (need > T->left_rhs_cap) {
        if (T->left_rhs) SBLAS_HIP(hipFree(T->left_rhs));
        T->left_rhs = nullptr;
        T->left_rhs_cap = 0;
        SBLAS_HIP(hipMalloc(&T->left_rhs, sizeof(double) * need));
        T->left_rhs_cap = need;
    }
    SBLAS_HIP(hipMemsetAsync(T->ctl, 0, kCtlBytes, s));
    SBLAS_HIP(hipMemsetAsync(T->done, 0, sizeof(int) * T->n, s));
    SBLAS_HIP(hipMemsetAsync(T->left_rhs, 0, sizeof(double) * need, s));
    const int grid = grid_for(T->device);
#define SBLAS_TRSM_PUSH(O)                                                                        \
    hipLaunchKernelGGL(k_trsm_push<O>, dim3(grid), dim3(256), 0, s, T->colptr, T->rowidx, T->val, \
                       T->in_degree, T->n, T->substitution, rhs, d_b, d_x, T->done, T->left_rhs,  \
                       T->ctl)
    if (opt == kOptNnz) SBLAS_TRSM_PUSH(kOptNnz);
    else if (opt == kOptRhs) SBLAS_TRSM_PUSH(kOptRhs);
    else SBLAS_TRSM_PUSH(kOptAuto);
#undef SBLAS_TRSM_PUSH
    SBLAS_HIP(hipGetLastError());
    unsigned h[kCtlBytes / 4] = {0};
    SBLAS_HIP(hipMemcpyAsync(h, T->ctl, kCtlBytes, hipMemcpyDeviceToHost, s));
    SBLAS_HIP(hipStreamSynchronize(s));
    if (h[kAbort]) {
        set_error("sptrsm: spin limit exceeded (matrix not triangular or missing diagonal?)");
        return SBLAS_ERR_HIP;
    }
    return SBLAS_OK;
}

int sblas_trsv_levels(sblas_trsv T, int *nlevel)
{
    if (!T || !nlevel) return SBLAS_ERR_INVALID;
    if (T->nlevels < 0) {
        DeviceGuard g(T->device);
        std::vector<int> cp((size_t)T->n + 1), ri((size_t)T->nnz);
        SBLAS_HIP(hipMemcpy(cp.data(), T->colptr, sizeof(int) * cp.size(), hipMemcpyDeviceToHost));
        if (T->nnz) SBLAS_HIP(hipMemcpy(ri.data(), T->rowidx, sizeof(int) * ri.size(), hipMemcpyDeviceToHost));
        std::vector<int> lev;
        int nl = 0;
        host_levels(T, cp, ri, lev, nl);
        T->nlevels = nl;
    }
    *nlevel = T->nlevels;
    return SBLAS_OK;
}

int sblas_trsv_destroy(sblas_trsv T)
{
    if (!T) return SBLAS_OK;
    {
        DeviceGuard g(T->device);
        (void)hipFree(T->colptr);
        (void)hipFree(T->rowidx);
        (void)hipFree(T->val);
        (void)hipFree(T->in_degree);
        (void)hipFree(T->rrowptr);
        (void)hipFree(T->rcol);
        (void)hipFree(T->rval);
        (void)hipFree(T->done);
        (void)hipFree(T->left);
        (void)hipFree(T->left_rhs);
        (void)hipFree(T->ctl);
        (void)hipFree(T->lrow);
        (void)hipFree(T->lrp);
        (void)hipFree(T->lcol);
        (void)hipFree(T->lval);
        (void)hipFree(T->lptr_d);
        (void)hipFree(T->larrive);
    }
    delete T;
    return SBLAS_OK;
}


}  // extern "C"

namespace {

// Multi-device solve from HOST CSC (diagonal first / last per column as in the
// reference), as a persistent handle: sblas_trsv_mgpu_create builds the
// blocks once (CSC -> CSR of L, nnz-balanced blocks of the solve order, each
// block's CSR rows uploaded to its device, fine-grained x per block), and
// every sblas_trsv_mgpu_run only uploads b, resets x / the control words,
// launches and copies x back.  nblocks blocks of the solve order; block d
// runs on ordinal (d % ndev) % count.  balance 0 = nnz-balanced blocks
// (sptrsv_v1/v2's intent), 1 = equal row counts (sptrsv_v3's
// floor(d*m/(np*task)), sptrsv_v3/src/sptrsv_syncfree_cuda.h:276-300).
// Every block has its own stream and all are launched before any is waited
// for, so blocks that share a GPU run CONCURRENTLY like blocks on different
// GPUs: each gets grid_for(dev) / (blocks on dev) workgroups, so the blocks
// of one device are co-resident.  Launches go in block order; a block only
// waits for lower blocks, which were enqueued first on every hardware queue,
// so streams sharing a queue cannot deadlock.  An experiment build with
// -DSBLAS_TRSV_MGPU_SERIAL=1 runs
// the blocks of one device in order on one stream instead (A/B timing).
struct TrsvMgpuDev {
    int phys = 0;
    int nloc = 0;
    int *rowptr = nullptr, *col = nullptr;
    double *val = nullptr, *b = nullptr;
    unsigned long long *x = nullptr;
    unsigned long long **xs = nullptr;
    unsigned *ctl = nullptr;
    std::vector<double> hb;  // staging of the block's b rows
};

}  // namespace

struct sblas_trsv_mgpu_s {
    int n = 0, rhs = 1, nblocks = 0, ndev = 0;
    bool bwd = false, serial = false;
    int pull_threads = 0;  // fixed at create (0: 256 threads per workgroup)
    std::vector<int> ob;                  // block boundaries in the solve order
    std::vector<TrsvMgpuDev> D;
    std::vector<hipStream_t> streams;     // per block (serial: per device's first block)
    std::vector<int> on_phys, first_on;
    std::vector<std::pair<int, int>> peers;  // peer links taken (peer_acquire), released on destroy
    hipStream_t stream_of(int d) const { return streams[serial ? first_on[D[d].phys] : d]; }
};

namespace {

void trsv_mgpu_free(sblas_trsv_mgpu_s *H)
{
    for (auto &q : H->D) {
        DeviceGuard g(q.phys);
        (void)hipFree(q.rowptr);
        (void)hipFree(q.col);
        (void)hipFree(q.val);
        (void)hipFree(q.b);
        (void)hipFree(q.x);
        (void)hipFree(q.xs);
        (void)hipFree(q.ctl);
    }
    for (int d = 0; d < (int)H->streams.size(); ++d)
        if (H->streams[d]) {
            DeviceGuard g(H->D[d].phys);
            (void)hipStreamDestroy(H->streams[d]);
        }
    for (const auto &pr : H->peers) peer_release(pr.first, pr.second);
    delete H;
}

#define MG(expr)                                                               \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            set_error("trsv_mgpu: %s -> %s", #expr, hipGetErrorString(e_));    \
            return SBLAS_ERR_HIP;                                              \
        }                                                                      \
    } while (0)

int trsv_mgpu_build(sblas_trsv_mgpu_s *H, const int *colptr, const int *rowidx, const double *val, int n,
                    int substitution, int rhs, int nblocks, int ndev, int balance)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SBLAS_ERR_NODEV;
    const int ngpu = nblocks;
    H->n = n;
    H->rhs = rhs;
    H->nblocks = nblocks;
    H->ndev = ndev;
#ifndef SBLAS_TRSV_MGPU_SERIAL  // experiment builds: one device's blocks in order on one stream
#define SBLAS_TRSV_MGPU_SERIAL 0
#endif
    H->serial = SBLAS_TRSV_MGPU_SERIAL != 0;
    H->pull_threads = pull_threads_env();
    const int nnz = colptr[n];
    const bool bwd = H->bwd = substitution == 1;
    // CSC of L == CSR of L^T; stable transpose gives CSR of L with columns
    // ascending (diagonal last for lower, first for upper)
    std::vector<int> rp((size_t)n + 1, 0), cl((size_t)std::max(nnz, 1));
    std::vector<double> vl((size_t)std::max(nnz, 1));
    for (int e = 0; e < nnz; ++e) rp[(size_t)rowidx[e] + 1]++;
    for (int i = 0; i < n; ++i) rp[(size_t)i + 1] += rp[(size_t)i];
    {
        std::vector<int> nx(rp.begin(), rp.end() - 1);
        for (int c = 0; c < n; ++c)
            for (int e = colptr[c]; e < colptr[c + 1]; ++e) {
                const int o = nx[(size_t)rowidx[e]]++;
                cl[(size_t)o] = c;
                vl[(size_t)o] = val[e];
            }
    }
    // order index o -> row i; nnz-balanced blocks of the order
    auto row_of = [&](int o) { return bwd ? n - 1 - o : o; };
    std::vector<int> &ob = H->ob;
    ob.assign((size_t)ngpu + 1, n);
    ob[0] = 0;
    if (balance == 1) {
        for (int d = 1; d < ngpu; ++d) ob[d] = (int)((long long)d * n / ngpu);
    } else {
        long long acc = 0;
        int d = 1;
        for (int o = 0; o < n && d < ngpu; ++o) {
            const int i = row_of(o);
            acc += rp[(size_t)i + 1] - rp[(size_t)i];
            while (d < ngpu && acc >= (long long)nnz * d / ngpu) ob[d++] = o + 1;
        }
        for (; d < ngpu; ++d) ob[d] = n;
    }
    H->D.assign(ngpu, TrsvMgpuDev{});
    H->streams.assign(ngpu, nullptr);
    H->on_phys.assign(count, 0);
    H->first_on.assign(count, -1);
    const int nphys = std::min(count, ndev);
    for (int d = 0; d < ngpu; ++d) {
        H->D[d].phys = (d % ndev) % count;
        H->on_phys[H->D[d].phys]++;
        if (H->first_on[H->D[d].phys] < 0) H->first_on[H->D[d].phys] = d;
    }
    for (int d = 0; d < ngpu; ++d) {
        // serial mode: the blocks of one device share its first block's stream
        if (H->serial && H->first_on[H->D[d].phys] != d) continue;
        DeviceGuard g(H->D[d].phys);
        MG(hipStreamCreateWithFlags(&H->streams[d], hipStreamNonBlocking));
    }
    // producers store x_i into every later block's fine-grained x: blocks on
    // distinct devices need the peer link, and without it the build fails
    // here -- before anything is launched, so no block can spin on an x it
    // will never receive (sptrsv_v3's NVSHMEM setup fails the same way,
    // sptrsv_syncfree_cuda.h:245-249).  The sblas_test_deny_peer_access hook
    // treats blocks sharing one GPU as distinct devices, so a one-GPU box
    // exercises the refusal.
    for (int p = 0; p < nphys; ++p)
        for (int q = 0; q < nphys; ++q) {
            if (q == p) continue;
            SBLAS_TRY(peer_acquire(p, q, "trsv_mgpu"));
            H->peers.emplace_back(p, q);
        }
    if (ngpu > 1 && peer_denied()) SBLAS_TRY(peer_acquire(H->D[0].phys, H->D[1].phys, "trsv_mgpu"));
    std::vector<unsigned long long *> xs(ngpu);
    for (int d = 0; d < ngpu; ++d) {
        TrsvMgpuDev &q = H->D[d];
        DeviceGuard g(q.phys);
        const int nloc = q.nloc = ob[d + 1] - ob[d];
        std::vector<int> lrp((size_t)nloc + 1, 0), lcol;
        std::vector<double> lval;
        for (int t = 0; t < nloc; ++t) {
            const int i = row_of(ob[d] + t);
            for (int e = rp[(size_t)i]; e < rp[(size_t)i + 1]; ++e) {
                lcol.push_back(cl[(size_t)e]);
                lval.push_back(vl[(size_t)e]);
            }
            lrp[(size_t)t + 1] = (int)lcol.size();
        }
        q.hb.assign((size_t)std::max(nloc, 1) * rhs, 0.0);
        MG(hipMalloc(&q.rowptr, sizeof(int) * ((size_t)nloc + 1)));
        MG(hipMalloc(&q.col, sizeof(int) * std::max<size_t>(lcol.size(), 1)));
        MG(hipMalloc(&q.val, sizeof(double) * std::max<size_t>(lval.size(), 1)));
        MG(hipMalloc(&q.b, sizeof(double) * std::max(nloc, 1) * rhs));
        MG(hipMalloc(&q.ctl, kCtlBytes));
        MG(hipExtMallocWithFlags((void **)&q.x, sizeof(double) * std::max(n, 1) * rhs,
                                 hipDeviceMallocFinegrained));
        MG(hipMalloc(&q.xs, sizeof(void *) * ngpu));
        MG(hipMemcpy(q.rowptr, lrp.data(), sizeof(int) * lrp.size(), hipMemcpyHostToDevice));
        if (!lcol.empty()) {
            MG(hipMemcpy(q.col, lcol.data(), sizeof(int) * lcol.size(), hipMemcpyHostToDevice));
            MG(hipMemcpy(q.val, lval.data(), sizeof(double) * lval.size(), hipMemcpyHostToDevice));
        }
        xs[d] = q.x;
    }
    for (int d = 0; d < ngpu; ++d) {
        DeviceGuard g(H->D[d].phys);
        MG(hipMemcpy(H->D[d].xs, xs.data(), sizeof(void *) * ngpu, hipMemcpyHostToDevice));
    }
    return SBLAS_OK;
}

int trsv_mgpu_run(sblas_trsv_mgpu_s *H, const double *b, double *x, double *solve_ms)
{
    const int ngpu = H->nblocks, n = H->n, rhs = H->rhs;
    const bool bwd = H->bwd;
    const std::vector<int> &ob = H->ob;
    auto row_of = [&](int o) { return bwd ? n - 1 - o : o; };
    // b rows of each block in its solve order; reset: sentinel x everywhere,
    // zero control words
    for (int d = 0; d < ngpu; ++d) {
        TrsvMgpuDev &q = H->D[d];
        DeviceGuard g(q.phys);
        hipStream_t s = H->stream_of(d);
        for (int t = 0; t < q.nloc; ++t) {
            const int i = row_of(ob[d] + t);
            for (int k = 0; k < rhs; ++k) q.hb[(size_t)t * rhs + k] = b[(size_t)i * rhs + k];
        }
        if (q.nloc)
            MG(hipMemcpyAsync(q.b, q.hb.data(), sizeof(double) * q.nloc * rhs, hipMemcpyHostToDevice, s));
        fill_pending(q.x, (long long)n * rhs, s);
        MG(hipMemsetAsync(q.ctl, 0, kCtlBytes, s));
    }
    for (int d = 0; d < ngpu; ++d) {
        DeviceGuard g(H->D[d].phys);
        MG(hipStreamSynchronize(H->stream_of(d)));
    }
    const double t0 = sblas_get_time();
    for (int d = 0; d < ngpu; ++d) {
        TrsvMgpuDev &q = H->D[d];
        DeviceGuard g(q.phys);
        const int nloc = q.nloc;
        // co-resident blocks: the device's workgroup budget split between them
        const int grid = H->serial ? grid_for(q.phys) : std::max(1, grid_for(q.phys) / H->on_phys[q.phys]);
        if (nloc > 0 && rhs == 1) {
            TrsvPart P{q.rowptr, q.col, q.val, q.b, q.xs, ngpu, d, ob[d], nloc, n, bwd ? 1 : 0};
            hipLaunchKernelGGL(k_trsv_pull_part, dim3(grid), dim3(H->pull_threads ? H->pull_threads : 256), 0, H->stream_of(d), P,
                               q.ctl);
        } else if (nloc > 0) {
            TrsmArgs P{q.rowptr, q.col, q.val, q.b,    q.x, q.xs, ngpu, d, ob[d], nloc, n, rhs, bwd ? 1 : 0, 0,
                       nullptr, 1};
            launch_trsm(P, q.ctl, grid, H->stream_of(d));
        }
        MG(hipGetLastError());
    }
    for (int d = 0; d < ngpu; ++d) {
        DeviceGuard g(H->D[d].phys);
        MG(hipStreamSynchronize(H->stream_of(d)));
    }
    if (solve_ms) *solve_ms = (sblas_get_time() - t0) * 1e3;
    for (int d = 0; d < ngpu; ++d) {
        TrsvMgpuDev &q = H->D[d];
        DeviceGuard g(q.phys);
        unsigned h[kCtlBytes / 4] = {0};
        MG(hipMemcpy(h, q.ctl, kCtlBytes, hipMemcpyDeviceToHost));
        if (h[kAbort]) {
            set_error("trsv_mgpu: partition %d exceeded its spin limit", d);
            return SBLAS_ERR_HIP;
        }
        // x rows of this block: contiguous rows in row space
        if (q.nloc == 0) continue;
        const size_t ia = (size_t)(bwd ? n - ob[d + 1] : ob[d]) * rhs;
        MG(hipMemcpy(x + ia, (double *)q.x + ia, sizeof(double) * q.nloc * rhs, hipMemcpyDeviceToHost));
    }
    return SBLAS_OK;
}
#undef MG

int trsv_mgpu_create(sblas_trsv_mgpu *out, const int *colptr, const int *rowidx, const double *val, int n,
                     int substitution, int rhs, int nblocks, int ndev, int balance)
{
    if (!out || n < 0 || nblocks <= 0 || ndev <= 0 || rhs <= 0 || !colptr || (substitution != 0 && substitution != 1) ||
        (balance != 0 && balance != 1))
        return SBLAS_ERR_INVALID;
    auto *H = new sblas_trsv_mgpu_s();
    const int st = trsv_mgpu_build(H, colptr, rowidx, val, n, substitution, rhs, nblocks, ndev, balance);
    if (st != SBLAS_OK) {
        trsv_mgpu_free(H);
        return st;
    }
    *out = H;
    return SBLAS_OK;
}

// one-shot form: create, run once, destroy
int trsv_mgpu_impl(const int *colptr, const int *rowidx, const double *val, int n, int substitution, int rhs,
                   const double *b, double *x, int nblocks, int ndev, int balance, double *solve_ms)
{
    if (!b || !x) return SBLAS_ERR_INVALID;
    sblas_trsv_mgpu H = nullptr;
    SBLAS_TRY(trsv_mgpu_create(&H, colptr, rowidx, val, n, substitution, rhs, nblocks, ndev, balance));
    const int st = trsv_mgpu_run(H, b, x, solve_ms);
    trsv_mgpu_free(H);
    return st;
}
}  // namespace

extern "C" {

int sblas_trsv_mgpu_solve(const int *colptr, const int *rowidx, const double *val, int n,
                          int substitution, int rhs, const double *b, double *x, int ngpu,
                          double *solve_ms)
{
    return trsv_mgpu_impl(colptr, rowidx, val, n, substitution, rhs, b, x, ngpu, ngpu, 0, solve_ms);
}

int sblas_trsv_mgpu_solve_tasks(const int *colptr, const int *rowidx, const double *val, int n,
                                int substitution, int rhs, const double *b, double *x, int ngpu,
                                int tasks, int balance, double *solve_ms)
{
    if (tasks <= 0 || ngpu <= 0 || (balance != 0 && balance != 1)) return SBLAS_ERR_INVALID;
    return trsv_mgpu_impl(colptr, rowidx, val, n, substitution, rhs, b, x, ngpu * tasks, ngpu,
                          balance, solve_ms);
}

int sblas_trsv_mgpu_create(sblas_trsv_mgpu *out, const int *colptr, const int *rowidx, const double *val,
                           int n, int substitution, int rhs, int ngpu, int tasks, int balance)
{
    if (tasks <= 0 || ngpu <= 0) return SBLAS_ERR_INVALID;
    return trsv_mgpu_create(out, colptr, rowidx, val, n, substitution, rhs, ngpu * tasks, ngpu, balance);
}

int sblas_trsv_mgpu_run(sblas_trsv_mgpu H, const double *b, double *x, double *solve_ms)
{
    if (!H || !b || !x) return SBLAS_ERR_INVALID;
    return trsv_mgpu_run(H, b, x, solve_ms);
}

int sblas_trsv_mgpu_info(sblas_trsv_mgpu H, int *nblocks, int *block_device, int *block_rows)
{
    if (!H) return SBLAS_ERR_INVALID;
    if (nblocks) *nblocks = H->nblocks;
    for (int d = 0; d < H->nblocks; ++d) {
        if (block_device) block_device[d] = H->D[d].phys;
        if (block_rows) block_rows[d] = H->D[d].nloc;
    }
    return SBLAS_OK;
}

int sblas_trsv_mgpu_destroy(sblas_trsv_mgpu H)
{
    if (H) trsv_mgpu_free(H);
    return SBLAS_OK;
}
}  // extern "C"
