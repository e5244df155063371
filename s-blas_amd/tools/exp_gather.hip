// exp_gather.hip -- microbenchmark: what does a random fp64 x gather cost
// beside the 12 B/nnz CSR stream, on MI355X?  (DESIGN.md §4 floor argument)
//
// Streams nnz (col int32, val f64) pairs with 16-B loads, gathers x[col] and
// accumulates; the column generator decides where the gathers land:
//   mode 0: x[0]                          (stream only, no gather cost)
//   mode 1: uniform over all n            (config 2: 16 MB of x)
//   mode 2: uniform over the XCD's 1/8    (blockIdx % 8 picks the slice, 2 MB)
//   mode 3: uniform over a 1/4 slice      (blockIdx % 4, 4 MB; two XCDs each)
//   mode 4: uniform over a 1/16 slice per XCD (1 MB)
// Columns are written by a setup kernel so the timed kernel reads them.
// A second kernel gathers only (columns hashed in registers, no stream).
//   hipcc --offload-arch=gfx950 -O3 exp_gather.hip -o exp_gather && ./exp_gather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned hash32(unsigned a)
{
    a ^= a >> 16; a *= 0x7feb352dU; a ^= a >> 15; a *= 0x846ca68bU; a ^= a >> 16;
    return a;
}

__device__ __forceinline__ int pick(long long e, long long blk, int n, int mode)
{
    const unsigned h = hash32((unsigned)e * 2654435761u + 12345u);
    switch (mode) {
    case 0: return 0;
    case 1: return (int)(h % (unsigned)n);
    case 2: { const int W = n / 8; return (int)(blk % 8) * W + (int)(h % (unsigned)W); }
    case 3: { const int W = n / 4; return (int)(blk % 4) * W + (int)(h % (unsigned)W); }
    default: { const int W = n / 16; return (int)(blk % 8) * W + (int)(h % (unsigned)W); }
    }
}

// one 256-thread block covers CH elements; block b's columns follow `mode`
__global__ void k_setup(int *col, double *val, long long nnz, int n, int mode, int CH)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nnz) return;
    col[e] = pick(e, e / CH, n, mode);
    val[e] = 1.0 + (e & 0xff) * 1e-3;
}

// K groups of 4 elements per lane per pass; all loads issued before use.
template <int K>
__global__ __launch_bounds__(256) void k_stream_gather(const int *__restrict__ col,
                                                       const double *__restrict__ val,
                                                       const double *__restrict__ x, long long nnz,
                                                       int CH, double *__restrict__ out)
{
    const long long b0 = (long long)blockIdx.x * CH;
    const long long b1 = b0 + CH < nnz ? b0 + CH : nnz;
    double s = 0.0;
    for (long long e = b0 + 4LL * threadIdx.x; e < b1; e += 4LL * 256 * K) {
        v4i c[K];
        v2d va[K], vb[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            long long ek = e + 4LL * 256 * k;
            if (ek >= b1) ek = e;
            c[k] = __builtin_nontemporal_load(reinterpret_cast<const v4i *>(col + ek));
            va[k] = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(val + ek));
            vb[k] = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(val + ek + 2));
        }
        double xv[K][4];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            xv[k][0] = x[c[k].x];
            xv[k][1] = x[c[k].y];
            xv[k][2] = x[c[k].z];
            xv[k][3] = x[c[k].w];
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            s += va[k].x * xv[k][0] + va[k].y * xv[k][1] + vb[k].x * xv[k][2] + vb[k].y * xv[k][3];
    }
    out[(long long)blockIdx.x * 256 + threadIdx.x] = s;
}

// Lane-consecutive layout: wave-instruction k of a lane group gathers 64
// CONSECUTIVE elements (4-B col / 8-B val loads), so sorted columns put
// several lanes of one instruction on one x line (coalesced by the TA).
template <int K>
__global__ __launch_bounds__(256) void k_stream_gather_lc(const int *__restrict__ col,
                                                          const double *__restrict__ val,
                                                          const double *__restrict__ x,
                                                          long long nnz, int CH,
                                                          double *__restrict__ out)
{
    const long long b0 = (long long)blockIdx.x * CH;
    const long long b1 = b0 + CH < nnz ? b0 + CH : nnz;
    double s = 0.0;
    for (long long e = b0 + threadIdx.x; e < b1; e += 256LL * K) {
        int c[K];
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            long long ek = e + 256LL * k;
            if (ek >= b1) ek = e;
            c[k] = __builtin_nontemporal_load(col + ek);
            v[k] = __builtin_nontemporal_load(val + ek);
        }
        double xv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) xv[k] = x[c[k]];
#pragma unroll
        for (int k = 0; k < K; ++k) s += v[k] * xv[k];
    }
    out[(long long)blockIdx.x * 256 + threadIdx.x] = s;
}

// gathers only, three load flavours: 0 plain, 1 nontemporal, 2 agent-scope
// relaxed atomic load (L1 bypass)
template <int F>
__global__ __launch_bounds__(256) void k_gather_flavour(const double *__restrict__ x, long long nnz,
                                                        int n, int mode, int CH,
                                                        double *__restrict__ out)
{
    const long long b0 = (long long)blockIdx.x * CH;
    const long long b1 = b0 + CH < nnz ? b0 + CH : nnz;
    double s = 0.0;
    for (long long e = b0 + threadIdx.x; e < b1; e += 256LL * 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const long long ek = e + 256LL * k;
            const double *p = x + pick(ek < b1 ? ek : e, blockIdx.x, n, mode);
            if (F == 0) v[k] = *p;
            else if (F == 1) v[k] = __builtin_nontemporal_load(p);
            else v[k] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    out[(long long)blockIdx.x * 256 + threadIdx.x] = s;
}

// gathers only: 8 per lane in flight, columns from a hash (no HBM stream)
__global__ __launch_bounds__(256) void k_gather_only(const double *__restrict__ x, long long nnz,
                                                     int n, int mode, int CH,
                                                     double *__restrict__ out)
{
    const long long b0 = (long long)blockIdx.x * CH;
    const long long b1 = b0 + CH < nnz ? b0 + CH : nnz;
    double s = 0.0;
    for (long long e = b0 + threadIdx.x; e < b1; e += 256LL * 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const long long ek = e + 256LL * k;
            v[k] = x[pick(ek < b1 ? ek : e, blockIdx.x, n, mode)];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    out[(long long)blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename F>
float timeit(F launch, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

int main()
{
    const int n = 2000000;
    const long long nnz = 39750000;
    int *col;
    double *val, *x, *out;
    CK(hipMalloc(&col, sizeof(int) * (nnz + 64)));
    CK(hipMalloc(&val, sizeof(double) * (nnz + 64)));
    CK(hipMalloc(&x, sizeof(double) * n));
    CK(hipMalloc(&out, sizeof(double) * 256 * ((nnz + 511) / 512 + 1)));
    CK(hipMemset(x, 0, sizeof(double) * n));
    const double bytes = 12.0 * nnz;
    // Sorted-window modes (host generated): block b of CH elements draws its
    // columns uniformly from panel p = (b % 8) * 4 + (b / 8) % 4 of width
    // n / 32 (500 KB of x, XCD-staggered), either sorted (mode 5: lanes of a
    // wave share x lines) or in random order (mode 6).
    for (int mode : {1, 2}) {
        const int CH = 8192;
        const unsigned grid = (unsigned)((nnz + CH - 1) / CH);
        const float f0 = timeit([&] { k_gather_flavour<0><<<grid, 256>>>(x, nnz, n, mode, CH, out); }, 20);
        const float f1 = timeit([&] { k_gather_flavour<1><<<grid, 256>>>(x, nnz, n, mode, CH, out); }, 20);
        const float f2 = timeit([&] { k_gather_flavour<2><<<grid, 256>>>(x, nnz, n, mode, CH, out); }, 20);
        printf("gather-only mode=%d  plain %7.1f us  nontemporal %7.1f us  agent-atomic %7.1f us\n",
               mode, f0 * 1e3, f1 * 1e3, f2 * 1e3);
        fflush(stdout);
    }
    {
        std::vector<int> h((size_t)nnz);
        const int W = n / 32;
        unsigned long long s = 0x1234567ULL;
        auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
        for (int CH : {4096, 8192, 16384}) {
            const unsigned grid = (unsigned)((nnz + CH - 1) / CH);
            for (int mode = 5; mode <= 6; ++mode) {
                for (long long b = 0; b * CH < nnz; ++b) {
                    const long long e0 = b * CH, e1 = std::min<long long>(nnz, e0 + CH);
                    const int p = (int)((b % 8) * 4 + (b / 8) % 4);
                    for (long long e = e0; e < e1; ++e) h[e] = p * W + (int)(rnd() % W);
                    if (mode == 5) std::sort(h.begin() + e0, h.begin() + e1);
                }
                CK(hipMemcpy(col, h.data(), sizeof(int) * nnz, hipMemcpyHostToDevice));
                const float t1 = timeit([&] { k_stream_gather<1><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
                const float t4 = timeit([&] { k_stream_gather<4><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
                const float l8 = timeit([&] { k_stream_gather_lc<8><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
                const float l16 = timeit([&] { k_stream_gather_lc<16><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
                printf("CH=%5d mode=%d  stream+gather K=1 %7.1f us (%5.2f TB/s)  K=4 %7.1f us (%5.2f)  "
                       "lane-consecutive K=8 %7.1f us (%5.2f)  K=16 %7.1f us (%5.2f)\n",
                       CH, mode, t1 * 1e3, bytes / t1 / 1e9, t4 * 1e3, bytes / t4 / 1e9,
                       l8 * 1e3, bytes / l8 / 1e9, l16 * 1e3, bytes / l16 / 1e9);
                fflush(stdout);
            }
        }
    }
    const int CHs[] = {2048, 8192};
    for (int CH : CHs) {
        const unsigned grid = (unsigned)((nnz + CH - 1) / CH);
        for (int mode = 0; mode <= 4; ++mode) {
            k_setup<<<(unsigned)((nnz + 255) / 256), 256>>>(col, val, nnz, n, mode, CH);
            CK(hipDeviceSynchronize());
            const float t1 = timeit([&] { k_stream_gather<1><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
            const float t2 = timeit([&] { k_stream_gather<2><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
            const float t4 = timeit([&] { k_stream_gather<4><<<grid, 256>>>(col, val, x, nnz, CH, out); }, 20);
            const float tg = timeit([&] { k_gather_only<<<grid, 256>>>(x, nnz, n, mode, CH, out); }, 20);
            printf("CH=%5d mode=%d  stream+gather K=1 %7.1f us (%5.2f TB/s)  K=2 %7.1f us (%5.2f)  "
                   "K=4 %7.1f us (%5.2f)   gather-only %7.1f us (%.1f G gathers/s)\n",
                   CH, mode, t1 * 1e3, bytes / t1 / 1e9, t2 * 1e3, bytes / t2 / 1e9, t4 * 1e3,
                   bytes / t4 / 1e9, tg * 1e3, nnz / tg / 1e6);
            fflush(stdout);
        }
    }
    CK(hipFree(col));
    CK(hipFree(val));
    CK(hipFree(x));
    CK(hipFree(out));
    return 0;
}
