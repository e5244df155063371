// exp_sgather.hip -- microbenchmark: can the scalar (constant) cache path add
// random fp64 gather throughput beside the vector path's L1/TA, on MI355X?
// (xsort is bound by each CU's L1->L2 request rate.)
//
// Gathers only, uniform over the XCD's 2 MiB slice of a 16 MiB x (blockIdx % 8
// picks the slice: L2-resident, like xsort's column groups):
//   mode 0: vector  -- 8 gathers in flight per lane (64 per wave instruction)
//   mode 1: scalar  -- the wave's address in SGPRs, s_load_dwordx2, 8 in flight
//   mode 2: both    -- every wave issues its vector gathers and, between them,
//                      S scalar ones (S = 8 per 8 vector instructions)
// Reports gathers per second (a vector instruction counts 64, a scalar load 1).
//   hipcc --offload-arch=gfx950 -O3 exp_sgather.hip -o exp_sgather && ./exp_sgather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__device__ __forceinline__ unsigned hash32(unsigned a)
{
    a ^= a >> 16; a *= 0x7feb352dU; a ^= a >> 15; a *= 0x846ca68bU; a ^= a >> 16;
    return a;
}

template <int kMode>
__global__ __launch_bounds__(256) void k_gather(const double *__restrict__ x, int n, int iters,
                                                double *__restrict__ out)
{
    const int W = n / 8;
    const int base = (int)(blockIdx.x % 8) * W;
    const unsigned lane = threadIdx.x & 63;
    const unsigned wave = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u + (threadIdx.x >> 6)));
    double s = 0.0;
    for (int it = 0; it < iters; ++it) {
        double v[8];
        double sv[8];
        if (kMode != 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned h = hash32((wave * 977u + (unsigned)it) * 8u + (unsigned)k + lane * 0x9E3779B9u);
                v[k] = x[base + (int)(h % (unsigned)W)];
            }
        }
        if (kMode != 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const unsigned h = __builtin_amdgcn_readfirstlane(hash32((wave * 131u + (unsigned)it) * 8u + (unsigned)k));
                sv[k] = x[base + (int)(h % (unsigned)W)];  // uniform address: s_load_dwordx2
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (kMode != 1) s += v[k];
            if (kMode != 0) s += sv[k];
        }
    }
    if (s == 12345.678) out[threadIdx.x] = s;  // keep the loads
}

int main()
{
    const int n = 2 << 20;  // 16 MiB of x
    double *x = nullptr, *out = nullptr;
    CK(hipMalloc(&x, sizeof(double) * n));
    CK(hipMalloc(&out, sizeof(double) * 256));
    CK(hipMemset(x, 0, sizeof(double) * n));
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int iters = 256;
    for (int wgs_per_cu = 2; wgs_per_cu <= 8; wgs_per_cu *= 2) {
        const int grid = ncu * wgs_per_cu;
        for (int mode = 0; mode < 3; ++mode) {
            auto kern = mode == 0 ? k_gather<0> : mode == 1 ? k_gather<1> : k_gather<2>;
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, x, n, iters, out);  // warm
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, x, n, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double waves = (double)grid * 4 * 5;
            const double vec = mode != 1 ? waves * iters * 8 * 64 : 0;
            const double sca = mode != 0 ? waves * iters * 8 : 0;
            printf("wg/cu %d mode %d  %.1f us/launch  vector %.1f G/s  scalar %.2f G/s  total %.1f G/s\n", wgs_per_cu,
                   mode, ms * 1e3 / 5, vec / (ms * 1e-3) / 1e9, sca / (ms * 1e-3) / 1e9,
                   (vec + sca) / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
