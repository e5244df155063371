// spf.hip -- experiment: does a scalar-path (SQC) prefetch of a stream into
// L2 shorten a vector stream that is bound by vector-L1 miss capacity?
// Workgroup b reads its own contiguous span with 4 vector waves (2 x 16-B
// loads per lane in flight, like xsort's entry stream); with kPf a fifth
// wave touches the span's lines with scalar loads up to `dist` bytes ahead of
// the vector front (an LDS counter).  Modes: 0 vector only, 1 vector + scalar
// prefetch, 2 scalar touch only (bytes covered / time).
// Build: hipcc --offload-arch=gfx950 -O3 exp_spf.hip -o exp_spf ; run: ./exp_spf
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((address_space(4))) const unsigned cu32;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int kMode>
__global__ __launch_bounds__(320) void k_spf(const v4u *__restrict__ src, long long n16, long long dist16,
                                             int pstep16, unsigned long long *sink)
{
    __shared__ long long s_front;
    const long long span = (n16 + gridDim.x - 1) / gridDim.x;
    const long long b0 = (long long)blockIdx.x * span;
    const long long end = std::min(n16, b0 + span);
    if (threadIdx.x == 0) s_front = kMode == 2 ? end : b0;
    __syncthreads();
    if (threadIdx.x >= 256) {
        if (kMode == 0) return;
        long long pf = b0;
        cu32 *p = (cu32 *)(unsigned long long)src;
        unsigned acc = 0;
        while (pf < end) {
            const long long front =
                (long long)__builtin_amdgcn_readfirstlane(
                    (int)(__hip_atomic_load(&s_front, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) - b0)) + b0;
            const long long tgt = std::min(end, front + dist16);
            if (pf >= tgt) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            unsigned v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = p[std::min(pf + (long long)u * pstep16, end - 1) * 4];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc ^= v[u];
            pf += 16LL * pstep16;
        }
        if (acc == 0x5bd1e995u) sink[1] = acc;
        return;
    }
    if (kMode == 2) return;
    unsigned long long acc = 0;
    long long i = b0 + threadIdx.x;
    for (; i + 256 < end; i += 512) {
        const v4u a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + 256);
        acc ^= (unsigned long long)(a.x ^ a.y ^ b.x ^ b.y) << 32 | (a.z ^ a.w ^ b.z ^ b.w);
        if (threadIdx.x == 0) __hip_atomic_store(&s_front, i + 512, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (acc == 0x5bd1e9955bd1e995ULL) sink[0] = acc;
}

int main(int argc, char **argv)
{
    const long long bytes = 4LL << 30, n16 = bytes / 16;
    v4u *src;
    unsigned long long *sink;
    if (hipMalloc(&src, bytes) != hipSuccess || hipMalloc(&sink, 16) != hipSuccess) return 1;
    (void)hipMemset(src, 1, bytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](int mode, int wgpc, long long distB, int pstepB) {
        std::vector<float> t;
        for (int r = 0; r < 5; ++r) {
            const int grid = cus * wgpc;
            const int thr = mode == 0 ? 256 : 320;
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k_spf<0>, dim3(grid), dim3(thr), 0, 0, src, n16, distB / 16, pstepB / 16, sink);
            else if (mode == 1) hipLaunchKernelGGL(k_spf<1>, dim3(grid), dim3(thr), 0, 0, src, n16, distB / 16, pstepB / 16, sink);
            else hipLaunchKernelGGL(k_spf<2>, dim3(grid), dim3(thr), 0, 0, src, n16, distB / 16, pstepB / 16, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("{\"mode\": %d, \"wg_per_cu\": %d, \"dist_B\": %lld, \"pstep_B\": %d, \"ms\": %.3f, \"GBps\": %.0f}\n", mode, wgpc,
               distB, pstepB, t[2], bytes / (t[2] * 1e-3) / 1e9);
        fflush(stdout);
    };
    if (hipGetLastError() != hipSuccess) return 1;
    for (int w : {1, 2, 4}) {
        run(0, w, 0, 64);
        for (long long d : {8192LL, 32768LL, 131072LL}) {
            run(1, w, d, 64);
            run(1, w, d, 128);
        }
    }
    for (int w : {1, 2, 4, 8}) {
        run(2, w, 0, 64);
        run(2, w, 0, 128);
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
