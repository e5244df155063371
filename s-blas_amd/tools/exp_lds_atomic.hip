// exp_lds_atomic -- calibration of ds_add_f64 (no return) throughput on
// gfx950 per address pattern (SpMM tall tile).  One 1024-thread
// workgroup per CU, 128 KiB LDS array of doubles, every wave issues `iters`
// atomics; patterns (per 16-lane group = the b64 atomic's lane group):
//   0 conflict-free: lane l of a group hits pair (l + t) mod 16 of its row
//   1 random rows (hash of lane, wave, iteration) -- the tall tile's case
//   2 C-tile shape: 8 lanes x contiguous doubles of one row, two rows of
//     opposite parity per 16-lane group, row stride 17 doubles
//   3 all lanes of a group on ONE address (worst case)
//   4 random rows, one ds_read_b64 + v_add + ds_write_b64 (owned, non-atomic)
//   hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics exp_lds_atomic.hip -o /tmp/exp_lds_atomic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kN = 16384;  // doubles (128 KiB)

__device__ __forceinline__ unsigned hash3(unsigned a, unsigned b, unsigned c)
{
    unsigned h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

template <int kPat>
__global__ __launch_bounds__(1024) void k_lds(int iters, double *out)
{
    __shared__ double a[kN];
    for (int i = threadIdx.x; i < kN; i += 1024) a[i] = 0.0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, l = lane & 15;
    const double v = 1.0 + lane;
    for (int t = 0; t < iters; ++t) {
        int idx;
        if (kPat == 0) idx = ((hash3(wv, g, t) % 1000) * 16 + ((l + t) & 15)) % kN;
        else if (kPat == 1 || kPat == 4) idx = hash3(lane, wv, t) % kN;
        else if (kPat == 2) {
            const int row = (int)((hash3(wv, g, t) % 480) * 2 + (l >> 3));  // two rows, opposite parity
            idx = row * 17 + 2 * (l & 7);
        } else idx = (int)(hash3(wv, g, t) % kN);
        if (kPat == 4) a[idx] = a[idx] + v;
        else atomicAdd(&a[idx], v);
    }
    __syncthreads();
    double s = 0.0;
    for (int i = threadIdx.x; i < kN; i += 1024) s += a[i];
    if (s == 12345.678) out[blockIdx.x] = s;  // keep the work
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    double *out;
    hipMalloc(&out, sizeof(double) * ncu);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, const char *name) {
        hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 0, 0, iters, out);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(ncu), dim3(1024), 0, 0, iters, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double ops = (double)ncu * 16 * iters;  // wave-instructions
        printf("%-34s %8.3f ms  %6.2f ns per wave-instr per CU  (%.2f cycles at 2.1 GHz)\n", name, ms,
               ms * 1e6 / (ops / ncu), ms * 1e6 / (ops / ncu) * 2.1);
    };
    run(k_lds<0>, "0 conflict-free pairs");
    run(k_lds<1>, "1 random rows");
    run(k_lds<2>, "2 C-tile (8 contiguous x 2 rows)");
    run(k_lds<3>, "3 one address per 16 lanes");
    run(k_lds<4>, "4 random, read+add+write (racy)");
    return 0;
}
