// exp_stream.hip -- microbenchmark: how long does a COLD streaming read of
// B bytes take on MI355X, as a function of B?  This is the floor for a
// per-rank SpMV slice at N ranks: the slice's algorithmic bytes
// cannot be read faster than this, whatever the kernel.
//
// Before each timed launch a 1 GiB read sweep evicts the Infinity Cache and
// the L2s (as bench.py's cold steps).  The timed kernel reads the buffer with
// 16-B nontemporal loads, 4 in flight per thread, one grid of `wgs`
// 256-thread workgroups striding over the buffer, and writes one value per
// workgroup (so nothing is optimised away).  The span is taken by
// hipExtLaunchKernelGGL's start/stop events (kernel start .. kernel end).
//   hipcc --offload-arch=gfx950 -O3 exp_stream.hip -o exp_stream && ./exp_stream
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const v2d *__restrict__ p, long long n16, double *out)
{
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    double s = 0.0;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const v2d a = __builtin_nontemporal_load(p + i);
        const v2d b = __builtin_nontemporal_load(p + i + stride);
        const v2d c = __builtin_nontemporal_load(p + i + 2 * stride);
        const v2d d = __builtin_nontemporal_load(p + i + 3 * stride);
        s += a.x + a.y + b.x + b.y + c.x + c.y + d.x + d.y;
    }
    for (; i < n16; i += stride) {
        const v2d a = __builtin_nontemporal_load(p + i);
        s += a.x + a.y;
    }
    if (s == 12345.678) out[blockIdx.x] = s;  // practically never; keeps the loads
}

__global__ void k_sweep(const double *__restrict__ p, long long n, double *out)
{
    double s = 0.0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        s += p[i];
    if (s == 12345.678) out[0] = s;
}

int main(int argc, char **argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 8;
    const long long sweep_n = (1LL << 30) / 8;
    double *sweep = nullptr, *buf = nullptr, *out = nullptr;
    const long long max_bytes = 512LL << 20;
    CK(hipMalloc(&sweep, sweep_n * 8));
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(sweep, 0, sweep_n * 8));
    CK(hipMemset(buf, 0, max_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const long long sizes_mb[] = {8, 16, 32, 48, 67, 81, 128, 145, 256, 512};
    const int wgs_list[] = {1024, 2048, 4096};
    printf("{\"probe\": \"cold streaming read, 1 GiB read sweep before each launch\", \"rows\": [\n");
    bool first = true;
    for (long long mb : sizes_mb) {
        const long long bytes = mb << 20;
        for (int wgs : wgs_list) {
            std::vector<float> ms;
            for (int r = 0; r < reps + 2; ++r) {
                hipLaunchKernelGGL(k_sweep, dim3(4096), dim3(256), 0, 0, sweep, sweep_n, out);
                CK(hipDeviceSynchronize());
                hipExtLaunchKernelGGL(k_read, dim3(wgs), dim3(256), 0, 0, e0, e1, 0,
                                      (const v2d *)buf, bytes / 16, out);
                CK(hipGetLastError());
                CK(hipEventSynchronize(e1));
                float t = 0.f;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (r >= 2) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const double med = ms[ms.size() / 2] * 1e3;
            printf("%s  {\"MiB\": %lld, \"workgroups\": %d, \"us_median\": %.1f, \"us_min\": %.1f, \"GBps\": %.0f}",
                   first ? "" : ",\n", mb, wgs, med, ms[0] * 1e3, bytes / med / 1e3);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
