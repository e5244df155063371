// Experiment (not product code): store -> poll latency between two
// workgroups with mixed scopes: the producer's store at agent scope (sc1:
// written through past the XCD's L2) or workgroup scope (sc0), the consumer's
// poll at agent scope (sc1: past the L2) or workgroup scope (sc0: misses the
// CU's L1, may hit the XCD's L2).  Peer 8 shares XCD 0 (round-robin dispatch,
// checked with XCC_ID), peer 1 does not.  Every spin is bounded (TIMEOUT is
// printed instead of hanging).
//
//   hipcc --offload-arch=gfx950 -O3 exp_hop2.hip -o exp_hop2 && ./exp_hop2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr unsigned kSpin = 1u << 20;

__device__ inline int xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7; }

template <int kSt, int kLd>
__global__ void k_hop(unsigned *w, int peer, int iters, unsigned long long *out)
{
    const int b = blockIdx.x;
    if ((b != 0 && b != peer) || threadIdx.x != 0) return;
    unsigned *mine = w + (b == 0 ? 0 : 64), *other = w + (b == 0 ? 64 : 0);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned bad = 0;
    for (int i = 0; i < iters && !bad; ++i) {
        const unsigned ping = 2u * i + 1, pong = 2u * i + 2;
        const unsigned want = b == 0 ? pong : ping;
        if (b == 0) __hip_atomic_store(other, ping, __ATOMIC_RELAXED, kSt);
        unsigned s = 0;
        while (__hip_atomic_load(mine, __ATOMIC_RELAXED, kLd) != want && ++s < kSpin) {}
        bad = s >= kSpin;
        if (b != 0) __hip_atomic_store(other, pong, __ATOMIC_RELAXED, kSt);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const int slot = b == 0 ? 0 : 1;
    out[slot * 4 + 0] = t1 - t0;
    out[slot * 4 + 1] = (unsigned long long)xcc_id();
    out[slot * 4 + 2] = bad;
}

template <int kSt, int kLd>
static void run(const char *name, unsigned *w, unsigned long long *out, int iters)
{
    for (int peer : {8, 16, 1, 4}) {
        unsigned long long h[8] = {};
        CK(hipMemset(w, 0, 4096));
        CK(hipMemset(out, 0, 64));
        hipLaunchKernelGGL((k_hop<kSt, kLd>), dim3(peer + 1), dim3(64), 0, 0, w, peer, iters, out);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, 64, hipMemcpyDeviceToHost));
        const double ns = 10.0 * (double)h[0] / (2.0 * iters);  // s_memrealtime: 100 MHz
        printf("%-28s peer %2d (xcd %llu -> %llu): one-way %.0f ns%s\n", name, peer, h[1], h[5], ns,
               (h[2] || h[6]) ? "  TIMEOUT" : "");
    }
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    unsigned long long *out;
    unsigned *w;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&w, 4096));
    run<__HIP_MEMORY_SCOPE_AGENT, __HIP_MEMORY_SCOPE_AGENT>("store agent, poll agent", w, out, iters);
    run<__HIP_MEMORY_SCOPE_AGENT, __HIP_MEMORY_SCOPE_WORKGROUP>("store agent, poll wg", w, out, iters);
    run<__HIP_MEMORY_SCOPE_WORKGROUP, __HIP_MEMORY_SCOPE_WORKGROUP>("store wg, poll wg", w, out, iters);
    run<__HIP_MEMORY_SCOPE_WORKGROUP, __HIP_MEMORY_SCOPE_AGENT>("store wg, poll agent", w, out, iters);
    CK(hipFree(w));
    CK(hipFree(out));
    return 0;
}
