// Experiment (not product code): the one-way store -> poll latency between two
// workgroups, the "hop" that bounds the sync-free SpTRSV.
// Workgroup A (block 0) and workgroup B (block `peer`) ping-pong a counter
// `iters` times: A stores 2i+1 into B's word and waits for 2i+2 in its own, B
// answers.  One-way latency = elapsed / (2 iters).  block `peer` sits on XCD
// peer % 8 (round-robin dispatch; checked with the XCC_ID register), so peer
// = 1 crosses XCDs and peer = 8 stays on XCD 0.  Memory: 0 hipMalloc, 1
// fine-grained (hipDeviceMallocFinegrained), 2 uncached
// (hipDeviceMallocUncached).  Scope: 0 agent, 1 system.  Every spin is bounded.
//
//   hipcc --offload-arch=gfx950 -O3 exp_hop.hip -o exp_hop && ./exp_hop
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr unsigned kSpin = 1u << 20;

__device__ inline int xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7; }

template <int kScope>
__device__ inline void put(unsigned *p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, kScope); }
template <int kScope>
__device__ inline unsigned get(unsigned *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, kScope); }

// Background load (k_hop_bg): blocks other than the pair poll pseudo-random
// 8-B words of a 64 MiB array with agent-scope loads (one outstanding load
// per lane, like a pending SpTRSV lane) until the pair sets the stop word.
template <int kScope>
__global__ void k_hop(unsigned *w, int peer, int iters, unsigned long long *out,
                      const unsigned long long *bgarr, int bg_lanes) {
    const int b = blockIdx.x;
    if (b != 0 && b != peer) {
        if (b > peer && (int)((b - peer - 1) * blockDim.x + threadIdx.x) < bg_lanes) {
            unsigned h = (b * 2654435761u) ^ (threadIdx.x * 40503u);
            unsigned long long acc = 0;
            for (unsigned s = 0; s < (1u << 22); ++s) {
                h = h * 1664525u + 1013904223u;
                acc += __hip_atomic_load(bgarr + (h >> 9), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((s & 63) == 0 && __hip_atomic_load(w + 128, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            }
            if (acc == 42) out[7] = acc;  // keep the loads
        }
        return;
    }
    if (threadIdx.x != 0) return;
    unsigned *mine = w + (b == 0 ? 0 : 64), *other = w + (b == 0 ? 64 : 0);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned bad = 0;
    for (int i = 0; i < iters && !bad; ++i) {
        const unsigned ping = 2u * i + 1, pong = 2u * i + 2;
        if (b == 0) {
            put<kScope>(other, ping);
            unsigned s = 0;
            while (get<kScope>(mine) != pong && ++s < kSpin) {}
            bad = s >= kSpin;
        } else {
            unsigned s = 0;
            while (get<kScope>(mine) != ping && ++s < kSpin) {}
            bad = s >= kSpin;
            put<kScope>(other, pong);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(w + 128, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // stop the pollers
    const int slot = b == 0 ? 0 : 1;
    out[slot * 4 + 0] = t1 - t0;
    out[slot * 4 + 1] = (unsigned long long)xcc_id();
    out[slot * 4 + 2] = bad;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    unsigned long long *out, *bgarr;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&bgarr, 64 << 20));
    CK(hipMemset(bgarr, 0, 64 << 20));
    const char *mem_names[3] = {"hipMalloc", "finegrained", "uncached"};
    for (int mem = 0; mem < 3; ++mem) {
        unsigned *w;
        if (mem == 0) CK(hipMalloc(&w, 4096));
        else CK(hipExtMallocWithFlags((void **)&w, 4096, mem == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
        for (int scope = 0; scope < 2; ++scope)
            for (int peer : {1, 8, 4})
                for (int bg : {0, 8192, 32768, 65536}) {
                    if (bg && (mem != 0 || scope != 0 || peer != 1)) continue;
                    unsigned long long h[8] = {};
                    CK(hipMemset(w, 0, 4096));
                    CK(hipMemset(out, 0, 64));
                    // pair + pollers, 256-thread blocks: <= 2 x 256 CUs x 4 waves, all resident
                    const int blocks = peer + 1 + (bg + 255) / 256;
                    if (scope == 0) hipLaunchKernelGGL(k_hop<__HIP_MEMORY_SCOPE_AGENT>, dim3(blocks), dim3(bg ? 256 : 64), 0, 0, w, peer, iters, out, bgarr, bg);
                    else hipLaunchKernelGGL(k_hop<__HIP_MEMORY_SCOPE_SYSTEM>, dim3(blocks), dim3(64), 0, 0, w, peer, iters, out, bgarr, bg);
                    CK(hipGetLastError());
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(h, out, 64, hipMemcpyDeviceToHost));
                    // s_memrealtime runs at 100 MHz: 10 ns a tick
                    const double ns = 10.0 * (double)h[0] / (2.0 * iters);
                    printf("mem %-11s scope %-6s peer %d (xcd %llu -> %llu) pollers %5d: one-way %.0f ns%s\n", mem_names[mem],
                           scope ? "system" : "agent", peer, h[1], h[5], bg, ns, (h[2] || h[6]) ? "  TIMEOUT" : "");
                }
        CK(hipFree(w));
    }
    CK(hipFree(bgarr));
    CK(hipFree(out));
    return 0;
}
