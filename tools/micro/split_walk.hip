// Why splitting one heavy walk over several one-wave blocks was 8-13x slower
// (DESIGN.md §4, round 4): each part wrote its slice of the entry's 4-B events
// with agent-scope stores (the parts sit on different XCDs, whose L2s are not
// coherent), bumped a per-entry completion counter, and the last part gathered
// the slices.  This probe times the pieces of that protocol on their own:
//   plain      every wave stores its slice with plain dword stores (the one-wave walk)
//   agent      the same stores at agent scope (what the split walk used)
//   plain+rel  plain stores, one agent release fence per wave, then the counter add;
//              the last part of an entry reads the entry back (acquire) -- the
//              protocol the guide prescribes for a cross-XCD hand-off
//   agent+cnt  agent-scope stores, the counter add, the last part reads back
// for P = 1, 2, 4 parts per entry (P consecutive blocks: dealt round-robin over
// the XCDs, so the parts of an entry sit on different XCDs).
// build: hipcc -O3 --offload-arch=gfx950 -o split_walk split_walk.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

enum Mode { PLAIN = 0, AGENT = 1, PLAIN_REL = 2, AGENT_CNT = 3 };

// entry e = blockIdx.x / P, part q = blockIdx.x % P; the entry's S dwords,
// part q writes [q*S/P, (q+1)*S/P) in 64-dword chunks (one wave per block)
template <int MODE>
__global__ void __launch_bounds__(64) k_parts(uint32_t* __restrict__ ev, uint32_t* __restrict__ cnt,
                                              uint32_t* __restrict__ sink, uint32_t S, uint32_t P) {
    const uint32_t e = blockIdx.x / P, q = blockIdx.x % P;
    const uint32_t lo = q * (S / P), hi = lo + S / P;
    uint32_t* r = ev + (size_t)e * S;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += 64) {
        const uint32_t v = e * 2654435761u + i;
        if (MODE == AGENT || MODE == AGENT_CNT)
            __hip_atomic_store(r + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            r[i] = v;
    }
    if (MODE == PLAIN || MODE == AGENT) return;
    if (MODE == PLAIN_REL) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    uint32_t last = 0;
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(cnt + e, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == P - 1 ? 1u : 0u;
    last = __shfl(last, 0, 64);
    if (!last) return;
    if (MODE == PLAIN_REL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    uint32_t acc = 0;                                   // the gather: the whole entry, read back
    for (uint32_t i = threadIdx.x; i < S; i += 64)
        acc += __hip_atomic_load(r + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (acc == 0xdeadbeefu) sink[e] = acc;              // keeps the loads
}

template <int MODE>
static float run(uint32_t* ev, uint32_t* cnt, uint32_t* sink, uint32_t E, uint32_t S, uint32_t P) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemset(cnt, 0, (size_t)E * 4));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_parts<MODE>, dim3(E * P), dim3(64), 0, 0, ev, cnt, sink, S, P);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep) best = ms < best ? ms : best;          // the first run warms up
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return best * 1000.0f;
}

int main() {
    // entries like the strip diff's heavy walks: 4096 entries x 2048 events
    const uint32_t E = 4096, S = 2048;
    uint32_t *ev, *cnt, *sink;
    CK(hipMalloc(&ev, (size_t)E * S * 4));
    CK(hipMalloc(&cnt, (size_t)E * 4));
    CK(hipMalloc(&sink, (size_t)E * 4));
    printf("entries %u x %u dwords (%.1f MB)\n", E, S, E * S * 4 / 1e6);
    for (uint32_t P : {1u, 2u, 4u}) {
        const float t0 = run<PLAIN>(ev, cnt, sink, E, S, P);
        const float t1 = run<AGENT>(ev, cnt, sink, E, S, P);
        const float t2 = run<PLAIN_REL>(ev, cnt, sink, E, S, P);
        const float t3 = run<AGENT_CNT>(ev, cnt, sink, E, S, P);
        printf("P=%u  plain %8.1f us  agent %8.1f us  plain+rel+cnt+gather %8.1f us  agent+cnt+gather %8.1f us\n", P,
               t0, t1, t2, t3);
    }
    CK(hipFree(ev));
    CK(hipFree(cnt));
    CK(hipFree(sink));
    return 0;
}
