// Read-traffic calibration probe: what FETCH_SIZE and
// TCC_EA0_RDREQ report for k_mover_c's access pattern, against a known byte
// count.  k_mover_c reads 16-B grid entries (gn) and 32-B mover-grid entries
// (gm, two 16-B words) in short contiguous runs (a window's row ranges), one
// entry per lane, at arbitrary 16-B offsets.  MI355X_MICROARCH.md validates the
// x2 FETCH_SIZE correction only for wide coalesced streaming reads; this probe
// measures the same counters for:
//   g_stream       16 B per lane, fully coalesced (the guide's calibrated case)
//   g_runs<R>      runs of R consecutive 16-B entries at random 16-B offsets,
//                  R lanes of a wave per run (R = 8, 16, 32, 64)
//   g_runs32<R>    runs of R consecutive 32-B entries, two 16-B loads per lane
// over a 2 GiB table (well past the 256 MiB Infinity Cache), 256 MiB of payload
// per kernel.  Prints bytes and time per kernel; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./gather
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -- ./gather
// build: hipcc -O3 --offload-arch=gfx950 -o gather gather.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ void g_stream(const uint4* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x9e3779b9u) out[0] = s;
}

// each wave handles `iters` runs of R entries (16 B) starting at random entries
template <int R>
__global__ void g_runs(const uint4* __restrict__ a, size_t n, uint32_t iters, uint32_t* out) {
    const uint32_t ln = threadIdx.x & 63;
    const uint64_t wv = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    uint32_t s = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint64_t st = mix(wv * 1000003ull + it) % (n - 64);
#pragma unroll
        for (int k = 0; k < 64 / R; ++k) {             // 64 / R runs per 64 lanes, like a chunk over several rows
            const uint64_t st2 = k ? mix(st + k) % (n - 64) : st;
            if (ln / R == (uint32_t)k) {
                const uint4 v = a[st2 + (ln % R)];
                s += v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (s == 0x9e3779b9u) out[0] = s;
}

// the same with 32-B entries, read as two 16-B words per lane
template <int R>
__global__ void g_runs32(const uint4* __restrict__ a, size_t n32, uint32_t iters, uint32_t* out) {
    const uint32_t ln = threadIdx.x & 63;
    const uint64_t wv = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    uint32_t s = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint64_t st = mix(wv * 7000003ull + it) % (n32 - 64);
#pragma unroll
        for (int k = 0; k < 64 / R; ++k) {
            const uint64_t st2 = k ? mix(st + k) % (n32 - 64) : st;
            if (ln / R == (uint32_t)k) {
                const uint4* p = a + 2 * (st2 + (ln % R));
                const uint4 v = p[0], w = p[1];
                s += v.x ^ v.y ^ w.z ^ w.w;
            }
        }
    }
    if (s == 0x9e3779b9u) out[0] = s;
}

template <typename K>
static int timed(const char* name, K launch, double bytes) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();                                            // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-14s bytes/launch %.1f MB  %.1f us  %.2f TB/s\n", name, bytes / 1e6, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    return 0;
}

int main() {
    const size_t N = (2ull << 30) / 16;                 // 2 GiB of 16-B entries
    uint4* a = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&a, N * 16));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(a, 1, N * 16));
    const double payload = 256.0 * (1 << 20);
    const size_t n_stream = (size_t)(payload / 16);
    const uint32_t threads = 256, iters = 16;
    // waves * iters * 64 lanes * 16 B = payload
    const uint32_t waves16 = (uint32_t)(payload / (64.0 * 16 * iters));
    const uint32_t waves32 = (uint32_t)(payload / (64.0 * 32 * iters));
    printf("table %.1f GiB, payload %.0f MB per kernel\n", N * 16.0 / (1 << 30), payload / 1e6);
    if (timed("g_stream", [&] { hipLaunchKernelGGL(g_stream, dim3(8192), dim3(threads), 0, 0, a, n_stream, out); },
              payload))
        return 1;
#define RUNS(R)                                                                                          \
    if (timed("g_runs<" #R ">", [&] {                                                                    \
            hipLaunchKernelGGL(g_runs<R>, dim3(waves16 * 64 / threads), dim3(threads), 0, 0, a, N, iters, out); \
        }, payload)) return 1;                                                                           \
    if (timed("g_runs32<" #R ">", [&] {                                                                  \
            hipLaunchKernelGGL(g_runs32<R>, dim3(waves32 * 64 / threads), dim3(threads), 0, 0, a, N / 2, iters, out); \
        }, payload)) return 1;
    RUNS(8)
    RUNS(16)
    RUNS(32)
    RUNS(64)
    CK(hipDeviceSynchronize());
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
