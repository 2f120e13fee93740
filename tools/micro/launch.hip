// launch.hip — host launch cost of a chain of small dependent kernels on one
// stream (a decomposed-world strip's tick is ~30 kernels of 3-8 us each):
// (a) hipLaunchKernelGGL per kernel, (b) the same chain captured once into a
// hipGraph and replayed, (c) (b) with every node's arguments updated before
// each replay (hipGraphExecKernelNodeSetParams: the tick's arguments change).
// Each kernel has a ~600-byte argument struct (TickBufs-sized) and does a few
// dependent loads.  Prints wall us per chain (host issue + device) and host
// issue us per chain.
// build: hipcc -O2 --offload-arch=gfx950 -o tools/micro/launch tools/micro/launch.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

struct Big {
    unsigned long long* p;
    uint32_t n, k;
    unsigned long long pad[72];
};

__global__ void k_small(unsigned long long* p, uint32_t n, uint32_t k) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned long long v = p[i];
    for (uint32_t j = 0; j < 3; ++j) v = p[(v + j + k) % n];
    p[i] = v + 1;
}

__global__ void k_chain(Big b) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= b.n) return;
    unsigned long long v = b.p[i];
    for (uint32_t j = 0; j < 3; ++j) v = b.p[(v + j + b.k) % b.n];
    b.p[i] = v + 1;
}

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } \
    } while (0)

int main() {
    const int K = 30, REPS = 200;
    const uint32_t N = 1 << 16;
    unsigned long long* p;
    CK(hipMalloc(&p, N * 8));
    CK(hipMemset(p, 0, N * 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Big b{};
    b.p = p;
    b.n = N;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto us = [](auto a, auto z) { return std::chrono::duration<double, std::micro>(z - a).count(); };
    for (uint32_t grid : {64u, 512u}) {
        // (a) individual launches
        for (int w = 0; w < 20; ++w)
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), 0, s, b);
        CK(hipStreamSynchronize(s));
        double issue = 0;
        auto t0 = now();
        for (int r = 0; r < REPS; ++r) {
            auto a = now();
            for (int k = 0; k < K; ++k) {
                b.k = k;
                hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), 0, s, b);
            }
            issue += us(a, now());
            CK(hipStreamSynchronize(s));
        }
        const double wall_a = us(t0, now()) / REPS, issue_a = issue / REPS;
        // (a2) individual launches with a 16-byte argument list
        issue = 0;
        t0 = now();
        for (int r = 0; r < REPS; ++r) {
            auto a = now();
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, p, N, (uint32_t)k);
            issue += us(a, now());
            CK(hipStreamSynchronize(s));
        }
        printf("grid %4u: small-arg launches wall %.1f us (issue %.1f)\n", grid, us(t0, now()) / REPS, issue / REPS);
        // (b) captured graph
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < K; ++k) {
            b.k = k;
            hipLaunchKernelGGL(k_chain, dim3(grid), dim3(256), 0, s, b);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        size_t nn = 0;
        CK(hipGraphGetNodes(g, nullptr, &nn));
        std::vector<hipGraphNode_t> nodes(nn);
        CK(hipGraphGetNodes(g, nodes.data(), &nn));
        for (int w = 0; w < 20; ++w) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        issue = 0;
        t0 = now();
        for (int r = 0; r < REPS; ++r) {
            auto a = now();
            CK(hipGraphLaunch(ge, s));
            issue += us(a, now());
            CK(hipStreamSynchronize(s));
        }
        const double wall_b = us(t0, now()) / REPS, issue_b = issue / REPS;
        // (c) graph with every node's arguments set before each replay
        issue = 0;
        t0 = now();
        for (int r = 0; r < REPS; ++r) {
            auto a = now();
            for (size_t k = 0; k < nn; ++k) {
                hipKernelNodeParams kp{};
                CK(hipGraphKernelNodeGetParams(nodes[k], &kp));
                b.k = (uint32_t)(k + r);
                void* args[] = {&b};
                kp.kernelParams = args;
                CK(hipGraphExecKernelNodeSetParams(ge, nodes[k], &kp));
            }
            CK(hipGraphLaunch(ge, s));
            issue += us(a, now());
            CK(hipStreamSynchronize(s));
        }
        const double wall_c = us(t0, now()) / REPS, issue_c = issue / REPS;
        printf("grid %4u x256, %d kernels: launches wall %.1f us (issue %.1f) | graph wall %.1f us (issue %.1f) | "
               "graph+setparams wall %.1f us (issue %.1f)\n",
               grid, K, wall_a, issue_a, wall_b, issue_b, wall_c, issue_c);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    // device time of one kernel alone
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int k = 0; k < 100; ++k) hipLaunchKernelGGL(k_chain, dim3(512), dim3(256), 0, s, b);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("back-to-back device time per kernel (512 blocks): %.2f us\n", ms * 1000 / 100);
    return 0;
}
