// PCIe probe: how fast device -> host copies of the collect's output sizes
// land in host memory on this box (the ceiling of the end-to-end tick, whose
// events, records and wire packets cross PCIe), by host buffer kind and by the
// number of streams a copy is split over.
// build: hipcc -O3 --offload-arch=gfx950 -o pcie pcie.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static double run(void* dst, void* src, size_t bytes, int nstreams, hipStream_t* st, bool d2h, int reps) {
    const size_t chunk = (bytes / nstreams + 4095) & ~(size_t)4095;
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < nstreams; ++k) {
            const size_t off = k * chunk;
            if (off >= bytes) break;
            const size_t n = std::min(chunk, bytes - off);
            CK(hipMemcpyAsync((char*)dst + off, (char*)src + off, n, d2h ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice,
                              st[k]));
        }
        for (int k = 0; k < nstreams; ++k) CK(hipStreamSynchronize(st[k]));
        auto t1 = std::chrono::steady_clock::now();
        best = std::min(best, std::chrono::duration<double>(t1 - t0).count());
    }
    return bytes / best / 1e9;
}

int main(int argc, char** argv) {
    const size_t sizes[] = {30ull << 20, 350ull << 20, 700ull << 20};
    void* dev;
    CK(hipMalloc(&dev, 700ull << 20));
    CK(hipMemset(dev, 1, 700ull << 20));
    hipStream_t st[8];
    for (int k = 0; k < 8; ++k) CK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
    struct Kind { const char* name; unsigned flags; int reg; } kinds[] = {
        {"hipHostMalloc default", hipHostMallocDefault, 0},
        {"hipHostMalloc noncoherent", hipHostMallocNonCoherent, 0},
        {"hipHostMalloc coherent", hipHostMallocCoherent, 0},
        {"malloc + hipHostRegister", 0, 1},
        {"malloc (pageable)", 0, 2},
    };
    for (auto& kd : kinds) {
        void* h = nullptr;
        if (kd.reg == 0) CK(hipHostMalloc(&h, 700ull << 20, kd.flags));
        else {
            h = aligned_alloc(4096, 700ull << 20);
            memset(h, 0, 700ull << 20);
            if (kd.reg == 1) CK(hipHostRegister(h, 700ull << 20, hipHostRegisterDefault));
        }
        for (size_t b : sizes)
            for (int ns : {1, 2, 4}) {
                const double d2h = run(h, dev, b, ns, st, true, 3);
                const double h2d = run(dev, h, b, ns, st, false, 3);
                printf("%-28s %5zu MB  streams %d  D2H %6.1f GB/s  H2D %6.1f GB/s\n", kd.name, b >> 20, ns, d2h, h2d);
                fflush(stdout);
            }
        if (kd.reg == 0) CK(hipHostFree(h));
        else {
            if (kd.reg == 1) CK(hipHostUnregister(h));
            free(h);
        }
    }
    // allocation cost of a pinned buffer of the wire size
    auto t0 = std::chrono::steady_clock::now();
    void* h2;
    CK(hipHostMalloc(&h2, 700ull << 20, hipHostMallocDefault));
    auto t1 = std::chrono::steady_clock::now();
    CK(hipHostFree(h2));
    auto t2 = std::chrono::steady_clock::now();
    printf("hipHostMalloc 700 MB: %.1f ms, hipHostFree: %.1f ms\n",
           std::chrono::duration<double, std::milli>(t1 - t0).count(),
           std::chrono::duration<double, std::milli>(t2 - t1).count());
    return 0;
}
