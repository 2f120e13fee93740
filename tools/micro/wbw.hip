// Write-bandwidth probe: how fast HBM absorbs pure streaming writes on this
// part (the ceiling of the record-writing kernels, which only write).
// build: hipcc -O3 --offload-arch=gfx950 -o wbw wbw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void w16(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void w16nt(u32x4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(v, p + i);
    }
}
__global__ void w8nt(unsigned long long* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((unsigned long long)i, p + i);
}
// 24-B records, one 8-B field per store at a 24-B stride (the record writers' pattern)
__global__ void w24(unsigned long long* p, size_t nrec) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec; i += (size_t)gridDim.x * blockDim.x) {
        __builtin_nontemporal_store((unsigned long long)i, p + 3 * i);
        __builtin_nontemporal_store((unsigned long long)i + 1, p + 3 * i + 1);
        __builtin_nontemporal_store((unsigned long long)i + 2, p + 3 * i + 2);
    }
}
__global__ void w24p(unsigned long long* p, size_t nrec) {   // the same, plain stores
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec; i += (size_t)gridDim.x * blockDim.x) {
        p[3 * i] = i;
        p[3 * i + 1] = i + 1;
        p[3 * i + 2] = i + 2;
    }
}
// 24-B records in runs of 35 at random 24-B offsets (one run per half-wave), plain / nt
template <bool NTS>
__global__ void w24runs(unsigned long long* p, size_t nrec) {
    const size_t runs = nrec / 40;
    const uint32_t ln = threadIdx.x & 63u, half = ln >> 5, hl = ln & 31u;
    for (size_t r = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 32; r < runs; r += (size_t)gridDim.x * blockDim.x / 32) {
        const size_t base = r * 40 + (r * 2654435761u) % 5;   // run start, 0..4 records of slack
        for (uint32_t k = hl; k < 35; k += 32) {
            unsigned long long* q = p + 3 * (base + k);
            if (NTS) {
                __builtin_nontemporal_store((unsigned long long)k, q);
                __builtin_nontemporal_store((unsigned long long)r, q + 1);
                __builtin_nontemporal_store((unsigned long long)half, q + 2);
            } else {
                q[0] = k; q[1] = r; q[2] = half;
            }
        }
    }
}
__global__ void r16(const uint4* p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i].x ^ p[i].w;
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = 1ull << 30;
    void* p;
    uint32_t* o;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grid = 256 * 16, blk = 256;
    for (int k = 0; k < 8; ++k) {
        for (int rep = 0; rep < 4; ++rep) {
            (void)hipEventRecord(a);
            if (k == 0) hipLaunchKernelGGL(w16, dim3(grid), dim3(blk), 0, 0, (uint4*)p, bytes / 16);
            if (k == 1) hipLaunchKernelGGL(w16nt, dim3(grid), dim3(blk), 0, 0, (u32x4*)p, bytes / 16);
            if (k == 2) hipLaunchKernelGGL(w8nt, dim3(grid), dim3(blk), 0, 0, (unsigned long long*)p, bytes / 8);
            if (k == 3) hipLaunchKernelGGL(w24, dim3(grid), dim3(blk), 0, 0, (unsigned long long*)p, bytes / 24);
            if (k == 5) hipLaunchKernelGGL(w24p, dim3(grid), dim3(blk), 0, 0, (unsigned long long*)p, bytes / 24);
            if (k == 6) hipLaunchKernelGGL((w24runs<true>), dim3(grid), dim3(blk), 0, 0, (unsigned long long*)p, bytes / 24);
            if (k == 7) hipLaunchKernelGGL((w24runs<false>), dim3(grid), dim3(blk), 0, 0, (unsigned long long*)p, bytes / 24);
            if (k == 4) hipLaunchKernelGGL(r16, dim3(grid), dim3(blk), 0, 0, (const uint4*)p, bytes / 16, o);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            if (rep == 3) {
                const char* nm[] = {"write 16B/lane", "write 16B/lane nt", "write 8B/lane nt", "write 24B rec 3x8B nt", "read 16B/lane", "write 24B rec plain", "24B runs of 35 nt", "24B runs of 35 plain"};
                const double b = k >= 6 ? (double)(bytes / 24 / 40) * 35 * 24 : (double)bytes;
                printf("%-24s %8.1f us  %6.2f TB/s\n", nm[k], ms * 1e3, b / (ms * 1e-3) / 1e12);
            }
        }
    }
    return 0;
}
