// Standalone check of the DPP wave scan (prim.hpp) against a host prefix sum.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../goworld_amd/csrc/dev_common.hpp"
#include <algorithm>
using namespace gw;
__global__ void k(const uint32_t* in, uint32_t* out, unsigned long long* out2) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    out[i] = wave_incl_scan<uint32_t>(in[i]);
    // 64-bit: carries across the halves (inputs scaled past 2^32)
    out2[i] = wave_incl_scan<uint64_t>((uint64_t)in[i] * 0x1234567ull + 0xfffffff0ull);
}
__global__ void ks(const uint32_t* in, uint32_t* out) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    out[i] = wave_sort64(in[i]);
}
int main() {
    const int W = 4096;
    std::vector<uint32_t> h(W * 64), o(W * 64);
    std::vector<unsigned long long> o2(W * 64);
    srand(1);
    for (auto& v : h) v = (rand() % 3 == 0) ? 0 : (uint32_t)(rand() % 100000);
    uint32_t *din, *dout;
    unsigned long long* dout2;
    if (hipMalloc(&din, h.size() * 4) || hipMalloc(&dout, h.size() * 4) || hipMalloc(&dout2, h.size() * 8)) return 2;
    if (hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice)) return 2;
    hipLaunchKernelGGL(k, dim3(W), dim3(64), 0, 0, din, dout, dout2);
    if (hipDeviceSynchronize() || hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost) ||
        hipMemcpy(o2.data(), dout2, o2.size() * 8, hipMemcpyDeviceToHost)) return 2;
    long bad = 0;
    for (int w = 0; w < W; ++w) {
        uint32_t acc = 0;
        unsigned long long acc2 = 0;
        for (int l = 0; l < 64; ++l) {
            acc += h[w * 64 + l];
            acc2 += (unsigned long long)h[w * 64 + l] * 0x1234567ull + 0xfffffff0ull;
            bad += o[w * 64 + l] != acc;
            bad += o2[w * 64 + l] != acc2;
        }
    }
    std::vector<uint32_t> so(W * 64);
    hipLaunchKernelGGL(ks, dim3(W), dim3(64), 0, 0, din, dout);
    if (hipDeviceSynchronize() || hipMemcpy(so.data(), dout, so.size() * 4, hipMemcpyDeviceToHost)) return 2;
    for (int w = 0; w < W; ++w) {
        std::vector<uint32_t> e(h.begin() + w * 64, h.begin() + w * 64 + 64);
        std::sort(e.begin(), e.end());
        for (int l = 0; l < 64; ++l) bad += so[w * 64 + l] != e[l];
    }
    printf("scan_check: %ld mismatches over %d waves (scans, 64-bit scans, wave sort)\n", bad, W);
    return bad ? 1 : 0;
}
