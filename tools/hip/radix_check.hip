// Standalone check of radix_sort2 (prim.hpp, one kernel per pass) against a
// host stable sort, for sizes around the tile edges, plus the gw_event output.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>
#include "../../goworld_amd/csrc/dev_common.hpp"
using namespace gw;
int main() {
    const uint64_t sizes[] = {1, 7, 100, 4095, 4096, 4097, 12289, 100000, 3700000};
    long bad = 0;
    srand(7);
    for (uint64_t n : sizes) {
        for (int bits : {11, 21, 25}) {
            std::vector<uint32_t> k(n), v(n);
            for (uint64_t i = 0; i < n; ++i) {
                k[i] = ((uint32_t)rand() ^ ((uint32_t)rand() << 15)) & ((1u << bits) - 1);
                if (i % 5 == 0 && i) k[i] = k[i - 1];          // runs of equal keys (stability)
                v[i] = (uint32_t)i;
            }
            const uint64_t cap = n + 5000;                     // n_max above n: the device count decides
            uint32_t *k0, *v0, *k1, *v1, *scr;
            gw_event* aos;
            unsigned long long* nd;
            hipMalloc(&k0, cap * 4); hipMalloc(&v0, cap * 4); hipMalloc(&k1, cap * 4); hipMalloc(&v1, cap * 4);
            hipMalloc(&aos, cap * 8);
            hipMalloc(&scr, radix2_scratch_words(cap) * 4 + 64);
            hipMalloc(&nd, 8);
            hipMemcpy(k0, k.data(), n * 4, hipMemcpyHostToDevice);
            hipMemcpy(v0, v.data(), n * 4, hipMemcpyHostToDevice);
            unsigned long long nn = n;
            hipMemcpy(nd, &nn, 8, hipMemcpyHostToDevice);
            radix_sort2(k0, v0, k1, v1, cap, (const uint64_t*)nd, 0, bits, scr, 0, aos, (1u << (bits - 1)) - 1);
            hipDeviceSynchronize();
            std::vector<gw_event> got(n);
            hipMemcpy(got.data(), aos, n * 8, hipMemcpyDeviceToHost);
            std::vector<uint32_t> idx(n);
            std::iota(idx.begin(), idx.end(), 0u);
            std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return k[a] < k[b]; });
            long b0 = 0;
            for (uint64_t i = 0; i < n; ++i)
                if (got[i].watcher != (k[idx[i]] & ((1u << (bits - 1)) - 1)) || got[i].target != v[idx[i]]) ++b0;
            if (b0) printf("n=%lu bits=%d: %ld mismatches (first: got %u/%u want %u/%u)\n", (unsigned long)n, bits, b0,
                           got[0].watcher, got[0].target, k[idx[0]], v[idx[0]]);
            bad += b0;
            hipFree(k0); hipFree(v0); hipFree(k1); hipFree(v1); hipFree(aos); hipFree(scr); hipFree(nd);
        }
    }
    printf("radix_check: %ld mismatches\n", bad);
    return bad != 0;
}
