// Which SIMD of its CU each wave of a workgroup lands on (HW_ID register: SIMD_ID bits 5:4,
// CU_ID bits 11:8, SH_ID bit 12, SE_ID bits 15:13), for 2-, 4- and 8-wave workgroups launched with
// as many workgroups as a config-2 run of that block size.  Prints, for the first 4 workgroups, the
// SIMD of each wave, and the histogram of waves per (CU, SIMD) slot.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void k_probe(unsigned *out, int spin) {
    unsigned id = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    if (threadIdx.x % 64 == 0) out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = id;
    // keep the waves resident a while so that the whole grid is placed at once
    long t0 = clock64();
    while (clock64() - t0 < spin) {}
}

int main() {
    const int total_waves = 1024;
    for (int wpb : {2, 4, 8}) {
        const int blocks = total_waves / wpb;
        unsigned *d;
        hipMalloc(&d, total_waves * 4);
        hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(wpb * 64), 0, 0, d, 2000000);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        std::vector<unsigned> h(total_waves);
        hipMemcpy(h.data(), d, total_waves * 4, hipMemcpyDeviceToHost);
        hipFree(d);
        printf("%d-wave blocks, %d blocks:\n", wpb, blocks);
        for (int b = 0; b < 4; ++b) {
            printf("  block %d:", b);
            for (int w = 0; w < wpb; ++w) {
                unsigned id = h[b * wpb + w];
                printf(" w%d->se%u.sh%u.cu%u.simd%u", w, (id >> 13) & 7, (id >> 12) & 1, (id >> 8) & 15, (id >> 4) & 3);
            }
            printf("\n");
        }
        std::map<unsigned, int> slot;  // (xcc-agnostic) se/sh/cu/simd -> waves
        for (unsigned id : h) slot[id & 0xFF30u]++;
        std::map<int, int> hist;
        for (auto &kv : slot) hist[kv.second]++;
        printf("  waves per (se,sh,cu,simd) slot (slots seen %zu; note: XCC id not in HW_ID):", slot.size());
        for (auto &kv : hist) printf(" %d waves: %d slots;", kv.first, kv.second);
        printf("\n");
    }
    return 0;
}
