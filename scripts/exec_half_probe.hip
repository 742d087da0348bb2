// Does a wave whose exec mask has lanes off issue its FP64 VALU faster?  Each active lane runs 8
// independent v_fma_f64 chains (enough ILP to keep one wave issuing back to back; the loop unrolled by
// 8, so 64 FMAs per branch); lanes >= active
// leave before the loop.  Times, for 1 and 2 waves per SIMD (1,024 / 2,048 waves on 256 CUs):
// active = 64, 32, 16 lanes per wave.  If the SIMD skips idle lane groups, 32 active lanes take
// about half the time of 64; if not, the same time (then two half-waves per SIMD cost twice one full
// wave per filter).  Build: hipcc --offload-arch=gfx950 -O3 scripts/exec_half_probe.hip -o /tmp/ehp
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k_fma(int iters, int active, double *out) {
    const int lane = threadIdx.x & 63;
    if (lane >= active) return;
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = 1.0 + 1e-9 * (threadIdx.x + k);
    const double m = 0.999999999, c = 1e-12;
#pragma unroll 8
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = fma(a[k], m, c);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    const int iters = 200000;
    double *d;
    hipMalloc(&d, 2048 * 64 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_fma, dim3(256), dim3(256), 0, 0, 1000, 64, d);  // warm-up
    hipDeviceSynchronize();
    for (int wps : {1, 2}) {
        for (int active : {64, 32, 16}) {
            const int blocks = 256 * wps;  // 4 waves per block: wps waves per SIMD on 256 CUs
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, iters, active, d);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            // lane-FMAs per second over the whole chip
            const double lane_fma = (double)blocks * 4 * active * 8.0 * iters;
            printf("waves/SIMD %d, active lanes %2d: %8.3f ms, %.3e lane-FMA/s\n",
                   wps, active, best, lane_fma / (best * 1e-3));
        }
    }
    hipFree(d);
    return 0;
}
