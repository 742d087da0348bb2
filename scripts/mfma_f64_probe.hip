// mfma_f64_probe.hip -- diagnostic for the FP64 MFMA co-issue idea:
//   1. operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 (one-hot A experiments)
//   2. issue cost of that MFMA, of v_fma_f64, and of a mix of both in one wave (do they overlap?)
// build: hipcc --offload-arch=gfx950 -O3 scripts/mfma_f64_probe.hip -o build/mfma_f64_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void k_layout(const double *a, const double *b, double *d) {
    const int l = threadIdx.x;
    d[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 0, 0, 0);
}

template <int MF, int VA>  // MF mfma chains (4 accumulators each step), VA independent FMA chains x 8
__global__ __launch_bounds__(256) void k_rate(int iters, double *out, double s) {
    const int l = threadIdx.x;
    double acc[4] = {l * 1e-3, l * 2e-3, l * 3e-3, l * 4e-3};
    double v[8];
    for (int k = 0; k < 8; ++k) v[k] = l * 1e-4 + k;
    const double a = 1.0 + l * 1e-9, b = 0.999;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < MF; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < VA; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fma(v[k], s, 1e-7);
    }
    double t = acc[0] + acc[1] + acc[2] + acc[3];
    for (int k = 0; k < 8; ++k) t += v[k];
    out[blockIdx.x * 256 + l] = t;
}

template <int MF, int VA>
static float run(int iters, double *out, hipEvent_t e0, hipEvent_t e1) {
    const int blocks = 1024;  // 4,096 waves: 4 per SIMD
    hipLaunchKernelGGL((k_rate<MF, VA>), dim3(blocks), dim3(256), 0, 0, iters, out, 0.9999999);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_rate<MF, VA>), dim3(blocks), dim3(256), 0, 0, iters, out, 0.9999999);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    double *a, *b, *d, *out;
    CK(hipMallocManaged(&a, 64 * 8));
    CK(hipMallocManaged(&b, 64 * 8));
    CK(hipMallocManaged(&d, 64 * 8));
    CK(hipMalloc(&out, 1024 * 256 * 8));
    // 1. layout: A one-hot at lane La, B[lane] = 100 + lane; the nonzero D lanes show the row / block
    //    of La and their values name the B lanes of La's k index
    for (int La = 0; La < 64; La += 1) {
        for (int l = 0; l < 64; ++l) {
            a[l] = (l == La) ? 1.0 : 0.0;
            b[l] = 100 + l;
        }
        hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, a, b, d);
        CK(hipDeviceSynchronize());
        std::printf("A@%2d:", La);
        for (int l = 0; l < 64; ++l)
            if (d[l] != 0.0) std::printf(" D%d=B%d", l, (int)d[l] - 100);
        std::printf("\n");
    }
    // 2. rates (4 waves per SIMD)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = 2000;
    const double waves = 1024.0 * 4;
    const float t_v = run<0, 4>(it, out, e0, e1);   // 32 FMA per iter
    const float t_m = run<4, 0>(it, out, e0, e1);   // 4 MFMA per iter
    const float t_mv = run<4, 4>(it, out, e0, e1);  // both
    const float t_m2v = run<2, 4>(it, out, e0, e1);
    const float t_m1v = run<1, 4>(it, out, e0, e1);
    const double vinstr = waves * it * 32, minstr = waves * it * 4;
    std::printf("VALU only : %.3f ms  (%.3g wave-FMA/ns)\n", t_v, vinstr / (t_v * 1e6));
    std::printf("MFMA only : %.3f ms  (%.3g wave-MFMA/ns)\n", t_m, minstr / (t_m * 1e6));
    std::printf("4 MFMA + 32 FMA per iter: %.3f ms (sum of alone %.3f, max %.3f)\n", t_mv, t_v + t_m, t_v > t_m ? t_v : t_m);
    std::printf("2 MFMA + 32 FMA per iter: %.3f ms (VALU alone %.3f, MFMA alone would be %.3f)\n", t_m2v, t_v, t_m / 2);
    std::printf("1 MFMA + 32 FMA per iter: %.3f ms (VALU alone %.3f, MFMA alone would be %.3f)\n", t_m1v, t_v, t_m / 4);
    return 0;
}
