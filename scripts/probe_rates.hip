// probe_rates.hip -- diagnostic: vector issue cost of the instructions the fused kernel's hot
// loop is made of, relative to v_fma_f64, at 4 waves per SIMD (the kernel's occupancy).
// Each lane runs 8 independent chains of one instruction kind (so issue, not latency, binds);
// cost = kernel time / (chains * iterations) normalised by the v_fma_f64 run.
// build: hipcc --offload-arch=gfx950 -O3 scripts/probe_rates.hip -o build/probe_rates
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) (void)(x)

constexpr int kIters = 4096;

#define CHAINS(OP)                                                                  \
    _Pragma("unroll 1") for (int it = 0; it < kIters; ++it) {                      \
        _Pragma("unroll") for (int c = 0; c < 8; ++c) { OP; }                       \
    }

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(double *out, double seed) {
    double v[8];
    float f[8];
    for (int c = 0; c < 8; ++c) {
        v[c] = seed + 0.001 * (threadIdx.x + c);
        f[c] = (float)v[c];
    }
    const double a = 0.999999, b = 1e-7;
    if (KIND == 0) CHAINS(v[c] = fma(v[c], a, b))
    if (KIND == 1) CHAINS(v[c] = __builtin_amdgcn_rsq(v[c]))
    if (KIND == 2) CHAINS(v[c] = __builtin_amdgcn_rcp(v[c]))
    if (KIND == 3) CHAINS(asm volatile("v_cvt_f64_f32 %0, %1" : "+v"(v[c]) : "v"(f[c])))
    if (KIND == 4) CHAINS(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(f[c]) : "v"(f[(c + 1) & 7])))
    if (KIND == 5) CHAINS(v[c] = v[c] * a)
    if (KIND == 6) CHAINS(f[c] = __builtin_amdgcn_rsqf(f[c]))
    if (KIND == 7) CHAINS(asm volatile("v_cvt_f32_f64 %0, %1" : "+v"(f[c]) : "v"(v[c])))
    if (KIND == 8) CHAINS(f[c] = __builtin_amdgcn_rcpf(f[c]))
    if (KIND == 9) CHAINS(f[c] = fmaf(f[c], (float)a, (float)b))
    if (KIND == 10) CHAINS(v[c] = v[c] + a)
    double s = 0;
    for (int c = 0; c < 8; ++c) s += v[c] + f[c];
    if (s == 12345.678) out[threadIdx.x] = s;  // keep the chains alive
}

template <int KIND>
float run(double *out) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = 256 * 4 * 4;  // 4 waves per block -> 16 waves per CU -> 4 per SIMD
    hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1.5);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1.5);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5;
}

int main() {
    double *out;
    CK(hipMalloc(&out, 4096));
    const char *names[] = {"v_fma_f64", "v_rsq_f64", "v_rcp_f64", "v_cvt_f64_f32", "v_cndmask_b32", "v_mul_f64",
                           "v_rsq_f32", "v_cvt_f32_f64", "v_rcp_f32", "v_fma_f32", "v_add_f64"};
    float t[11] = {run<0>(out), run<1>(out), run<2>(out), run<3>(out), run<4>(out), run<5>(out),
                   run<6>(out), run<7>(out), run<8>(out), run<9>(out), run<10>(out)};
    for (int k = 0; k < 11; ++k)
        printf("%-40s %8.3f ms  cost %.2f x v_fma_f64\n", names[k], t[k], t[k] / t[0]);
    CK(hipFree(out));
    return 0;
}
