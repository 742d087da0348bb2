// probe_latency.hip -- diagnostic: dependent-issue latency (cycles from one instruction to the next
// that consumes its result) of the instructions the fused kernel's hot loop is made of, with ONE
// wave per SIMD (config 2's occupancy, where a record's dependency chain is what binds).
// Each lane runs one dependent chain; cycles = s_memtime delta / (iterations * chain length),
// reported in shader-clock cycles via the wall-clock ratio measured in the same run.
// build: hipcc --offload-arch=gfx950 -O3 scripts/probe_latency.hip -o build/probe_latency
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;
constexpr int kChain = 16;

template <int KIND>
__global__ __launch_bounds__(64) void k_lat(double *out, unsigned long long *cyc, double seed) {
    double v = seed + 1e-3 * threadIdx.x;
    const double a = 0.999999, b = 1e-7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int c = 0; c < kChain; ++c) {
            if (KIND == 0) v = fma(v, a, b);
            if (KIND == 1) v = v * a;
            if (KIND == 2) v = v + b;
            if (KIND == 3) v = __builtin_amdgcn_rsq(v);
            if (KIND == 4) v = __builtin_amdgcn_rcp(v);
            if (KIND == 5) v = (double)(float)v;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static double run(const char *name, double *d, unsigned long long *c, int blocks) {
    hipLaunchKernelGGL(k_lat<KIND>, dim3(blocks), dim3(64), 0, 0, d, c, 1.5);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_lat<KIND>, dim3(blocks), dim3(64), 0, 0, d, c, 1.5);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost);
    const double ops = (double)kIters * kChain;
    // kernel time per dependent op in ns (launch overhead is negligible at these lengths)
    const double ns = ms * 1e6 / ops;
    printf("%-22s %8.3f ms  %7.3f ns per dependent op  (s_memtime ticks %llu, %.3f per op)\n", name, ms, ns, h,
           (double)h / ops);
    return ns;
}

int main() {
    int dev = 0, cus = 0, clk = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    const int blocks = 4 * cus;  // one 64-lane wave per SIMD
    double *d;
    unsigned long long *c;
    (void)hipMalloc(&d, blocks * 64 * sizeof(double));
    (void)hipMalloc(&c, blocks * sizeof(unsigned long long));
    printf("%d CUs, %d one-wave blocks (one wave per SIMD), max clock %.0f MHz\n", cus, blocks, clk / 1e3);
    run<0>("v_fma_f64", d, c, blocks);
    run<1>("v_mul_f64", d, c, blocks);
    run<2>("v_add_f64", d, c, blocks);
    run<3>("v_rsq_f64", d, c, blocks);
    run<4>("v_rcp_f64", d, c, blocks);
    run<5>("cvt f64->f32->f64", d, c, blocks);
    return 0;
}
