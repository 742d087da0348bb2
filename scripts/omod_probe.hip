// omod_probe.hip -- diagnostic: does the VOP3 output modifier (omod div:2 / div:4) apply to
// v_fma_f64 / v_mul_f64 on gfx950, with the MODE register's IEEE bit set (the compute default) and
// cleared by the kernel itself?  The fused kernel would use it to fold exact power-of-two scalings
// (the rsqrt Newton step's 1/2, the gyro's w/2) into the instruction that produces the value.
// build: hipcc --offload-arch=gfx950 -O2 scripts/omod_probe.hip -o build/omod_probe
#include <hip/hip_runtime.h>

#include <cstdio>

// MODE register (hwreg id 1), field IEEE = bit 9: simm16 = id | offset << 6 | (size - 1) << 11
constexpr int kModeIeee = 1 | (9 << 6) | (0 << 11);
constexpr int kModeAll = 1 | (0 << 6) | (31 << 11);
// FP_DENORM field for f64/f16 = bits 7:6 (0 = flush in and out)
constexpr int kModeDenorm64 = 1 | (6 << 6) | (1 << 11);

// CLEAR: bit 0 clears IEEE, bit 1 clears the f64 denormal mode
template <int CLEAR>
__global__ void k_probe(const double *in, double *out, unsigned *mode) {
    if (CLEAR & 1) __builtin_amdgcn_s_setreg(kModeIeee, 0);
    if (CLEAR & 2) __builtin_amdgcn_s_setreg(kModeDenorm64, 0);
    const int i = threadIdx.x;
    const double a = in[3 * i], b = in[3 * i + 1], c = in[3 * i + 2];
    double r0, r1, r2, r3;
    asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r0) : "v"(a), "v"(b), "v"(c));
    asm volatile("v_fma_f64 %0, %1, %2, %3 div:2" : "=v"(r1) : "v"(a), "v"(b), "v"(c));
    asm volatile("v_mul_f64 %0, %1, %2 mul:4" : "=v"(r2) : "v"(a), "v"(b));
    asm volatile("v_fma_f64 %0, -%1, %2, 1.0 div:2" : "=v"(r3) : "v"(a), "v"(b));
    out[4 * i + 0] = r0;
    out[4 * i + 1] = r1;
    out[4 * i + 2] = r2;
    out[4 * i + 3] = r3;
    if (i == 0) mode[0] = __builtin_amdgcn_s_getreg(kModeAll);
}

int main() {
    const int n = 64;
    double hin[3 * n];
    for (int i = 0; i < n; ++i) {
        hin[3 * i] = 1.0 + 0.013 * i;
        hin[3 * i + 1] = -0.7 + 0.031 * i;
        hin[3 * i + 2] = 0.25 * i - 3.0;
    }
    hin[0] = 0.0;  // signed-zero corner: 0 * b + (-0.0)
    hin[2] = -0.0;
    double *din, *dout;
    unsigned *dmode;
    (void)hipMalloc(&din, sizeof(hin));
    (void)hipMalloc(&dout, 4 * n * sizeof(double));
    (void)hipMalloc(&dmode, 4);
    (void)hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
    for (int clear = 0; clear < 4; ++clear) {
        if (clear == 0) hipLaunchKernelGGL(k_probe<0>, dim3(1), dim3(n), 0, 0, din, dout, dmode);
        if (clear == 1) hipLaunchKernelGGL(k_probe<1>, dim3(1), dim3(n), 0, 0, din, dout, dmode);
        if (clear == 2) hipLaunchKernelGGL(k_probe<2>, dim3(1), dim3(n), 0, 0, din, dout, dmode);
        if (clear == 3) hipLaunchKernelGGL(k_probe<3>, dim3(1), dim3(n), 0, 0, din, dout, dmode);
        double h[4 * n];
        unsigned mode = 0;
        (void)hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
        (void)hipMemcpy(&mode, dmode, 4, hipMemcpyDeviceToHost);
        int ok_div2 = 0, ok_div4 = 0, ok_newton = 0;
        for (int i = 0; i < n; ++i) {
            const double a = hin[3 * i], b = hin[3 * i + 1], c = hin[3 * i + 2];
            ok_div2 += h[4 * i + 1] == __builtin_fma(a, b, c) * 0.5;
            ok_div4 += h[4 * i + 2] == (a * b) * 4.0;
            ok_newton += h[4 * i + 3] == __builtin_fma(-a, b, 1.0) * 0.5;
        }
        std::printf("clear=%d (MODE=0x%08x): fma div:2 exact %d/%d, mul mul:4 exact %d/%d, fma(-a,b,1) div:2 exact %d/%d;"
                    " lane0 plain %g div2 %g (signbit %d)\n",
                    clear, mode, ok_div2, n, ok_div4, n, ok_newton, n, h[0], h[1],
                    (int)__builtin_signbit(h[1]));
    }
    return 0;
}
