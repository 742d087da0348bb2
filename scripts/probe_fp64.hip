// probe_fp64.hip -- diagnostic: accuracy of the gfx950 v_rcp_f64 / v_rsq_f64 seeds and of
// 1 or 2 Newton steps, in ulps against correctly rounded 1/x and 1/sqrt(x).
// build: hipcc --offload-arch=gfx950 -O3 scripts/probe_fp64.hip -o build/probe_fp64
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__device__ double rcp_n(double x, int it) {
    double r = __builtin_amdgcn_rcp(x);
    for (int i = 0; i < it; ++i) {
        double e = fma(-x, r, 1.0);
        r = fma(r, e, r);
    }
    return r;
}

__device__ double rsq_n(double x, int it) {
    double y = __builtin_amdgcn_rsq(x);
    for (int i = 0; i < it; ++i) {
        double e = fma(-x * y, y, 1.0);
        y = fma(y, 0.5 * e, y);
    }
    return y;
}

__device__ double ulps(double got, double want) {
    long long a, b;
    memcpy(&a, &got, 8);
    memcpy(&b, &want, 8);
    return fabs((double)(a - b));
}

__global__ void probe(int n, const double *xs, double *out /* 6 x n */) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = xs[i];
    double r = 1.0 / x, s = 1.0 / sqrt(x);
    for (int it = 0; it < 3; ++it) {
        out[(2 * it) * n + i] = ulps(rcp_n(x, it), r);
        out[(2 * it + 1) * n + i] = ulps(rsq_n(x, it), s);
    }
}

int main() {
    const int n = 1 << 22;
    std::vector<double> xs(n);
    uint64_t st = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        double u = (double)(st >> 11) * 0x1.0p-53;
        xs[i] = std::pow(10.0, -6.0 + 12.0 * u);  // 1e-6 .. 1e6
    }
    double *dx, *dout;
    hipMalloc(&dx, n * 8);
    hipMalloc(&dout, 6 * (size_t)n * 8);
    hipMemcpy(dx, xs.data(), n * 8, hipMemcpyHostToDevice);
    probe<<<(n + 255) / 256, 256>>>(n, dx, dout);
    std::vector<double> out(6 * (size_t)n);
    hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
    const char *names[6] = {"rcp seed", "rsq seed", "rcp +1 Newton", "rsq +1 Newton", "rcp +2 Newton", "rsq +2 Newton"};
    for (int k = 0; k < 6; ++k) {
        double mx = 0, mean = 0;
        for (int i = 0; i < n; ++i) {
            double v = out[(size_t)k * n + i];
            mx = v > mx ? v : mx;
            mean += v;
        }
        printf("%-16s max %.3g ulp, mean %.3g ulp (rel ~ %.3g)\n", names[k], mx, mean / n, mx * 0x1.0p-52);
    }
    return 0;
}
