// pekf_synth.hip -- device generator of synthetic IMU streams, bit-identical to
// poseestimationkf_amd/synth.py (the host mirror used to regenerate sampled filters).
// Every floating-point operation is one correctly rounded IEEE op, in the same order as
// the host code; this file is compiled with -ffp-contract=off (no FMA contraction).
#include "pekf_internal.hpp"

#pragma clang fp contract(off)

namespace pekf {

constexpr int kSynthBlock = 256;
constexpr uint32_t kInitStep = 0xFFFFFFFFu;
constexpr uint32_t kDtMin = 4000000u, kDtSpan = 16000001u, kMissThresh = 5033165u;

struct U4 {
    uint32_t v[4];
};

// Philox4x32-10 (Salmon et al., SC'11)
__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                     uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    return U4{{c0, c1, c2, c3}};
}

__device__ __forceinline__ double noise(const U4 &x, double scale) {
    const double k = 5.9604644775390625e-08;  // 2^-24
    const double u0 = (double)(x.v[0] >> 8) * k, u1 = (double)(x.v[1] >> 8) * k;
    const double u2 = (double)(x.v[2] >> 8) * k, u3 = (double)(x.v[3] >> 8) * k;
    return ((((u0 + u1) + u2) + u3) - 2.0) * scale;
}

__device__ __forceinline__ void normalise3(double &x, double &y, double &z) {
    const double n = sqrt((x * x + y * y) + z * z);
    x = x / n;
    y = y / n;
    z = z / n;
}

// R(q)^T v (body <- world), same expression order as synth._body
__device__ __forceinline__ void body(const double *q, const double *v, double *o) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double r00 = 1.0 - 2.0 * (y * y + z * z), r01 = 2.0 * (x * y - w * z), r02 = 2.0 * (x * z + w * y);
    const double r10 = 2.0 * (x * y + w * z), r11 = 1.0 - 2.0 * (x * x + z * z), r12 = 2.0 * (y * z - w * x);
    const double r20 = 2.0 * (x * z - w * y), r21 = 2.0 * (y * z + w * x), r22 = 1.0 - 2.0 * (x * x + y * y);
    o[0] = (r00 * v[0] + r10 * v[1]) + r20 * v[2];
    o[1] = (r01 * v[0] + r11 * v[1]) + r21 * v[2];
    o[2] = (r02 * v[0] + r12 * v[1]) + r22 * v[2];
}

__device__ __forceinline__ void measure(const double *q, const double *ref, const U4 &n0, const U4 &n1,
                                        const U4 &n2, double scale, float *f) {
    double b[3];
    body(q, ref, b);
    double a0 = b[0] + noise(n0, scale), a1 = b[1] + noise(n1, scale), a2 = b[2] + noise(n2, scale);
    normalise3(a0, a1, a2);
    f[0] = (float)a0;
    f[1] = (float)a1;
    f[2] = (float)a2;
    if (fabsf(f[2]) >= 1.0f) f[2] = copysignf(0.99999994f, f[2]);
    if (f[2] == 0.0f) f[2] = 1e-30f;
}

__global__ __launch_bounds__(kSynthBlock) void k_synth(int64_t batch, int64_t window, int64_t first,
                                                       uint32_t seed, int missing, double s_ref,
                                                       double s_w, double s_g, double s_a, double s_m,
                                                       double ar_w, float4 *gd, float4 *am, float2 *my,
                                                       double *refs) {
    const int64_t i = (int64_t)blockIdx.x * kSynthBlock + threadIdx.x;
    if (i >= batch) return;
    const uint32_t id = (uint32_t)(first + i);
    // reference vectors (synth.reference_vectors)
    double ref_a[3], ref_m[3];
    {
        double n[6];
#pragma unroll
        for (int s = 0; s < 6; ++s) n[s] = noise(philox(kInitStep, s, 0, 0, seed, id), s_ref);
        double ax = 0.0 + n[0], ay = 0.0 + n[1], az = 1.0 + n[2];
        double mx = 0.5 + n[3], my_ = 0.0 + n[4], mz = -0.8660254037844386 + n[5];
        normalise3(ax, ay, az);
        normalise3(mx, my_, mz);
        ref_a[0] = (double)(float)ax; ref_a[1] = (double)(float)ay; ref_a[2] = (double)(float)az;
        ref_m[0] = (double)(float)mx; ref_m[1] = (double)(float)my_; ref_m[2] = (double)(float)mz;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            refs[6 * i + k] = ref_a[k];
            refs[6 * i + 3 + k] = ref_m[k];
        }
    }
    double w[3] = {0.0, 0.0, 0.0};
    double q[4] = {1.0, 0.0, 0.0, 0.0};
    for (int64_t t = 0; t < window; ++t) {
        const uint32_t ts = (uint32_t)t;
        const U4 s0 = philox(ts, 0, 0, 0, seed, id);
        uint32_t dt = kDtMin + s0.v[0] % kDtSpan;
        uint32_t word = dt;
        if (missing && (s0.v[1] >> 8) < kMissThresh) word |= PEKF_MISSING_MAG_BIT;
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k] = ar_w * w[k] + noise(philox(ts, 1 + k, 0, 0, seed, id), s_w);
        const double h = (double)dt * 1e-9;
        const double th2 = 0.25 * ((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
        const double x = (h * h) * th2;
        const double ca = (1.0 - x * 0.5) + (x * x) / 24.0;
        const double cb = h * (1.0 - x / 6.0);
        const double r0 = 0.5 * ((-(w[0] * q[1]) - w[1] * q[2]) - w[2] * q[3]);
        const double r1 = 0.5 * ((w[0] * q[0] + w[2] * q[2]) - w[1] * q[3]);
        const double r2 = 0.5 * ((w[1] * q[0] - w[2] * q[1]) + w[0] * q[3]);
        const double r3 = 0.5 * ((w[2] * q[0] + w[1] * q[1]) - w[0] * q[2]);
        q[0] = ca * q[0] + cb * r0;
        q[1] = ca * q[1] + cb * r1;
        q[2] = ca * q[2] + cb * r2;
        q[3] = ca * q[3] + cb * r3;
        const double n = sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
        q[0] = q[0] / n;
        q[1] = q[1] / n;
        q[2] = q[2] / n;
        q[3] = q[3] / n;
        float g[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) g[k] = (float)(w[k] + noise(philox(ts, 4 + k, 0, 0, seed, id), s_g));
        float fa[3], fm[3];
        measure(q, ref_a, philox(ts, 7, 0, 0, seed, id), philox(ts, 8, 0, 0, seed, id),
                philox(ts, 9, 0, 0, seed, id), s_a, fa);
        measure(q, ref_m, philox(ts, 10, 0, 0, seed, id), philox(ts, 11, 0, 0, seed, id),
                philox(ts, 12, 0, 0, seed, id), s_m, fm);
        const int64_t o = t * batch + i;
        gd[o] = make_float4(g[0], g[1], g[2], __uint_as_float(word));
        am[o] = make_float4(fa[0], fa[1], fa[2], fm[0]);
        my[o] = make_float2(fm[1], fm[2]);
    }
}

}  // namespace pekf

using namespace pekf;

extern "C" int pekf_synth_dev(int64_t batch, int64_t window, int64_t first_filter, uint32_t seed,
                              int missing_mag, const double *scales, double ar_w, void *plane_gd,
                              void *plane_am, void *plane_my, double *refs, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && window >= 0 && first_filter >= 0, "negative size");
    if (batch == 0 || window == 0) return PEKF_OK;
    PEKF_CHECK_ARG(scales && plane_gd && plane_am && plane_my && refs, "null pointer");
    PEKF_CHECK_ARG(first_filter + batch <= ((int64_t)1 << 32), "filter ids must fit in 32 bits");
    PEKF_CHECK_ARG(window <= 0xFFFFFFFFll, "window must fit in 32 bits");
    hipLaunchKernelGGL(k_synth, dim3(grid_for(batch, kSynthBlock)), dim3(kSynthBlock), 0,
                       as_stream(stream), batch, window, first_filter, seed, missing_mag, scales[0],
                       scales[1], scales[2], scales[3], scales[4], ar_w,
                       static_cast<float4 *>(plane_gd), static_cast<float4 *>(plane_am),
                       static_cast<float2 *>(plane_my), refs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_synth");
    return PEKF_OK;
}
