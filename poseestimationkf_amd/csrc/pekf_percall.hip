// pekf_percall.hip -- per-call operators behind the drop-in Python API (one thread per item).
//
// These keep the reference's dense formulation (ExtendedKalmanFilter.py, Wahba.py) so
// each call matches NumPy to rounding; the fused time-loop kernel is pekf_run.hip.
#include <cstring>
#include <vector>

#include "pekf_internal.hpp"
#include "pekf_math.hpp"

namespace pekf {

constexpr int kBlock = 256;

__device__ __forceinline__ void d_rk4(int64_t i, const double *q0, const double *dt,
                                               const double *w, double *out) {
    rk4_literal(q0 + 4 * i, dt[i], w + 3 * i, out + 4 * i);
}

__global__ __launch_bounds__(kBlock) void k_rk4(int64_t n, const double *q0, const double *dt,
                                               const double *w, double *out, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_rk4(i, q0, dt, w, out);
    done.signal();  // the whole block reaches this point (no early return)
}

__device__ __forceinline__ void d_norm(int64_t i, int64_t len, const double *a,
                                                double *out) {
    double s = 0.0;
    for (int64_t k = 0; k < len; ++k) s += a[i * len + k] * a[i * len + k];
    out[i] = sqrt(s);
}

__global__ __launch_bounds__(kBlock) void k_norm(int64_t n, int64_t len, const double *a,
                                                double *out, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_norm(i, len, a, out);
    done.signal();  // the whole block reaches this point (no early return)
}

__device__ __forceinline__ void d_jac_a(int64_t i, const double *w, double *A) {
    omega_half(w + 3 * i, A + 16 * i);
}

__global__ __launch_bounds__(kBlock) void k_jac_a(int64_t n, const double *w, double *A, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_jac_a(i, w, A);
    done.signal();  // the whole block reaches this point (no early return)
}

__device__ __forceinline__ void d_jac_b(int64_t i, const double *q, double *J) {
    xi_half(q + 4 * i, J + 12 * i);
}

__global__ __launch_bounds__(kBlock) void k_jac_b(int64_t n, const double *q, double *J, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_jac_b(i, q, J);
    done.signal();  // the whole block reaches this point (no early return)
}

// conj(q1) (x) q2 as the reference's 4x4 left-multiplication (ExtendedKalmanFilter.py:16-23)
__device__ __forceinline__ void d_comparator(int64_t i, const double *q1,
                                                      const double *q2, double *out) {
    const double *a = q1 + 4 * i, *b = q2 + 4 * i;
    const double c0 = a[0], c1 = -a[1], c2 = -a[2], c3 = -a[3];
    const double L[16] = {c0, -c1, -c2, -c3, c1, c0, -c3, c2, c2, c3, c0, -c1, c3, -c2, c1, c0};
    matmul<4, 4, 1>(L, b, out + 4 * i);
}

__global__ __launch_bounds__(kBlock) void k_comparator(int64_t n, const double *q1,
                                                      const double *q2, double *out, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_comparator(i, q1, q2, out);
    done.signal();  // the whole block reaches this point (no early return)
}

// KalmanFilter.Prediction (ExtendedKalmanFilter.py:58-68)
__device__ __forceinline__ void d_predict(int64_t i, const double *gyro,
                                                   const double *dt, const double *X,
                                                   const double *P, const double *Q,
                                                   const double *R, double *z, double *Pm,
                                                   double *K, int32_t *status) {
    double A[16], At[16], Jb[12], Jbt[12], t16[16], a16[16], t12[12], b16[16], S[16], Si[16], pm[16];
    omega_half(gyro + 3 * i, A);
    xi_half(X + 4 * i, Jb);
    transpose<4, 4>(A, At);
    transpose<4, 3>(Jb, Jbt);
    matmul<4, 4, 4>(A, P + 16 * i, t16);
    matmul<4, 4, 4>(t16, At, a16);
    matmul<4, 3, 3>(Jb, Q + 9 * i, t12);
    matmul<4, 3, 4>(t12, Jbt, b16);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        pm[k] = a16[k] + b16[k];
        S[k] = pm[k] + R[16 * i + k];
        Pm[16 * i + k] = pm[k];
    }
    rk4_literal(X + 4 * i, dt[i], gyro + 3 * i, z + 4 * i);
    const bool ok = inverse4(S, Si);
    if (status) status[i] = ok ? 0 : 1;
    if (!ok) {
#pragma unroll
        for (int k = 0; k < 16; ++k) K[16 * i + k] = NAN;
        return;
    }
    matmul<4, 4, 4>(pm, Si, K + 16 * i);
}

__global__ __launch_bounds__(kBlock) void k_predict(int64_t n, const double *gyro,
                                                   const double *dt, const double *X,
                                                   const double *P, const double *Q,
                                                   const double *R, double *z, double *Pm,
                                                   double *K, int32_t *status, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_predict(i, gyro, dt, X, P, Q, R, z, Pm, K, status);
    done.signal();  // the whole block reaches this point (no early return)
}

// KalmanFilter.Correction (ExtendedKalmanFilter.py:70-80)
__device__ __forceinline__ void d_correct(int64_t i, const double *mag,
                                                   const double *acc, const double *z,
                                                   const double *P, const double *K,
                                                   const double *acc0, const double *mag0,
                                                   double *X, double *Pout, int32_t *status) {
    const double *a = acc + 3 * i, *zz = z + 4 * i, *kk = K + 16 * i, *pp = P + 16 * i;
    const double ka = fabs(a[2]);
    if (status) status[i] = wahba_b_finite(acc0 + 3 * i, mag0 + 3 * i, a, mag + 3 * i, ka, 1.0 - ka) ? 0 : 1;
    double R[9], y[4], e[4], ke[4], kp[16], x[4];
    wahba_rotation_vectors(acc0 + 3 * i, mag0 + 3 * i, a, mag + 3 * i, ka, 1.0 - ka, R);
    rotm_to_quat(R, y);
    const double cmp = y[0] * zz[0] + y[1] * zz[1] + y[2] * zz[2] + y[3] * zz[3];
    if (cmp < 0.0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = -y[k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = y[k] - zz[k];
    matmul<4, 4, 1>(kk, e, ke);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = zz[k] + ke[k];
    matmul<4, 4, 4>(kk, pp, kp);
#pragma unroll
    for (int k = 0; k < 16; ++k) Pout[16 * i + k] = pp[k] - kp[k];
    const double nrm = loop_norm4(x);
#pragma unroll
    for (int k = 0; k < 4; ++k) X[4 * i + k] = x[k] / nrm;
}

__global__ __launch_bounds__(kBlock) void k_correct(int64_t n, const double *mag,
                                                   const double *acc, const double *z,
                                                   const double *P, const double *K,
                                                   const double *acc0, const double *mag0,
                                                   double *X, double *Pout, int32_t *status, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_correct(i, mag, acc, z, P, K, acc0, mag0, X, Pout, status);
    done.signal();  // the whole block reaches this point (no early return)
}

template <bool QUAT>
__device__ __forceinline__ void d_wahba(int64_t i, const double *acc0,
                                                 const double *mag0, const double *acc,
                                                 const double *mag, const double *ka,
                                                 const double *km, double *out, int32_t *status) {
    if (status)
        status[i] = wahba_b_finite(acc0 + 3 * i, mag0 + 3 * i, acc + 3 * i, mag + 3 * i, ka[i], km[i]) ? 0 : 1;
    double R[9];
    wahba_rotation_vectors(acc0 + 3 * i, mag0 + 3 * i, acc + 3 * i, mag + 3 * i, ka[i], km[i], R);
    if (QUAT) {
        rotm_to_quat(R, out + 4 * i);
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) out[9 * i + k] = R[k];
    }
}

template <bool QUAT>
__global__ __launch_bounds__(kBlock) void k_wahba(int64_t n, const double *acc0,
                                                 const double *mag0, const double *acc,
                                                 const double *mag, const double *ka,
                                                 const double *km, double *out, int32_t *status, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_wahba<QUAT>(i, acc0, mag0, acc, mag, ka, km, out, status);
    done.signal();  // the whole block reaches this point (no early return)
}

__device__ __forceinline__ void d_r2q(int64_t i, const double *M, double *q) {
    rotm_to_quat(M + 9 * i, q + 4 * i);
}

__global__ __launch_bounds__(kBlock) void k_r2q(int64_t n, const double *M, double *q, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) d_r2q(i, M, q);
    done.signal();  // the whole block reaches this point (no early return)
}

// n = 1 calls (what main_file.py makes, one record at a time): the inputs travel by value in the
// kernel-argument segment with the dispatch itself instead of being read over PCIe from pinned
// host memory, so the kernel starts with its operands in hand.  The body is the same device
// function as the batched kernel, on a private copy (promoted to registers after inlining).
constexpr int kBlobDoubles = 64;
struct Blob {
    double v[kBlobDoubles];
};
enum : int { kCallPredict = 0, kCallCorrect = 1, kCallWahbaQuat = 2 };

template <int OP>
__global__ __launch_bounds__(64) void k_call1(Blob b, double *out, int32_t *status, Done done) {
    if (threadIdx.x == 0) {
        double v[kBlobDoubles];
#pragma unroll
        for (int k = 0; k < kBlobDoubles; ++k) v[k] = b.v[k];
        if (OP == kCallPredict)  // gyro 3, dt 1, X 4, P 16, Q 9, R 16 -> z 4, Pm 16, K 16
            d_predict(0, v, v + 3, v + 4, v + 8, v + 24, v + 33, out, out + 4, out + 20, status);
        else if (OP == kCallCorrect)  // mag 3, acc 3, z 4, P 16, K 16, acc0 3, mag0 3 -> X 4, P 16
            d_correct(0, v, v + 3, v + 6, v + 10, v + 26, v + 42, v + 45, out, out + 4, status);
        else  // acc0 3, mag0 3, acc 3, mag 3, ka 1, km 1 -> q 4
            d_wahba<true>(0, v, v + 3, v + 6, v + 9, v + 12, v + 13, out, status);
    }
    done.signal();
}

static int launched(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, what);
    return PEKF_OK;
}

#define PEKF_GRID(n) dim3(grid_for((n), kBlock)), dim3(kBlock)

// Host side of k_call1: packs the inputs (in order) into the Blob, runs the call with zero-copy
// outputs and returns them (in order) plus the status word.
template <int OP>
static int call1(std::initializer_list<HostArg> ins, std::initializer_list<HostOut> outs, int32_t *status) {
    Blob b;
    size_t off = 0;
    for (const HostArg &a : ins) {
        std::memcpy(reinterpret_cast<char *>(b.v) + off, a.ptr, a.bytes);
        off += a.bytes;
    }
    size_t ob = 0;
    for (const HostOut &o : outs) ob += o.bytes;
    double tmp[kBlobDoubles];
    Staging &s = Staging::get();
    void *out[2];
    if (int st = s.stage_in({}, {ob, sizeof(int32_t)}, nullptr, out)) return st;
    hipLaunchKernelGGL(k_call1<OP>, dim3(1), dim3(64), 0, s.stream(), b, static_cast<double *>(out[0]),
                       static_cast<int32_t *>(out[1]), s.done(1));
    if (int st = launched("k_call1")) return st;
    if (int st = s.stage_out({{tmp, ob}, {status, sizeof(int32_t)}}, out)) return st;
    off = 0;
    for (const HostOut &o : outs) {
        std::memcpy(o.ptr, reinterpret_cast<char *>(tmp) + off, o.bytes);
        off += o.bytes;
    }
    return PEKF_OK;
}

#define D(T, p) static_cast<T>(p)

}  // namespace pekf

using namespace pekf;

extern "C" {

// ------------------------------- device-pointer variants -------------------------------------

int pekf_rk4_dev(int64_t n, const double *q0, const double *dt_ns, const double *w, double *q_out,
                 void *stream) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(q0 && dt_ns && w && q_out, "null pointer");
    hipLaunchKernelGGL(k_rk4, PEKF_GRID(n), 0, as_stream(stream), n, q0, dt_ns, w, q_out, kNoSignal);
    return launched("k_rk4");
}

int pekf_predict_dev(int64_t n, const double *gyro, const double *dt_ns, const double *X,
                     const double *P, const double *Q, const double *R, double *z, double *Pm,
                     double *K, int32_t *status, void *stream) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(gyro && dt_ns && X && P && Q && R && z && Pm && K, "null pointer");
    hipLaunchKernelGGL(k_predict, PEKF_GRID(n), 0, as_stream(stream), n, gyro, dt_ns, X, P, Q, R,
                       z, Pm, K, status, kNoSignal);
    return launched("k_predict");
}

int pekf_correct_dev(int64_t n, const double *mag, const double *acc, const double *z,
                     const double *P, const double *K, const double *acc0, const double *mag0,
                     double *X, double *P_out, void *stream) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(mag && acc && z && P && K && acc0 && mag0 && X && P_out, "null pointer");
    hipLaunchKernelGGL(k_correct, PEKF_GRID(n), 0, as_stream(stream), n, mag, acc, z, P, K, acc0,
                       mag0, X, P_out, nullptr, kNoSignal);
    return launched("k_correct");
}

// ------------------------------- host-pointer variants ---------------------------------------

int pekf_rk4(int64_t n, const double *q0, const double *dt_ns, const double *w, double *q_out) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(q0 && dt_ns && w && q_out, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[3], *out[1];
    if (int st = s.stage_in({{q0, 4 * b}, {dt_ns, b}, {w, 3 * b}}, {4 * b}, in, out)) return st;
    hipLaunchKernelGGL(k_rk4, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(const double *, in[1]), D(const double *, in[2]), D(double *, out[0]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_rk4")) return st;
    return s.stage_out({{q_out, 4 * b}}, out);
}

int pekf_norm(int64_t n, int64_t len, const double *a, double *res) {
    PEKF_CHECK_ARG(n >= 0 && len >= 0, "negative size");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(a && res, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[1], *out[1];
    if (int st = s.stage_in({{a, (size_t)len * b}}, {b}, in, out)) return st;
    hipLaunchKernelGGL(k_norm, PEKF_GRID(n), 0, s.stream(), n, len, D(const double *, in[0]),
                       D(double *, out[0]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_norm")) return st;
    return s.stage_out({{res, b}}, out);
}

int pekf_jacobian_a(int64_t n, const double *w, double *A) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(w && A, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[1], *out[1];
    if (int st = s.stage_in({{w, 3 * b}}, {16 * b}, in, out)) return st;
    hipLaunchKernelGGL(k_jac_a, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(double *, out[0]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_jac_a")) return st;
    return s.stage_out({{A, 16 * b}}, out);
}

int pekf_jacobian_b(int64_t n, const double *q, double *Jb) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(q && Jb, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[1], *out[1];
    if (int st = s.stage_in({{q, 4 * b}}, {12 * b}, in, out)) return st;
    hipLaunchKernelGGL(k_jac_b, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(double *, out[0]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_jac_b")) return st;
    return s.stage_out({{Jb, 12 * b}}, out);
}

int pekf_comparator(int64_t n, const double *q1, const double *q2, double *res) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(q1 && q2 && res, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[2], *out[1];
    if (int st = s.stage_in({{q1, 4 * b}, {q2, 4 * b}}, {4 * b}, in, out)) return st;
    hipLaunchKernelGGL(k_comparator, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(const double *, in[1]), D(double *, out[0]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_comparator")) return st;
    return s.stage_out({{res, 4 * b}}, out);
}

int pekf_predict(int64_t n, const double *gyro, const double *dt_ns, const double *X,
                 const double *P, const double *Q, const double *R, double *z, double *Pm,
                 double *K) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(gyro && dt_ns && X && P && Q && R && z && Pm && K, "null pointer");
    if (int st = require_device()) return st;
    const size_t b = (size_t)n * sizeof(double);
    if (n == 1) {
        int32_t st1 = 0;
        if (int st = call1<kCallPredict>({{gyro, 3 * b}, {dt_ns, b}, {X, 4 * b}, {P, 16 * b}, {Q, 9 * b}, {R, 16 * b}},
                                         {{z, 4 * b}, {Pm, 16 * b}, {K, 16 * b}}, &st1))
            return st;
        return st1 ? set_error(PEKF_ERR_SINGULAR, "Singular matrix") : PEKF_OK;
    }
    Staging &s = Staging::get();
    const size_t sb = (size_t)n * sizeof(int32_t);
    std::vector<int32_t> status((size_t)n);
    void *in[6], *out[4];
    if (int st = s.stage_in({{gyro, 3 * b}, {dt_ns, b}, {X, 4 * b}, {P, 16 * b}, {Q, 9 * b}, {R, 16 * b}},
                            {4 * b, 16 * b, 16 * b, sb}, in, out))
        return st;
    hipLaunchKernelGGL(k_predict, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(const double *, in[1]), D(const double *, in[2]), D(const double *, in[3]),
                       D(const double *, in[4]), D(const double *, in[5]), D(double *, out[0]),
                       D(double *, out[1]), D(double *, out[2]), D(int32_t *, out[3]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_predict")) return st;
    if (int st = s.stage_out({{z, 4 * b}, {Pm, 16 * b}, {K, 16 * b}, {status.data(), sb}}, out)) return st;
    for (int32_t v : status)
        if (v) return set_error(PEKF_ERR_SINGULAR, "Singular matrix");
    return PEKF_OK;
}

int pekf_correct(int64_t n, const double *mag, const double *acc, const double *z,
                 const double *P, const double *K, const double *acc0, const double *mag0,
                 double *X, double *P_out) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(mag && acc && z && P && K && acc0 && mag0 && X && P_out, "null pointer");
    if (int st = require_device()) return st;
    const size_t b = (size_t)n * sizeof(double);
    if (n == 1) {
        int32_t st1 = 0;
        if (int st = call1<kCallCorrect>({{mag, 3 * b}, {acc, 3 * b}, {z, 4 * b}, {P, 16 * b}, {K, 16 * b},
                                          {acc0, 3 * b}, {mag0, 3 * b}},
                                         {{X, 4 * b}, {P_out, 16 * b}}, &st1))
            return st;
        return st1 ? set_error(PEKF_ERR_SVD, "SVD did not converge") : PEKF_OK;
    }
    Staging &s = Staging::get();
    const size_t sb = (size_t)n * sizeof(int32_t);
    std::vector<int32_t> status((size_t)n);
    void *in[7], *out[3];
    if (int st = s.stage_in({{mag, 3 * b}, {acc, 3 * b}, {z, 4 * b}, {P, 16 * b}, {K, 16 * b},
                             {acc0, 3 * b}, {mag0, 3 * b}},
                            {4 * b, 16 * b, sb}, in, out))
        return st;
    hipLaunchKernelGGL(k_correct, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(const double *, in[1]), D(const double *, in[2]), D(const double *, in[3]),
                       D(const double *, in[4]), D(const double *, in[5]), D(const double *, in[6]),
                       D(double *, out[0]), D(double *, out[1]), D(int32_t *, out[2]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_correct")) return st;
    if (int st = s.stage_out({{X, 4 * b}, {P_out, 16 * b}, {status.data(), sb}}, out)) return st;
    for (int32_t v : status)
        if (v) return set_error(PEKF_ERR_SVD, "SVD did not converge");
    return PEKF_OK;
}

static int wahba_host(bool quat, int64_t n, const double *acc0, const double *mag0,
                      const double *acc, const double *mag, const double *k_acc,
                      const double *k_mag, double *res) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(acc0 && mag0 && acc && mag && k_acc && k_mag && res, "null pointer");
    if (int st = require_device()) return st;
    const size_t b = (size_t)n * sizeof(double);
    if (n == 1 && quat) {
        int32_t st1 = 0;
        if (int st = call1<kCallWahbaQuat>({{acc0, 3 * b}, {mag0, 3 * b}, {acc, 3 * b}, {mag, 3 * b}, {k_acc, b},
                                            {k_mag, b}},
                                           {{res, 4 * b}}, &st1))
            return st;
        return st1 ? set_error(PEKF_ERR_SVD, "SVD did not converge") : PEKF_OK;
    }
    Staging &s = Staging::get();
    const size_t ob = (quat ? 4 : 9) * b;
    const size_t sb = (size_t)n * sizeof(int32_t);
    std::vector<int32_t> status((size_t)n);
    void *in[6], *out[2];
    if (int st = s.stage_in({{acc0, 3 * b}, {mag0, 3 * b}, {acc, 3 * b}, {mag, 3 * b}, {k_acc, b}, {k_mag, b}},
                            {ob, sb}, in, out))
        return st;
    if (quat)
        hipLaunchKernelGGL(k_wahba<true>, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                           D(const double *, in[1]), D(const double *, in[2]), D(const double *, in[3]),
                           D(const double *, in[4]), D(const double *, in[5]), D(double *, out[0]),
                           D(int32_t *, out[1]), s.done(grid_for(n, kBlock)));
    else
        hipLaunchKernelGGL(k_wahba<false>, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                           D(const double *, in[1]), D(const double *, in[2]), D(const double *, in[3]),
                           D(const double *, in[4]), D(const double *, in[5]), D(double *, out[0]),
                           D(int32_t *, out[1]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_wahba")) return st;
    if (int st = s.stage_out({{res, ob}, {status.data(), sb}}, out)) return st;
    for (int32_t v : status)
        if (v) return set_error(PEKF_ERR_SVD, "SVD did not converge");
    return PEKF_OK;
}

int pekf_wahba_rotation(int64_t n, const double *acc0, const double *mag0, const double *acc,
                        const double *mag, const double *k_acc, const double *k_mag, double *R) {
    return wahba_host(false, n, acc0, mag0, acc, mag, k_acc, k_mag, R);
}

int pekf_wahba_quaternion(int64_t n, const double *acc0, const double *mag0, const double *acc,
                          const double *mag, const double *k_acc, const double *k_mag, double *q) {
    return wahba_host(true, n, acc0, mag0, acc, mag, k_acc, k_mag, q);
}

int pekf_rotmat_to_quat(int64_t n, const double *M, double *q) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(M && q, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[1], *out[1];
    if (int st = s.stage_in({{M, 9 * b}}, {4 * b}, in, out)) return st;
    hipLaunchKernelGGL(k_r2q, PEKF_GRID(n), 0, s.stream(), n, D(const double *, in[0]),
                       D(double *, out[0]), s.done(grid_for(n, kBlock)));
    if (int st = launched("k_r2q")) return st;
    return s.stage_out({{q, 4 * b}}, out);
}

}  // extern "C"
