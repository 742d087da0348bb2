// pekf_percall.hip -- per-call operators behind the drop-in Python API (one thread per item).
//
// These keep the reference's dense formulation (ExtendedKalmanFilter.py, Wahba.py) so
// each call matches NumPy to rounding; the fused time-loop kernel is pekf_run.hip.  The batched
// kernels move their per-item operands through WaveTile (pekf_tile.hpp): coalesced block reads
// and writes, transposed through LDS; the d_* bodies work on per-lane copies.
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "pekf_internal.hpp"
#include "pekf_math.hpp"
#include "pekf_tile.hpp"

namespace pekf {

constexpr int kBlock = 256;

__device__ __forceinline__ void d_rk4(int64_t i, const double *q0, const double *dt,
                                               const double *w, double *out) {
    rk4_literal(q0 + 4 * i, dt[i], w + 3 * i, out + 4 * i);
}

// Pool of LDS for the WaveTiles of a block whose widest operand has W doubles per item.
#define PEKF_TILE(t, W, n)                                                  \
    __shared__ double pool_[kBlock / kWave * tile_doubles<W>()];           \
    const WaveTile t(pool_, tile_doubles<W>(), (n))

__global__ __launch_bounds__(kBlock) void k_rk4(int64_t n, const double *q0, const double *dt,
                                               const double *w, double *out, Done done) {
    PEKF_TILE(t, 4, n);
    double cq[4], cd[1], cw[3], vq[4], vd[1], vw[3], o[4];
    t.gather(q0, cq);
    t.gather(dt, cd);
    t.gather(w, cw);
    t.to_lanes(cq, vq);
    t.to_lanes(cd, vd);
    t.to_lanes(cw, vw);
    d_rk4(0, vq, vd, vw, o);
    t.store(out, o);
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
    PEKF_TILE(t, 16, n);
    double vw[3], o[16];
    t.load(w, vw);
    d_jac_a(0, vw, o);
    t.store(A, o);
    done.signal();  // the whole block reaches this point (no early return)
}

__device__ __forceinline__ void d_jac_b(int64_t i, const double *q, double *J) {
    xi_half(q + 4 * i, J + 12 * i);
}

__global__ __launch_bounds__(kBlock) void k_jac_b(int64_t n, const double *q, double *J, Done done) {
    PEKF_TILE(t, 12, n);
    double vq[4], o[12];
    t.load(q, vq);
    d_jac_b(0, vq, o);
    t.store(J, o);
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
    PEKF_TILE(t, 4, n);
    double c1[4], c2[4], v1[4], v2[4], o[4];
    t.gather(q1, c1);
    t.gather(q2, c2);
    t.to_lanes(c1, v1);
    t.to_lanes(c2, v2);
    d_comparator(0, v1, v2, o);
    t.store(out, o);
    done.signal();  // the whole block reaches this point (no early return)
}

// KalmanFilter.Prediction (ExtendedKalmanFilter.py:58-68), in two phases so that a batched
// kernel needs R only once P^- is formed.  Phase 1: P^- = A P A^T + Jb Q Jb^T (:59-61).
__device__ __forceinline__ void d_predict_cov(const double *gyro, const double *X, const double *P,
                                              const double *Q, double *pm) {
    double A[16], At[16], Jb[12], Jbt[12], t16[16], a16[16], t12[12], b16[16];
    omega_half(gyro, A);
    xi_half(X, Jb);
    transpose<4, 4>(A, At);
    transpose<4, 3>(Jb, Jbt);
    matmul<4, 4, 4>(A, P, t16);
    matmul<4, 4, 4>(t16, At, a16);
    matmul<4, 3, 3>(Jb, Q, t12);
    matmul<4, 3, 4>(t12, Jbt, b16);
#pragma unroll
    for (int k = 0; k < 16; ++k) pm[k] = a16[k] + b16[k];
}

// Phase 2: z = RK4 (:62), S = P^- + R, K = P^- inv(S) (:63-66); status 1 = singular S.
__device__ __forceinline__ void d_predict_gain(const double *gyro, const double *dt, const double *X,
                                               const double *pm, const double *R, double *z, double *K,
                                               int32_t *status) {
    double S[16], Si[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) S[k] = pm[k] + R[k];
    rk4_literal(X, dt[0], gyro, z);
    const bool ok = inverse4(S, Si);
    *status = ok ? 0 : 1;
    if (!ok) {
#pragma unroll
        for (int k = 0; k < 16; ++k) K[k] = NAN;
        return;
    }
    matmul<4, 4, 4>(pm, Si, K);
}

__device__ __forceinline__ void d_predict(const double *gyro, const double *dt, const double *X,
                                          const double *P, const double *Q, const double *R, double *z,
                                          double *Pm, double *K, int32_t *status) {
    d_predict_cov(gyro, X, P, Q, Pm);
    d_predict_gain(gyro, dt, X, Pm, R, z, K, status);
}

__global__ __launch_bounds__(kBlock) void k_predict(int64_t n, const double *gyro,
                                                   const double *dt, const double *X,
                                                   const double *P, const double *Q,
                                                   const double *R, double *z, double *Pm,
                                                   double *K, int32_t *status, Done done) {
    PEKF_TILE(t, 16, n);
    // every operand's loads are issued up front (one memory round trip per wave)
    double cg[3], cd[1], cx[4], cp[16], cq[9], cr[16], vg[3], vd[1], vx[4], vp[16], vq[9], vr[16];
    t.gather(gyro, cg);
    t.gather(dt, cd);
    t.gather(X, cx);
    t.gather(P, cp);
    t.gather(Q, cq);
    t.gather(R, cr);
    t.to_lanes(cg, vg);
    t.to_lanes(cd, vd);
    t.to_lanes(cx, vx);
    t.to_lanes(cp, vp);
    t.to_lanes(cq, vq);
    double opm[16];
    d_predict_cov(vg, vx, vp, vq, opm);
    t.store(Pm, opm);
    t.to_lanes(cr, vr);
    double oz[4], ok[16];
    int32_t st = 0;
    d_predict_gain(vg, vd, vx, opm, vr, oz, ok, &st);
    t.store(z, oz);
    t.store(K, ok);
    if (status && t.active()) status[t.first + t.lane] = st;
    done.signal();  // the whole block reaches this point (no early return)
}

// KalmanFilter.Correction (ExtendedKalmanFilter.py:70-80), in parts so that a batched kernel
// can form P - K P before the Wahba solve and keep only K live across it.  Phase 1: Y = Wahba(Acc, Mag, |Acc_z|,
// 1 - |Acc_z|) (:71), flipped when Y . z < 0 (:73-75); status 1 = non-finite B (SVD failure).
__device__ __forceinline__ void d_correct_measure(const double *mag, const double *acc, const double *z,
                                                  const double *acc0, const double *mag0, double *y,
                                                  int32_t *status) {
    const double ka = fabs(acc[2]);
    *status = wahba_b_finite(acc0, mag0, acc, mag, ka, 1.0 - ka) ? 0 : 1;
    double R[9];
    wahba_rotation_vectors(acc0, mag0, acc, mag, ka, 1.0 - ka, R);
    rotm_to_quat(R, y);
    const double cmp = y[0] * z[0] + y[1] * z[1] + y[2] * z[2] + y[3] * z[3];
    if (cmp < 0.0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = -y[k];
    }
}

// Phase 2: X = z + K (Y - z), X /= norm(X) (:76,78-79).
__device__ __forceinline__ void d_correct_state(const double *y, const double *z, const double *K, double *X) {
    double e[4], ke[4], x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = y[k] - z[k];
    matmul<4, 4, 1>(K, e, ke);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = z[k] + ke[k];
    const double nrm = loop_norm4(x);
#pragma unroll
    for (int k = 0; k < 4; ++k) X[k] = x[k] / nrm;
}

// P = P - K P (:77): independent of the measurement.
__device__ __forceinline__ void d_correct_cov(const double *P, const double *K, double *Pout) {
    double kp[16];
    matmul<4, 4, 4>(K, P, kp);
#pragma unroll
    for (int k = 0; k < 16; ++k) Pout[k] = P[k] - kp[k];
}

__device__ __forceinline__ void d_correct(const double *mag, const double *acc, const double *z,
                                          const double *P, const double *K, const double *acc0,
                                          const double *mag0, double *X, double *Pout, int32_t *status) {
    double y[4];
    d_correct_measure(mag, acc, z, acc0, mag0, y, status);
    d_correct_state(y, z, K, X);
    d_correct_cov(P, K, Pout);
}

__global__ __launch_bounds__(kBlock) void k_correct(int64_t n, const double *mag,
                                                   const double *acc, const double *z,
                                                   const double *P, const double *K,
                                                   const double *acc0, const double *mag0,
                                                   double *X, double *Pout, int32_t *status, Done done) {
    PEKF_TILE(t, 16, n);
    // every operand's loads are issued up front (one memory round trip per wave); P - K P does
    // not depend on the Wahba solve, so it is formed and stored first and only K stays live
    double cp[16], ck[16], cm[3], ca[3], cz[4], cm0[3], ca0[3];
    t.gather(P, cp);
    t.gather(K, ck);
    t.gather(mag, cm);
    t.gather(acc, ca);
    t.gather(z, cz);
    t.gather(acc0, ca0);
    t.gather(mag0, cm0);
    double vp[16], vk[16], op[16];
    t.to_lanes(cp, vp);
    t.to_lanes(ck, vk);
    d_correct_cov(vp, vk, op);
    t.store(Pout, op);
    double vm[3], va[3], vz[4], vm0[3], va0[3], y[4], ox[4];
    t.to_lanes(cm, vm);
    t.to_lanes(ca, va);
    t.to_lanes(cz, vz);
    t.to_lanes(ca0, va0);
    t.to_lanes(cm0, vm0);
    int32_t st = 0;
    d_correct_measure(vm, va, vz, va0, vm0, y, &st);
    d_correct_state(y, vz, vk, ox);
    t.store(X, ox);
    if (status && t.active()) status[t.first + t.lane] = st;
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
    PEKF_TILE(t, 9, n);
    double c0[3], c1[3], c2[3], c3[3], c4[1], c5[1], v0[3], v1[3], v2[3], v3[3], v4[1], v5[1];
    t.gather(acc0, c0);
    t.gather(mag0, c1);
    t.gather(acc, c2);
    t.gather(mag, c3);
    t.gather(ka, c4);
    t.gather(km, c5);
    t.to_lanes(c0, v0);
    t.to_lanes(c1, v1);
    t.to_lanes(c2, v2);
    t.to_lanes(c3, v3);
    t.to_lanes(c4, v4);
    t.to_lanes(c5, v5);
    double o[QUAT ? 4 : 9];
    int32_t st = 0;
    d_wahba<QUAT>(0, v0, v1, v2, v3, v4, v5, o, &st);
    t.store(out, o);
    if (status && t.active()) status[t.first + t.lane] = st;
    done.signal();  // the whole block reaches this point (no early return)
}

__device__ __forceinline__ void d_r2q(int64_t i, const double *M, double *q) {
    rotm_to_quat(M + 9 * i, q + 4 * i);
}

__global__ __launch_bounds__(kBlock) void k_r2q(int64_t n, const double *M, double *q, Done done) {
    PEKF_TILE(t, 9, n);
    double vm[9], o[4];
    t.load(M, vm);
    d_r2q(0, vm, o);
    t.store(q, o);
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
enum : int {
    kCallPredict = 0,    // gyro 3, dt 1, X 4, P 16, Q 9, R 16 -> z 4, Pm 16, K 16
    kCallCorrect = 1,    // mag 3, acc 3, z 4, P 16, K 16, acc0 3, mag0 3 -> X 4, P 16
    kCallWahbaQuat = 2,  // acc0 3, mag0 3, acc 3, mag 3, ka 1, km 1 -> q 4
    kCallWahbaRot = 3,   // as above -> R 9
    kCallRk4 = 4,        // q0 4, dt 1, w 3 -> q 4
    kCallJacA = 5,       // w 3 -> A 16
    kCallJacB = 6,       // q 4 -> Jb 12
    kCallComparator = 7, // q1 4, q2 4 -> 4
    kCallR2q = 8,        // M 9 -> q 4
};
constexpr int kCallMaxOut = 36;

__host__ __device__ constexpr int call1_outputs(int op) {
    return op == kCallPredict ? 36 : op == kCallCorrect ? 20 : op == kCallWahbaRot ? 9 : op == kCallJacA ? 16
           : op == kCallJacB ? 12 : 4;
}

// One n = 1 call on lane-private operands (the operand order above); status stays 0 for the
// operators that cannot fail.
__device__ __forceinline__ void dispatch1(int op, const double *v, double *o, int32_t *st) {
    switch (op) {
        case kCallPredict: d_predict(v, v + 3, v + 4, v + 8, v + 24, v + 33, o, o + 4, o + 20, st); break;
        case kCallCorrect: d_correct(v, v + 3, v + 6, v + 10, v + 26, v + 42, v + 45, o, o + 4, st); break;
        case kCallWahbaQuat: d_wahba<true>(0, v, v + 3, v + 6, v + 9, v + 12, v + 13, o, st); break;
        case kCallWahbaRot: d_wahba<false>(0, v, v + 3, v + 6, v + 9, v + 12, v + 13, o, st); break;
        case kCallRk4: d_rk4(0, v, v + 4, v + 5, o); break;
        case kCallJacA: d_jac_a(0, v, o); break;
        case kCallJacB: d_jac_b(0, v, o); break;
        case kCallComparator: d_comparator(0, v, v + 4, o); break;
        default: d_r2q(0, v, o); break;
    }
}

template <int OP>
__global__ __launch_bounds__(64) void k_call1(Blob b, double *out, int32_t *status, Done done) {
    if (threadIdx.x == 0) {
        double v[kBlobDoubles];
#pragma unroll
        for (int k = 0; k < kBlobDoubles; ++k) v[k] = b.v[k];
        *status = 0;
        dispatch1(OP, v, out, status);
    }
    done.signal();
}

// ---------------------------------------------------------------------------------------------
// Resident per-call service.  A launch per n = 1 call costs a dispatch and a completion signal
// (7.6 us round trip with an empty kernel, scripts/sync_probe.hip); a resident one-wave kernel
// polling a mailbox in coherent pinned host memory answers in ~4 us (scripts/pingpong_probe.hip).
// Mailbox (host memory, mapped):
//   request  [0, 512): 8 lines of 64 B = 7 payload doubles + a stamp word (hash32 of the line's
//            payload << 32 | op << 16 | seq16).  The host writes each line's payload, then its
//            stamp (release); the wave reads all 8 lines with one 512 B load and accepts a request
//            when the 8 stamps agree on a new sequence number AND every line's payload matches its
//            stamp's hash (the memory model does not promise a line to be read as one snapshot).
//   response [1024, ...): outputs (doubles), status, then the sequence number, written last
//            after a system-scope fence; the host polls it in its own memory.
// The kernel always ends: it exits on a stop request or after kSvcIdleMs without a request
// (measured on the constant-rate wall clock); the host restarts it on demand, so a process that
// stops calling leaves nothing running for more than kSvcIdleMs.
constexpr int kSvcLinePayload = 7;
constexpr int kSvcPayload = 8 * kSvcLinePayload;  // 56 doubles
constexpr size_t kSvcRespOff = 1024, kSvcStatusOff = kSvcRespOff + 64 * 8, kSvcSeqOff = kSvcStatusOff + 64;
constexpr size_t kSvcBytes = 2048;
constexpr uint32_t kSvcStop = 0xFFFFu;
constexpr int kSvcIdleMs = 5;

// 32-bit mix of one request word and its position, XORed over a line's 7 payload words into the
// line's stamp; the same function on both sides of the mailbox (32-bit multiplies only).
__host__ __device__ inline uint32_t svc_mix(uint64_t w, uint32_t pos) {
    uint32_t h = ((uint32_t)w ^ (pos * 0x9E3779B9u)) * 0x85EBCA6Bu;
    h ^= ((uint32_t)(w >> 32) + (h >> 15)) * 0xC2B2AE35u;
    return h ^ (h >> 16);
}

// XOR over each group of 8 lanes (DPP: quad_perm [1,0,3,2], [2,3,0,1], then row_half_mirror).
__device__ inline uint32_t xor8(uint32_t h) {
    h ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)h, 0xB1, 0xF, 0xF, false);
    h ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)h, 0x4E, 0xF, 0xF, false);
    h ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)h, 0x141, 0xF, 0xF, false);
    return h;
}

// The request's operation on lane 0, out of line so that the polling loop carries none of its
// hoisted constants (inlined, they were copied through AGPRs on every poll).
__device__ __noinline__ void svc_run(uint32_t op, double *sh, int32_t *sh_status) {
    // the payload as the Blob of k_call1 (same operand order, same device functions)
    double v[kSvcPayload];
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int j = 0; j < kSvcLinePayload; ++j) v[k * kSvcLinePayload + j] = sh[k * 8 + j];
    double o[kCallMaxOut] = {};
    int32_t st = 0;
    dispatch1((int)op, v, o, &st);
#pragma unroll
    for (int k = 0; k < kCallMaxOut; ++k) sh[k] = o[k];  // static indices: o stays in registers
    *sh_status = st;
}

// Prediction and Correction spread over the service wave's lanes.  On lane 0 alone a predict is ~620
// serial FP64 instructions (~0.9 us of a 5.2 us call, scripts/percall_latency.cpp against the bare
// round trip of scripts/pingpong_probe.hip), most of them the 4x4 products.  Here lane l < 16 forms
// entry (l / 4, l % 4) of each product with the source expression matmul<> uses for that entry (a
// dot product from s = 0.0, the same contraction), so every entry rounds as on lane 0: the answers
// stay bit-identical to the launch per call and to the batched kernels (tests/test_percall_service.py).
// The parts with no product structure -- RK4, the cofactor inverse, the Wahba solve -- run on every
// lane at once, which costs what they cost on one.  sx: LDS scratch shared through the wave.
constexpr int kSvcScratch = 112;

// v[lane] for lanes 0..3 without indexing registers by a lane-varying value
__device__ __forceinline__ double pick4(const double *v, int lane) {
    return lane == 0 ? v[0] : lane == 1 ? v[1] : lane == 2 ? v[2] : v[3];
}

__device__ __forceinline__ double dot_row_col(const double *a, int as, const double *b, int bs, int n) {
    double s = 0.0;
    for (int t = 0; t < n; ++t) s += a[t * as] * b[t * bs];  // matmul<>'s entry: s += a * b from 0.0
    return s;
}

// payload index of operand word k (8 lines of 7 doubles; sh[line * 8 + j])
__device__ __forceinline__ constexpr int svc_at(int k) { return (k / kSvcLinePayload) * 8 + k % kSvcLinePayload; }

__device__ __noinline__ void svc_predict_wave(double *sh, double *sx, int32_t *sh_status) {
    const int lane = threadIdx.x, l = lane & 15, i = l >> 2, j = l & 3;
    // operands (d_predict's order: gyro 3, dt 1, X 4, P 16, Q 9, R 16)
    double g[3], dt, x[4];
#pragma unroll
    for (int k = 0; k < 3; ++k) g[k] = sh[svc_at(k)];
    dt = sh[svc_at(3)];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = sh[svc_at(4 + k)];
    double *A = sx, *Jb = sx + 16, *P = sx + 28, *Q = sx + 44, *T = sx + 53, *T12 = sx + 69, *Si = sx + 81;
    if (lane < 16) P[l] = sh[svc_at(8 + l)];
    if (lane < 9) Q[lane] = sh[svc_at(24 + lane)];
    const double R = sh[svc_at(33 + l)];
    if (lane == 0) {
        double a[16], jb[12];
        omega_half(g, a);
        xi_half(x, jb);
#pragma unroll
        for (int k = 0; k < 16; ++k) A[k] = a[k];
#pragma unroll
        for (int k = 0; k < 12; ++k) Jb[k] = jb[k];
    }
    __syncthreads();
    // d_predict_cov: t16 = A P, t12 = Jb Q (lanes 16..27), then P- = t16 A^T + t12 Jb^T
    if (lane < 16) T[l] = dot_row_col(A + 4 * i, 1, P + j, 4, 4);
    if (lane >= 16 && lane < 28) {
        const int r = (lane - 16) / 3, c = (lane - 16) % 3;
        T12[lane - 16] = dot_row_col(Jb + 3 * r, 1, Q + c, 3, 3);
    }
    __syncthreads();
    const double a16 = dot_row_col(T + 4 * i, 1, A + 4 * j, 1, 4);     // (A P) A^T: At[t][j] = A[j][t]
    const double b16 = dot_row_col(T12 + 3 * i, 1, Jb + 3 * j, 1, 3);  // (Jb Q) Jb^T
    const double pm = a16 + b16;
    // d_predict_gain: S = P- + R, z = RK4, K = P- inv(S)
    const double s = pm + R;
    __syncthreads();
    if (lane < 16) {
        T[l] = s;
        P[l] = pm;  // P is no longer needed: it holds P- from here
    }
    __syncthreads();
    double S[16], inv[16], z[4];
#pragma unroll
    for (int k = 0; k < 16; ++k) S[k] = T[k];
    rk4_literal(x, dt, g, z);
    const bool ok = inverse4(S, inv);  // inv is written only when ok
    if (lane == 0 && ok) {
#pragma unroll
        for (int k = 0; k < 16; ++k) Si[k] = inv[k];
    }
    __syncthreads();
    const double kk = ok ? dot_row_col(P + 4 * i, 1, Si + j, 4, 4) : NAN;
    __syncthreads();
    // outputs in the order of call1_outputs: z 4, Pm 16, K 16
    if (lane < 4) sh[lane] = pick4(z, lane);
    if (lane < 16) {
        sh[4 + l] = pm;
        sh[20 + l] = kk;
    }
    if (lane == 0) *sh_status = ok ? 0 : 1;
}

__device__ __noinline__ void svc_correct_wave(double *sh, double *sx, int32_t *sh_status) {
    const int lane = threadIdx.x, l = lane & 15, i = l >> 2, j = l & 3;
    // operands (d_correct's order: mag 3, acc 3, z 4, P 16, K 16, acc0 3, mag0 3)
    double mag[3], acc[3], z[4], a0[3], m0[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        mag[k] = sh[svc_at(k)];
        acc[k] = sh[svc_at(3 + k)];
        a0[k] = sh[svc_at(42 + k)];
        m0[k] = sh[svc_at(45 + k)];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = sh[svc_at(6 + k)];
    double *P = sx, *K = sx + 16;
    if (lane < 16) {
        P[l] = sh[svc_at(10 + l)];
        K[l] = sh[svc_at(26 + l)];
    }
    __syncthreads();
    // d_correct_cov: P - K P, one entry per lane
    const double pout = P[l] - dot_row_col(K + 4 * i, 1, P + j, 4, 4);
    // d_correct_measure + d_correct_state on every lane (the same values on each)
    double y[4], kr[16], X[4];
    int32_t st = 0;
    d_correct_measure(mag, acc, z, a0, m0, y, &st);
#pragma unroll
    for (int k = 0; k < 16; ++k) kr[k] = K[k];
    d_correct_state(y, z, kr, X);
    __syncthreads();
    // outputs: X 4, P 16
    if (lane < 4) sh[lane] = pick4(X, lane);
    if (lane < 16) sh[4 + l] = pout;
    if (lane == 0) *sh_status = st;
}

__global__ __launch_bounds__(64) void k_service(char *box, unsigned long long idle_ticks) {
    __shared__ double sh[64];
    __shared__ double sx[kSvcScratch];
    __shared__ int32_t sh_status;
    const int lane = threadIdx.x;
    const uint64_t *req = reinterpret_cast<const uint64_t *>(box);
    double *resp = reinterpret_cast<double *>(box + kSvcRespOff);
    int32_t *resp_status = reinterpret_cast<int32_t *>(box + kSvcStatusOff);
    uint32_t *resp_seq = reinterpret_cast<uint32_t *>(box + kSvcSeqOff);
    uint32_t done = __hip_atomic_load(resp_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned long long t0 = wall_clock64();
    for (;;) {
        const uint64_t w = __hip_atomic_load(req + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
        const uint32_t tag = __builtin_amdgcn_readlane(lo, 7);
        const uint32_t seq = tag & 0xFFFFu, op = tag >> 16;
        bool wait = seq == done || __any((lane & 7) == 7 && lo != tag);
        if (!wait) {
            // Every line's stamp carries a hash of that line's 7 payload words (svc_mix): a line
            // whose payload words predate its stamp -- the memory model does not promise a 64 B
            // line to be read as one snapshot -- fails it and is read again at the next poll.  (A
            // seqlock re-read behind an acquire fence would cost one more PCIe round trip per
            // call: measured +1.2 us.)
            const uint32_t h = xor8((lane & 7) == 7 ? 0u : svc_mix(w, (uint32_t)lane));
            wait = __any((lane & 7) == 7 && h != hi);
        }
        if (wait) {
            if (wall_clock64() - t0 > idle_ticks) break;  // uniform
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        if (op == kSvcStop) {
            if (lane == 0) __hip_atomic_store(resp_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        sh[lane] = __longlong_as_double((long long)w);
        __syncthreads();
        const int n_out = call1_outputs((int)op);
        if (op == kCallPredict)
            svc_predict_wave(sh, sx, &sh_status);  // op is wave-uniform: every lane takes part
        else if (op == kCallCorrect)
            svc_correct_wave(sh, sx, &sh_status);
        else if (lane == 0)
            svc_run(op, sh, &sh_status);
        __syncthreads();
        if (lane < n_out) __hip_atomic_store(resp + lane, sh[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (lane == 0) __hip_atomic_store(resp_status, sh_status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __syncthreads();
        if (lane == 0) __hip_atomic_store(resp_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        done = seq;
        t0 = wall_clock64();
    }
}

// Host side: one service per device, shared by the process's threads (calls serialise on a mutex).
class Service {
  public:
    static std::atomic<int> &mode() {
        static std::atomic<int> m{[] {
            const char *e = std::getenv("PEKF_PERCALL");
            return e && std::strcmp(e, "launch") == 0 ? PEKF_PERCALL_LAUNCH : PEKF_PERCALL_SERVICE;
        }()};
        return m;
    }

    static Service *get() {  // nullptr: launch mode, or the service is unavailable
        if (mode().load() != PEKF_PERCALL_SERVICE) return nullptr;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
        Service &s = instances()[dev];  // instance dev serves device dev (set once, at construction)
        return s.broken_.load() ? nullptr : &s;
    }

    // One request: n_in doubles in, n_out doubles out.  Returns PEKF_OK, or an error (the caller
    // then falls back to a launch).
    int call(uint32_t op, const double *in, size_t n_in, double *out, int n_out, int32_t *status) {
        std::lock_guard<std::mutex> g(m_);
        if (int st = ensure_running()) return st;
        post(op, in, n_in);
        if (int st = await(true)) return st;
        const double *r = reinterpret_cast<const double *>(box_ + kSvcRespOff);
        std::memcpy(out, r, (size_t)n_out * sizeof(double));
        *status = *reinterpret_cast<volatile int32_t *>(box_ + kSvcStatusOff);
        last_ = std::chrono::steady_clock::now();
        return PEKF_OK;
    }

    // Stop the resident kernel (before a device-wide synchronisation, at exit).
    void quiesce() {
        std::lock_guard<std::mutex> g(m_);
        stop_locked();
    }

    static void quiesce_all();

  private:
    static constexpr int kMaxDevices = 16;
    static Service *instances() {
        static Service *per_device = [] {
            static Service all[kMaxDevices];
            for (int i = 0; i < kMaxDevices; ++i) all[i].dev_ = i;  // its wall-clock rate sets the idle limit
            return all;
        }();
        return per_device;
    }

    int ensure_running() {
        if (!box_) {
            if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess ||
                hipHostMalloc(reinterpret_cast<void **>(&box_), kSvcBytes, hipHostMallocMapped | hipHostMallocCoherent) !=
                    hipSuccess ||
                hipHostGetDevicePointer(reinterpret_cast<void **>(&box_dev_), box_, 0) != hipSuccess) {
                broken_ = true;
                return set_error(PEKF_ERR_HIP, "per-call service: setup failed");
            }
            std::memset(box_, 0, kSvcBytes);
            int khz = 0;
            if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_) != hipSuccess || khz <= 0) khz = 100000;
            idle_ticks_ = (unsigned long long)khz * kSvcIdleMs;
            static std::once_flag once;
            std::call_once(once, [] { std::atexit(Service::quiesce_all); });
        }
        // past half the idle period the kernel may be about to leave: restart it deliberately
        if (running_ && std::chrono::steady_clock::now() - last_ > std::chrono::microseconds(kSvcIdleMs * 500)) stop_locked();
        if (!running_) return launch();
        return PEKF_OK;
    }

    int launch() {
        hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, stream_, box_dev_, idle_ticks_);
        if (hipGetLastError() != hipSuccess) {
            broken_ = true;
            return set_error(PEKF_ERR_HIP, "per-call service: launch failed");
        }
        running_ = true;
        last_ = std::chrono::steady_clock::now();
        return PEKF_OK;
    }

    void post(uint32_t op, const double *in, size_t n_in) {
        seq_ = (seq_ + 1) & 0xFFFFu;  // 16-bit sequence number: the stamp's low half is op << 16 | seq
        const uint32_t tag = (op << 16) | seq_;
        for (int k = 0; k < 8; ++k) {
            double *line = reinterpret_cast<double *>(box_ + 64 * k);
            uint32_t h = 0;
            for (int j = 0; j < kSvcLinePayload; ++j) {
                const size_t i = (size_t)k * kSvcLinePayload + j;
                line[j] = i < n_in ? in[i] : 0.0;
                uint64_t bits;
                std::memcpy(&bits, &line[j], sizeof bits);
                h ^= svc_mix(bits, (uint32_t)(8 * k + j));
            }
            __atomic_store_n(reinterpret_cast<uint64_t *>(line + 7), ((uint64_t)h << 32) | tag, __ATOMIC_RELEASE);
        }
    }

    // Wait for the answer to seq_.  If the kernel ended without answering (it reached its idle
    // limit as the request was posted), restart it: the new kernel picks the request up.
    int await(bool restart) {
        volatile uint32_t *rs = reinterpret_cast<volatile uint32_t *>(box_ + kSvcSeqOff);
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned it = 0;; ++it) {
            if (__atomic_load_n(rs, __ATOMIC_ACQUIRE) == seq_) return PEKF_OK;
            if ((it & 255u) != 255u) continue;
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt < std::chrono::microseconds(200)) continue;
            if (hipStreamQuery(stream_) == hipSuccess) {  // the kernel has ended
                running_ = false;
                if (__atomic_load_n(rs, __ATOMIC_ACQUIRE) == seq_) return PEKF_OK;
                if (!restart) {
                    __atomic_store_n(const_cast<uint32_t *>(rs), seq_, __ATOMIC_RELEASE);
                    return PEKF_OK;
                }
                if (int st = launch()) return st;
                restart = false;  // at most one restart per request
            } else if (dt > std::chrono::seconds(2)) {
                broken_ = true;
                return set_error(PEKF_ERR_HIP, "per-call service: no answer within 2 s");
            }
        }
    }

    void stop_locked() {
        if (!running_) return;
        if (hipStreamQuery(stream_) == hipSuccess) {  // already left at its idle limit
            running_ = false;
            return;
        }
        post(kSvcStop, nullptr, 0);
        (void)await(false);
        (void)hipStreamSynchronize(stream_);
        running_ = false;
    }

    std::mutex m_;
    hipStream_t stream_ = nullptr;
    char *box_ = nullptr, *box_dev_ = nullptr;
    unsigned long long idle_ticks_ = 0;
    int dev_ = 0;
    uint32_t seq_ = 0;
    std::atomic<bool> running_{false};  // read without the lock by quiesce_all
    std::atomic<bool> broken_{false};  // read without the lock by get()
    std::chrono::steady_clock::time_point last_;
};

// only devices whose service kernel is running are touched (no context is created elsewhere)
void Service::quiesce_all() {
    Service *all = instances();
    int cur = -1;
    for (int d = 0; d < kMaxDevices; ++d) {
        if (!all[d].running_.load()) continue;
        if (cur < 0 && hipGetDevice(&cur) != hipSuccess) return;
        if (hipSetDevice(d) != hipSuccess) continue;
        all[d].quiesce();
    }
    if (cur >= 0) (void)hipSetDevice(cur);
}

void service_quiesce_all() { Service::quiesce_all(); }

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
    // the resident service when it is available, a launch of k_call1 otherwise (same d_* bodies)
    Service *svc = off <= kSvcPayload * sizeof(double) ? Service::get() : nullptr;
    if (svc) {
        if (svc->call(OP, b.v, off / sizeof(double), tmp, (int)(ob / sizeof(double)), status) == PEKF_OK) {
            off = 0;
            for (const HostOut &o : outs) {
                std::memcpy(o.ptr, reinterpret_cast<char *>(tmp) + off, o.bytes);
                off += o.bytes;
            }
            return PEKF_OK;
        }
    }
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

int pekf_set_percall_mode(int mode) {
    PEKF_CHECK_ARG(mode == PEKF_PERCALL_SERVICE || mode == PEKF_PERCALL_LAUNCH, "unknown per-call mode");
    if (mode == PEKF_PERCALL_LAUNCH) service_quiesce_all();
    Service::mode().store(mode);
    return PEKF_OK;
}

int pekf_get_percall_mode(int *mode) {
    PEKF_CHECK_ARG(mode, "mode is NULL");
    *mode = Service::mode().load();
    return PEKF_OK;
}

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
    if (n == 1) {
        int32_t st1 = 0;
        return call1<kCallRk4>({{q0, 32}, {dt_ns, 8}, {w, 24}}, {{q_out, 32}}, &st1);
    }
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
    if (n == 1) {
        int32_t st1 = 0;
        return call1<kCallJacA>({{w, 24}}, {{A, 128}}, &st1);
    }
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
    if (n == 1) {
        int32_t st1 = 0;
        return call1<kCallJacB>({{q, 32}}, {{Jb, 96}}, &st1);
    }
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
    if (n == 1) {
        int32_t st1 = 0;
        return call1<kCallComparator>({{q1, 32}, {q2, 32}}, {{res, 32}}, &st1);
    }
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
    if (n == 1) {
        int32_t st1 = 0;
        const std::initializer_list<HostArg> ins = {{acc0, 3 * b}, {mag0, 3 * b}, {acc, 3 * b}, {mag, 3 * b},
                                                    {k_acc, b}, {k_mag, b}};
        const int st = quat ? call1<kCallWahbaQuat>(ins, {{res, 4 * b}}, &st1)
                            : call1<kCallWahbaRot>(ins, {{res, 9 * b}}, &st1);
        if (st) return st;
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
    if (n == 1) {
        int32_t st1 = 0;
        return call1<kCallR2q>({{M, 72}}, {{q, 32}}, &st1);
    }
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
