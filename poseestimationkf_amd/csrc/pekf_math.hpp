// pekf_math.hpp -- FP64 device math of the quaternion EKF (gfx950, one lane per filter).
//
// Two families:
//  * literal building blocks that keep the reference's dense formulation, used by the
//    per-call kernels behind the drop-in API (results agree with NumPy to ~1e-15);
//  * the lane-resident forms used by the fused kernel, which exploit the algebra of the
//    reference model to cut the FP64 work per step (DESIGN.md "Fused step algebra"):
//      - 0.5*Omega(w) squares to -(|w|^2/4) I, so classical RK4 (ExtendedKalmanFilter.py:25-41)
//        is exactly  q1 = (1 - x/2 + x^2/24) q + h (1 - x/6) 0.5*Omega(w) q,  x = h^2 |w|^2 / 4;
//      - Xi(q) Xi(q)^T = |q|^2 I - q q^T, so Jb Q Jb^T = (q_scale/4)(|X|^2 I - X X^T) (:51-56,61);
//      - S = P- + rI is SPD, K = P- S^-1 = I - r S^-1 and P- - K P- = r K (:63-66,78);
//      - B (Wahba.py:11-13) has rank 2: its SVD rotation is R = Fw diag(P2, c) Fv^T with Fw, Fv
//        the Gram-Schmidt frames of (acc0, mag0) and (acc, mag), P2 the orthogonal polar factor
//        of the 2x2 core C = Fw^T B Fv and c = sign(det C) = sign(k_acc k_mag) (Wahba.py:14-16).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#define PEKF_DEV __device__ __forceinline__

// Rarely taken fallback branches of the fused step: PEKF_TAKEN(cond, c) is cond, marked unlikely (the
// fallback bodies are placed after the loop, so the common path falls straight through), except in the
// instruction-count build (make asm-common, -DPEKF_ISA_COMMON_PATH), where it is the constant c of
// the path a tracked lane takes, so scripts/isa_count.py counts what actually executes.
#ifdef PEKF_ISA_COMMON_PATH
#define PEKF_TAKEN(cond, common) (common)
#else
#define PEKF_TAKEN(cond, common) __builtin_expect(!!(cond), 0)
#endif

namespace pekf {

constexpr double kNsToS = 1e-09;  // ExtendedKalmanFilter.py:32 (10**-9)
constexpr double kSqrt2 = 1.4142135623730951;

// ------------------------------- literal (per-call) forms -------------------------------------

// 0.5*Omega(w), ExtendedKalmanFilter.py:27-30 and :44-47
PEKF_DEV void omega_half(const double *w, double *A) {
    A[0] = 0.0;          A[1] = -0.5 * w[0];  A[2] = -0.5 * w[1];  A[3] = -0.5 * w[2];
    A[4] = 0.5 * w[0];   A[5] = 0.0;          A[6] = 0.5 * w[2];   A[7] = -0.5 * w[1];
    A[8] = 0.5 * w[1];   A[9] = -0.5 * w[2];  A[10] = 0.0;         A[11] = 0.5 * w[0];
    A[12] = 0.5 * w[2];  A[13] = 0.5 * w[1];  A[14] = -0.5 * w[0]; A[15] = 0.0;
}

// 0.5*Xi(q), ExtendedKalmanFilter.py:52-55
PEKF_DEV void xi_half(const double *q, double *J) {
    J[0] = -0.5 * q[1];  J[1] = -0.5 * q[2];  J[2] = -0.5 * q[3];
    J[3] = 0.5 * q[0];   J[4] = 0.5 * q[3];   J[5] = -0.5 * q[2];
    J[6] = -0.5 * q[3];  J[7] = 0.5 * q[0];   J[8] = 0.5 * q[1];
    J[9] = 0.5 * q[2];   J[10] = -0.5 * q[1]; J[11] = 0.5 * q[0];
}

template <int N, int K, int M>
PEKF_DEV void matmul(const double *a, const double *b, double *c) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < M; ++j) {
            double s = 0.0;
#pragma unroll
            for (int t = 0; t < K; ++t) s += a[i * K + t] * b[t * M + j];
            c[i * M + j] = s;
        }
}

template <int N, int M>
PEKF_DEV void transpose(const double *a, double *at) {
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < M; ++j) at[j * N + i] = a[i * M + j];
}

// UtilityFunctions.norm (UtilityFunctions.py:16-21): sequential sum of squares
PEKF_DEV double loop_norm4(const double *a) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s += a[i] * a[i];
    return sqrt(s);
}

// Classical 4-stage RK4 (ExtendedKalmanFilter.py:25-41)
PEKF_DEV void rk4_literal(const double *q0, double dt_ns, const double *w, double *out) {
    double W[16], k1[4], k2[4], k3[4], k4[4], t[4];
    omega_half(w, W);
    const double h = dt_ns * kNsToS;
    matmul<4, 4, 1>(W, q0, k1);
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i] = q0[i] + h / 2 * k1[i];
    matmul<4, 4, 1>(W, t, k2);
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i] = q0[i] + h / 2 * k2[i];
    matmul<4, 4, 1>(W, t, k3);
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i] = q0[i] + h * k3[i];
    matmul<4, 4, 1>(W, t, k4);
    const double c = 1.0 / 6.0 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = q0[i] + c * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
    const double n = loop_norm4(out);
#pragma unroll
    for (int i = 0; i < 4; ++i) out[i] = out[i] / n;
}

// General 4x4 inverse by 2x2 cofactors (np.linalg.inv at ExtendedKalmanFilter.py:65).
// Returns false iff the determinant is exactly zero (LinAlgError "Singular matrix").
PEKF_DEV bool inverse4(const double *m, double *inv) {
    const double s0 = m[0] * m[5] - m[4] * m[1];
    const double s1 = m[0] * m[6] - m[4] * m[2];
    const double s2 = m[0] * m[7] - m[4] * m[3];
    const double s3 = m[1] * m[6] - m[5] * m[2];
    const double s4 = m[1] * m[7] - m[5] * m[3];
    const double s5 = m[2] * m[7] - m[6] * m[3];
    const double c5 = m[10] * m[15] - m[14] * m[11];
    const double c4 = m[9] * m[15] - m[13] * m[11];
    const double c3 = m[9] * m[14] - m[13] * m[10];
    const double c2 = m[8] * m[15] - m[12] * m[11];
    const double c1 = m[8] * m[14] - m[12] * m[10];
    const double c0 = m[8] * m[13] - m[12] * m[9];
    const double det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
    if (det == 0.0) return false;  // LAPACK raises only on an exactly singular pivot; NaN/inf propagate
    const double id = 1.0 / det;
    inv[0] = (m[5] * c5 - m[6] * c4 + m[7] * c3) * id;
    inv[1] = (-m[1] * c5 + m[2] * c4 - m[3] * c3) * id;
    inv[2] = (m[13] * s5 - m[14] * s4 + m[15] * s3) * id;
    inv[3] = (-m[9] * s5 + m[10] * s4 - m[11] * s3) * id;
    inv[4] = (-m[4] * c5 + m[6] * c2 - m[7] * c1) * id;
    inv[5] = (m[0] * c5 - m[2] * c2 + m[3] * c1) * id;
    inv[6] = (-m[12] * s5 + m[14] * s2 - m[15] * s1) * id;
    inv[7] = (m[8] * s5 - m[10] * s2 + m[11] * s1) * id;
    inv[8] = (m[4] * c4 - m[5] * c2 + m[7] * c0) * id;
    inv[9] = (-m[0] * c4 + m[1] * c2 - m[3] * c0) * id;
    inv[10] = (m[12] * s4 - m[13] * s2 + m[15] * s0) * id;
    inv[11] = (-m[8] * s4 + m[9] * s2 - m[11] * s0) * id;
    inv[12] = (-m[4] * c3 + m[5] * c1 - m[6] * c0) * id;
    inv[13] = (m[0] * c3 - m[1] * c1 + m[2] * c0) * id;
    inv[14] = (-m[12] * s3 + m[13] * s1 - m[14] * s0) * id;
    inv[15] = (m[8] * s3 - m[9] * s1 + m[10] * s0) * id;
    return true;
}

// Wahba.RotationMatrix2Quart (Wahba.py:19-47): 3 branches, strict '>' ties, no trace branch.
// Evaluated without contraction and with true division: bit-identical to the reference
// for the same M (tests/test_gpu_parity.py::test_r2q_bit_exact).
PEKF_DEV void rotm_to_quat(const double *M, double *q) {
#pragma clang fp contract(off)
    const double t1 = ((1.0 + M[0]) - M[4]) - M[8];
    const double t2 = ((1.0 - M[0]) + M[4]) - M[8];
    const double t3 = ((1.0 - M[0]) - M[4]) + M[8];
    if (t1 > t2 && t1 > t3) {
        const double S = sqrt(t1) * 2.0;
        q[0] = (M[7] - M[5]) / S; q[1] = 0.25 * S; q[2] = (M[1] + M[3]) / S; q[3] = (M[2] + M[6]) / S;
    } else if (t2 > t1 && t2 > t3) {
        const double S = sqrt(t2) * 2.0;
        q[0] = (M[2] - M[6]) / S; q[1] = (M[1] + M[3]) / S; q[2] = 0.25 * S; q[3] = (M[5] + M[7]) / S;
    } else {
        const double S = sqrt(t3) * 2.0;
        q[0] = (M[3] - M[1]) / S; q[1] = (M[2] + M[6]) / S; q[2] = (M[5] + M[7]) / S; q[3] = 0.25 * S;
    }
}

// ------------------------------- reciprocal / rsqrt ------------------------------------------
// FAST = false: IEEE division and sqrt (per-call kernels).  FAST = true (fused kernel): the
// hardware v_rcp_f64 / v_rsq_f64 seed (measured on MI355X: <= 5.6e-8 relative) plus ONE Newton
// step, measured <= 11 ulp (rcp) / <= 19 ulp (rsq), i.e. <= 4.2e-15 relative, over 1e-6..1e6
// (scripts/probe_fp64.hip); a second step would give 0 / 2 ulp for 4 more FP64 ops each.
// No scale / fixup sequences: operands here are positive and normal (DESIGN.md "FP64 budget").
constexpr int kNewtonSteps = 1;

template <bool FAST>
PEKF_DEV double recip(double x) {
    if (!FAST) return 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
#pragma unroll
    for (int it = 0; it < kNewtonSteps; ++it) r = fma(r, fma(-x, r, 1.0), r);
    return r;
}

// ------------------------------- VOP3 output modifier (omod) ---------------------------------
// An exact halving folded into the instruction that produces the value (omod div:2): no separate
// v_mul_f64 by 0.5.  The hardware applies omod only with the MODE register's IEEE bit clear and
// FP64 denormals flushed (scripts/omod_probe.hip, profiles/r2/probes/omod_probe.txt: with either
// left at the compute default the modifier is silently ignored), so only code between
// OmodMode::enter() and leave() may use these.  Halving commutes with rounding, so each result is
// bit-identical to the multiply by 0.5 it replaces; none of the values is denormal, and the one
// difference -- omod turns -0 into +0 -- reaches no result (it only ever feeds further sums).
PEKF_DEV double fma_half(double a, double b, double c) {  // (a b + c) / 2
    double d;
    asm("v_fma_f64 %0, %1, %2, %3 div:2" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
PEKF_DEV double fma_half_nc(double a, double b, double c) {  // (a b - c) / 2
    double d;
    asm("v_fma_f64 %0, %1, %2, -%3 div:2" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
PEKF_DEV double mul_half(double a, double b) {  // a b / 2
    double d;
    asm("v_mul_f64 %0, %1, %2 div:2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
PEKF_DEV double add_half(double a, double b) {  // (a + b) / 2
    double d;
    asm("v_add_f64 %0, %1, %2 div:2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
PEKF_DEV double sub_half(double a, double b) {  // (a - b) / 2
    double d;
    asm("v_add_f64 %0, %1, -%2 div:2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
PEKF_DEV double newton_half(double t, double y) {  // (t y + 1) / 2
    double d;
    asm("v_fma_f64 %0, %1, %2, 1.0 div:2" : "=v"(d) : "v"(t), "v"(y));
    return d;
}

// MODE register (hwreg 1) bits 9:6 = IEEE, DX10_CLAMP, FP_DENORM(f64/f16) hi/lo.  enter() clears
// IEEE and flushes FP64/FP16 denormals (DX10_CLAMP kept), leave() restores what the wave had.  The
// compiler models s_setreg of MODE as a definition every FP instruction reads, so no arithmetic
// moves across either call.  Away from min/max (not used between them) and denormal values (none
// arise: every quantity is a normalised sensor sample, a unit quaternion, a covariance entry of
// order r or their products), the arithmetic is that of the default mode.
struct OmodMode {
    static constexpr int kField = 1 | (6 << 6) | (3 << 11);  // hwreg(HW_REG_MODE, 6, 4)
    unsigned saved = 0;
    PEKF_DEV void enter() {
        saved = (unsigned)__builtin_amdgcn_s_getreg(kField);
        __builtin_amdgcn_s_setreg(kField, (int)(saved & 0x4u));
    }
    PEKF_DEV void leave() const { __builtin_amdgcn_s_setreg(kField, (int)saved); }
};

// FAST = 0: IEEE; 1: hardware seed + one Newton step; 2: the same step with its 1/2 folded into
// the fma by omod (bit-identical to 1; only inside OmodMode).
template <int FAST>
PEKF_DEV double rsqrt(double x) {
    if (!FAST) return 1.0 / sqrt(x);
    double y = __builtin_amdgcn_rsq(x);
#pragma unroll
    for (int it = 0; it < kNewtonSteps; ++it) {
        if (FAST == 2) {
            y = fma(y, newton_half(-x * y, y), y);  // (1 - x y^2) / 2 in one instruction
        } else {
            const double e = fma(-x * y, y, 1.0);  // 1 - x y^2
            y = fma(y, 0.5 * e, y);
        }
    }
    return y;
}

// ------------------------------- Wahba closed form -------------------------------------------

// Orthonormal frame of a vector pair (a, m): e1 = a/|a|, e2 = GramSchmidt(m), u3 = e1 x e2,
// with the coordinates of a and m in it: a = alpha e1, m = beta1 e1 + beta2 e2.
// sg = -1 gives the frame [e1, -e2, -u3] (beta2 -> -beta2), still proper: see wahba_rotation.
// Only the sign bit of sg is used (any value whose sign is wahba_sign's will do).
struct Frame {
    double e1[3], e2[3], u3[3];
    double alpha, beta1, beta2;
};

template <int FAST = 0>
PEKF_DEV void make_frame(const double *a, const double *m, Frame &F, double sg = 1.0) {
    const double sa = a[0] * a[0] + a[1] * a[1] + a[2] * a[2];
    const double ia = rsqrt<FAST>(sa);
    F.e1[0] = a[0] * ia; F.e1[1] = a[1] * ia; F.e1[2] = a[2] * ia;
    const double b1 = F.e1[0] * m[0] + F.e1[1] * m[1] + F.e1[2] * m[2];
    const double t0 = m[0] - b1 * F.e1[0], t1 = m[1] - b1 * F.e1[1], t2 = m[2] - b1 * F.e1[2];
    const double sb = t0 * t0 + t1 * t1 + t2 * t2;
    const double ib = copysign(rsqrt<FAST>(sb), sg);
    F.e2[0] = t0 * ib; F.e2[1] = t1 * ib; F.e2[2] = t2 * ib;
    F.u3[0] = F.e1[1] * F.e2[2] - F.e1[2] * F.e2[1];
    F.u3[1] = F.e1[2] * F.e2[0] - F.e1[0] * F.e2[2];
    F.u3[2] = F.e1[0] * F.e2[1] - F.e1[1] * F.e2[0];
    F.alpha = FAST ? sa * ia : sqrt(sa);
    F.beta1 = b1;
    F.beta2 = FAST ? sb * ib : copysign(sqrt(sb), sg);
}

// sign(det C) of the Wahba core below for weights (ka, km): +1 rotation, -1 reflection case.
PEKF_DEV double wahba_sign(double ka, double km) { return ka * km >= 0.0 ? 1.0 : -1.0; }

// R = argmax_{R in SO(3)} tr(R^T B), B = ka acc0 acc^T + km mag0 mag^T (Wahba.py:8-17):
// W = frame of the reference pair (acc0, mag0), V = frame of the current pair (acc, mag) built
// with sg = wahba_sign(ka, km).
//   C = Fw^T B Fv = [[c00, c01], [c10, c11]]: c00 = ka aW aV + km b1W b1V, c01 = km b1W b2V,
//   c10 = km b2W b1V, c11 = km b2W b2V, and det C = ka km aW aV b2W b2V exactly (a, b2 >= 0).
// For det C < 0 the optimum is Fw diag(P2r, -1) Fv^T with P2r the reflection polar factor;
// with the current frame flipped to Fv' = [e1, -e2, -u3] (V.beta2 -> -beta2) this is the
// rotation form R = Fw diag(P2, 1) Fv'^T, P2 = [[p, -s], [s, p]] the polar factor of
// C' = C diag(1, sg): (p, s) = (c00 + c11', c10 - c01'), one formula for both cases.
template <bool FAST = false>
PEKF_DEV void wahba_rotation(const Frame &W, const Frame &V, double ka, double km, double *R) {
    const double kw = km * W.beta2, kb = km * W.beta1;
    double p = ka * W.alpha * V.alpha + kb * V.beta1 + kw * V.beta2;
    double s = kw * V.beta1 - kb * V.beta2;
    const double ih = rsqrt<FAST>(p * p + s * s);
    p *= ih;
    s *= ih;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double g0 = W.e1[i] * p + W.e2[i] * s;     // Fw P2, column 0
        const double g1 = W.e2[i] * p - W.e1[i] * s;     // Fw P2, column 1
#pragma unroll
        for (int j = 0; j < (FAST ? 2 : 3); ++j) R[i * 3 + j] = g0 * V.e1[j] + g1 * V.e2[j] + W.u3[i] * V.u3[j];
    }
    if (FAST) {
        // R is proper orthogonal: its third column is the cross product of the first two
        // (6 operations instead of 9, and V.u3[2] is never needed)
        R[2] = R[3] * R[7] - R[6] * R[4];
        R[5] = R[6] * R[1] - R[0] * R[7];
        R[8] = R[0] * R[4] - R[3] * R[1];
    }
}

// True iff every entry of B = ka acc0 acc^T + km mag0 mag^T is finite (np.linalg.svd raises
// LinAlgError "SVD did not converge" otherwise, Wahba.py:14).
PEKF_DEV bool wahba_b_finite(const double *acc0, const double *mag0, const double *acc,
                             const double *mag, double ka, double km) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) ok &= isfinite(ka * (acc0[i] * acc[j]) + km * (mag0[i] * mag[j]));
    return ok;
}

// A frame whose pair does not span a plane to working accuracy: a zero vector (make_frame divides 0 by
// 0: NaN), or m parallel to a, where Gram-Schmidt's remainder t = m - (m.e1) e1 is rounding noise and e2
// = t/|t| is not orthogonal to e1 (|t| < 1e-12 |m|).  NaN inputs count as degenerate too.
PEKF_DEV bool frame_degenerate(const Frame &F) {
    return !(F.beta2 * F.beta2 > 1e-24 * (F.beta1 * F.beta1 + F.beta2 * F.beta2)) || !(F.e1[0] == F.e1[0]);
}

// ---- Wahba with a rank-deficient B (Wahba.py:8-17) ----
// A zero acc or mag sample, or acc parallel to mag, in either pair makes B = ka acc0 acc^T +
// km mag0 mag^T = w v^T.  Every rotation taking v/|v| to w/|w| attains the optimum tr(R^T B) = |w||v|,
// and np.linalg.svd (Wahba.py:14) picks one of them by the rounding noise of B's zero singular values,
// which no other evaluation reproduces; these take the shortest arc.  B = 0 (both samples zero) gives
// NaN, as the reference does there: its SVD returns U = V = I and RotationMatrix2Quart of the identity
// divides 0 by 0 (Wahba.py:41-46).  Branch-free (selects only): in the fused kernels they run inside
// the rare fallback branch, where a nested divergent branch would hold another exec mask in scalar
// registers across the whole loop.

// a normal of the unit vector v: v x the coordinate axis least aligned with v (not normalised)
PEKF_DEV void normal_of(const double *v, double *n) {
    const double ax = fabs(v[0]), ay = fabs(v[1]), az = fabs(v[2]);
    const bool j0 = ax <= ay && ax <= az, j1 = !j0 && ay <= az;
    n[0] = j0 ? 0.0 : (j1 ? -v[2] : v[1]);
    n[1] = j0 ? v[2] : (j1 ? 0.0 : -v[0]);
    n[2] = j0 ? -v[1] : (j1 ? v[0] : 0.0);
}

// the rotation taking the unit vector v to the unit vector w about v x w (Rodrigues); for w = -v half a
// turn about normal_of(v)
template <int FAST>
PEKF_DEV void shortest_arc(const double *v, const double *w, double *R) {
    const double c = v[0] * w[0] + v[1] * w[1] + v[2] * w[2];
    const double k[3] = {v[1] * w[2] - v[2] * w[1], v[2] * w[0] - v[0] * w[2], v[0] * w[1] - v[1] * w[0]};
    const double sk = k[0] * k[0] + k[1] * k[1] + k[2] * k[2];
    double n[3];
    normal_of(v, n);
    // R = c I + [k]x + (1 - c) h h^T, k = sin(theta) h (h: k's direction, or n where k = 0)
    const bool use_k = sk > 0.0;
    const double ih = rsqrt<FAST>(use_k ? sk : n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    const double h[3] = {(use_k ? k[0] : n[0]) * ih, (use_k ? k[1] : n[1]) * ih, (use_k ? k[2] : n[2]) * ih};
    const double d = 1.0 - c;
    R[0] = c + d * h[0] * h[0];    R[1] = d * h[0] * h[1] - k[2]; R[2] = d * h[0] * h[2] + k[1];
    R[3] = d * h[1] * h[0] + k[2]; R[4] = c + d * h[1] * h[1];    R[5] = d * h[1] * h[2] - k[0];
    R[6] = d * h[2] * h[0] - k[1]; R[7] = d * h[2] * h[1] + k[0]; R[8] = c + d * h[2] * h[2];
}

// Any rank-deficient B (the per-call operators, where either pair may be degenerate): B is formed, its
// longest row gives v's direction and B v the image's.
template <int FAST = 0>
PEKF_DEV void wahba_rank1_rotation(const double *acc0, const double *mag0, const double *acc, const double *mag,
                                   double ka, double km, double *R) {
    double B[9], rn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) B[3 * i + j] = ka * (acc0[i] * acc[j]) + km * (mag0[i] * mag[j]);
        rn[i] = B[3 * i] * B[3 * i] + B[3 * i + 1] * B[3 * i + 1] + B[3 * i + 2] * B[3 * i + 2];
    }
    const bool r0 = rn[0] >= rn[1] && rn[0] >= rn[2], r1 = !r0 && rn[1] >= rn[2];
    const double iv = rsqrt<FAST>(r0 ? rn[0] : (r1 ? rn[1] : rn[2]));
    double v[3], w[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = (r0 ? B[j] : (r1 ? B[3 + j] : B[6 + j])) * iv;
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = B[3 * i] * v[0] + B[3 * i + 1] * v[1] + B[3 * i + 2] * v[2];
    const double iw = rsqrt<FAST>(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    w[0] *= iw; w[1] *= iw; w[2] *= iw;
    shortest_arc<FAST>(v, w, R);
}

// The fused kernels' case: the reference pair spans a plane (it defines the filter's frame) and the
// current one does not.  Then v is acc's direction (mag's where acc = 0), acc = alpha v, mag = beta v and
// w = ka alpha acc0 + km beta mag0: no B, few registers.  v, w unit (NaN where B = 0).
template <int FAST>
PEKF_DEV void current_rank1_directions(const double *acc0, const double *mag0, const double *acc, const double *mag,
                                       double ka, double km, double *v, double *w) {
    const double sa = acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2];
    const bool ua = sa > 0.0;
    const double u[3] = {ua ? acc[0] : mag[0], ua ? acc[1] : mag[1], ua ? acc[2] : mag[2]};
    const double iu = rsqrt<FAST>(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    v[0] = u[0] * iu; v[1] = u[1] * iu; v[2] = u[2] * iu;
    const double al = ka * (acc[0] * v[0] + acc[1] * v[1] + acc[2] * v[2]);
    const double be = km * (mag[0] * v[0] + mag[1] * v[1] + mag[2] * v[2]);
    const double x[3] = {al * acc0[0] + be * mag0[0], al * acc0[1] + be * mag0[1], al * acc0[2] + be * mag0[2]};
    const double ix = rsqrt<FAST>(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    w[0] = x[0] * ix; w[1] = x[1] * ix; w[2] = x[2] * ix;
}

template <int FAST>
PEKF_DEV void wahba_current_rank1(const double *acc0, const double *mag0, const double *acc, const double *mag,
                                  double ka, double km, double *R) {
    double v[3], w[3];
    current_rank1_directions<FAST>(acc0, mag0, acc, mag, ka, km, v, w);
    shortest_arc<FAST>(v, w, R);
}

// wahba_current_rank1's rotation as its quaternion, for the fused kernels' fallback: the shortest arc
// from v to w is q = normalise(1 + v.w, v x w) (w = -v: half a turn, (0, normal_of(v))), in
// RotationMatrix2Quart's convention (R(q) v = w), so no rotation matrix is formed.
template <int FAST>
PEKF_DEV void wahba_current_rank1_quat(const double *acc0, const double *mag0, const double *acc, const double *mag,
                                       double ka, double km, double *q) {
    double v[3], w[3], n[3];
    current_rank1_directions<FAST>(acc0, mag0, acc, mag, ka, km, v, w);
    const double c1 = fma(v[0], w[0], fma(v[1], w[1], fma(v[2], w[2], 1.0)));
    const double k[3] = {v[1] * w[2] - v[2] * w[1], v[2] * w[0] - v[0] * w[2], v[0] * w[1] - v[1] * w[0]};
    normal_of(v, n);
    // w = -v exactly (a NaN w, i.e. B = 0, stays NaN)
    const bool half = !(c1 * c1 + k[0] * k[0] + k[1] * k[1] + k[2] * k[2] > 0.0) && (w[0] == w[0]);
    const double t[4] = {half ? 0.0 : c1, half ? n[0] : k[0], half ? n[1] : k[1], half ? n[2] : k[2]};
    const double it = rsqrt<FAST>(t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3]);
    q[0] = t[0] * it; q[1] = t[1] * it; q[2] = t[2] * it; q[3] = t[3] * it;
}

// the reference pair of a frame built with sg = 1: acc0 = alpha e1, mag0 = beta1 e1 + beta2 e2
PEKF_DEV void frame_pair(const Frame &F, double *a, double *m) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        a[i] = F.alpha * F.e1[i];
        m[i] = F.beta1 * F.e1[i] + F.beta2 * F.e2[i];
    }
}

PEKF_DEV void wahba_rotation_vectors(const double *acc0, const double *mag0, const double *acc,
                                     const double *mag, double ka, double km, double *R) {
    Frame W, V;
    make_frame(acc0, mag0, W);
    make_frame(acc, mag, V, wahba_sign(ka, km));
    if (frame_degenerate(W) || frame_degenerate(V))
        wahba_rank1_rotation(acc0, mag0, acc, mag, ka, km, R);
    else
        wahba_rotation(W, V, ka, km, R);
}

// Branch-free RotationMatrix2Quart for the fused kernel: the reference's branch choice
// (Wahba.py:28,35, strict '>', else branch 3) is made by selects, then ONE rsqrt gives both
// 1/S = 0.5/sqrt(t) and 0.25*S = 0.5*t/sqrt(t).  Agrees with rotm_to_quat to ~1 ulp; at an
// exact identity both give NaNs (which the filter update propagates identically).
// Scaled form: q = v * inv_s with inv_s = 1/S > 0 (the branch's own component of v is t, since
// S/4 = t/S), so a caller that only needs q up to a positive scale first (the hemisphere test
// of ExtendedKalmanFilter.py:73-75) folds the sign into the one scale factor.
PEKF_DEV void rotm_to_quat_scaled(const double *M, double *v, double &inv_s) {
    const double t1 = ((1.0 + M[0]) - M[4]) - M[8];
    const double t2 = ((1.0 - M[0]) + M[4]) - M[8];
    const double t3 = ((1.0 - M[0]) - M[4]) + M[8];
    const bool b1 = (t1 > t2) && (t1 > t3);
    const bool b2 = !b1 && (t2 > t1) && (t2 > t3);
    const bool b3 = !b1 && !b2;
    const double t = b1 ? t1 : (b2 ? t2 : t3);
    inv_s = 0.5 * rsqrt<true>(t);
    const double dw1 = M[7] - M[5], dw2 = M[2] - M[6], dw3 = M[3] - M[1];
    const double sxy = M[1] + M[3], sxz = M[2] + M[6], syz = M[5] + M[7];
    v[0] = b1 ? dw1 : (b2 ? dw2 : dw3);
    v[1] = b1 ? t : (b2 ? sxy : sxz);
    v[2] = b2 ? t : (b1 ? sxy : syz);
    v[3] = b3 ? t : (b1 ? sxz : syz);
}

PEKF_DEV void rotm_to_quat_fast(const double *M, double *q) {
    double v[4], inv_s;
    rotm_to_quat_scaled(M, v, inv_s);
    q[0] = v[0] * inv_s; q[1] = v[1] * inv_s; q[2] = v[2] * inv_s; q[3] = v[3] * inv_s;
}

// v = Q4(M) z with Q4 = 4 q q^T of the rotation M (see rotm_to_quat_toward); nv = |v|^2,
// t0 = 1 + tr M = 4 qw^2
PEKF_DEV void q4_times(const double *M, const double *z, double *v, double &nv, double &t0) {
    const double a = 1.0 + M[8], b = 1.0 - M[8], s = M[0] + M[4], d = M[0] - M[4];
    t0 = a + s;
    const double t1 = b + d, t2 = b - d, t3 = a - s;
    const double dw1 = M[7] - M[5], dw2 = M[2] - M[6], dw3 = M[3] - M[1];
    const double sxy = M[1] + M[3], sxz = M[2] + M[6], syz = M[5] + M[7];
    v[0] = fma(t0, z[0], fma(dw1, z[1], fma(dw2, z[2], dw3 * z[3])));
    v[1] = fma(dw1, z[0], fma(t1, z[1], fma(sxy, z[2], sxz * z[3])));
    v[2] = fma(dw2, z[0], fma(sxy, z[1], fma(t2, z[2], syz * z[3])));
    v[3] = fma(dw3, z[0], fma(sxz, z[1], fma(syz, z[2], t3 * z[3])));
    nv = fma(v[0], v[0], fma(v[1], v[1], fma(v[2], v[2], v[3] * v[3])));
}

// the reference's branch formula and strict '<' hemisphere test (Wahba.py:19-47,
// ExtendedKalmanFilter.py:73-75): Y = v * sc
PEKF_DEV void rotm_to_quat_flip_reference(const double *M, const double *z, double *v, double &sc) {
    double inv_s;
    rotm_to_quat_scaled(M, v, inv_s);
    const double cmp = v[0] * z[0] + v[1] * z[1] + v[2] * z[2] + v[3] * z[3];
    sc = cmp < 0.0 ? -inv_s : inv_s;
}

// Y = RotationMatrix2Quart(M) flipped into z's hemisphere (Wahba.py:19-47, then
// ExtendedKalmanFilter.py:73-75), for the fused kernel, returned as Y = v * sc.  The four candidate numerators of
// RotationMatrix2Quart are the columns of Q4 = 4 q q^T (diagonal 1 +- M00 +- M11 +- M22,
// off-diagonal the sums / differences of M's off-diagonal pairs), so v = Q4 z = 4 q (q.z) is q
// already carrying the sign of q.z: Y = v / |v|, no branch selects and no separate hemisphere
// test.  |v| = 4 |q.z| |z|, so where q is nearly orthogonal to z (|q.z| < 1/4: the measured
// attitude more than 150 degrees from the prediction) and where the reference's own branch
// formula is ill-conditioned (a rotation within ~1e-5 rad of the identity, where it divides by
// ~0 and, at the exact identity, returns NaN) the lane takes the reference's branch formula and
// strict '<' flip instead.  Neither occurs on a tracked stream, so the fallback costs a wave
// nothing unless one of its lanes needs it.
PEKF_DEV void rotm_to_quat_toward(const double *M, const double *z, double *v, double &sc) {
    double nv, t0;
    q4_times(M, z, v, nv, t0);
    sc = rsqrt<true>(nv);  // (the common path carries no data merge with the rare branch)
    if (PEKF_TAKEN(nv < 1.0 || t0 > 4.0 - 1e-10, false))
        rotm_to_quat_flip_reference(M, z, v, sc);  // (NaN operands never get here)
}

// ------------------------------- reference-frame basis ---------------------------------------
// The multi-record stream kernel runs each filter in the basis of its own Wahba reference frame:
// X' = q_W^* (x) X and P' = L(q_W^*) P L(q_W^*)^T, q_W the quaternion of Fw = [e1 e2 u3] of
// (acc0, mag0).  The filter is equivariant under this change of basis: Omega(w) = R(w) is right
// multiplication and commutes with the left multiplication L(q_W^*) (RK4 and A P A^T,
// ExtendedKalmanFilter.py:25-48,61), Xi(q) Xi(q)^T = |q|^2 I - q q^T, R = rI and the hemisphere
// test are invariant under the orthogonal L (:51-56,63-79), and Wahba's rotation becomes
// R' = Fw^T R = diag(P2, 1) Fv^T, whose quaternion is q_W^* (x) Y (Wahba.py:8-47, the quaternion
// of a product being the product of the quaternions).  R' is the current frame's rows rotated by
// P2: p e1 - s e2, s e1 + p e2, u3 -- 12 operations instead of the 36 of Fw diag(P2, 1) Fv^T.
struct RefW {
    static constexpr bool kRefBasis = true;
    double aW, b1W, b2W;  // the reference pair in its own frame: acc0 = (aW, 0, 0), mag0 = (b1W, b2W, 0)
    double q[4];          // q_W
    PEKF_DEV void quat(double *o) const { o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = q[3]; }
};

// quaternion of the proper frame [e1 e2 u3] (columns): Shepperd's largest diagonal of 4 q q^T,
// IEEE arithmetic; once per filter and launch.
PEKF_DEV void frame_quat(const Frame &F, double *q) {
    const double m00 = F.e1[0], m10 = F.e1[1], m20 = F.e1[2];
    const double m01 = F.e2[0], m11 = F.e2[1], m21 = F.e2[2];
    const double m02 = F.u3[0], m12 = F.u3[1], m22 = F.u3[2];
    const double t0 = 1.0 + m00 + m11 + m22, t1 = 1.0 + m00 - m11 - m22;
    const double t2 = 1.0 - m00 + m11 - m22, t3 = 1.0 - m00 - m11 + m22;
    const double w1 = m21 - m12, w2 = m02 - m20, w3 = m10 - m01;
    const double sxy = m01 + m10, sxz = m02 + m20, syz = m12 + m21;
    double v0, v1, v2, v3;
    if (t0 >= t1 && t0 >= t2 && t0 >= t3) {
        v0 = t0; v1 = w1; v2 = w2; v3 = w3;
    } else if (t1 >= t2 && t1 >= t3) {
        v0 = w1; v1 = t1; v2 = sxy; v3 = sxz;
    } else if (t2 >= t3) {
        v0 = w2; v1 = sxy; v2 = t2; v3 = syz;
    } else {
        v0 = w3; v1 = sxz; v2 = syz; v3 = t3;
    }
    const double in = 1.0 / sqrt(v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3);
    q[0] = v0 * in; q[1] = v1 * in; q[2] = v2 * in; q[3] = v3 * in;
}

// RefW whose q_W is recomputed from the filter's reference pair where it is needed (the rare
// |q.z| < 1/4 fallback, the launch's end) instead of being held: 8 fewer live VGPRs in the time loop.
// The recomputation is the same code on the same inputs, so it returns the same q_W bit for bit.
struct RefWLazy {
    static constexpr bool kRefBasis = true;
    double aW, b1W, b2W;
    const double *pair;  // acc0[3], mag0[3] of this filter
    PEKF_DEV void quat(double *o) const {
        Frame F;
        make_frame<true>(pair, pair + 3, F);
        frame_quat(F, o);
    }
};

// y = q (x) x (CONJ = false) or q^* (x) x (CONJ = true), i.e. L(q) x or L(q)^T x
template <bool CONJ>
PEKF_DEV void qmul_left(const double *q, const double *x, double *y) {
    const double q0 = q[0], q1 = CONJ ? -q[1] : q[1], q2 = CONJ ? -q[2] : q[2], q3 = CONJ ? -q[3] : q[3];
    y[0] = q0 * x[0] - q1 * x[1] - q2 * x[2] - q3 * x[3];
    y[1] = q0 * x[1] + q1 * x[0] + q2 * x[3] - q3 * x[2];
    y[2] = q0 * x[2] - q1 * x[3] + q2 * x[0] + q3 * x[1];
    y[3] = q0 * x[3] + q1 * x[2] - q2 * x[1] + q3 * x[0];
}

// rotation matrix of the unit quaternion q (q v q^* = M v)
PEKF_DEV void quat_to_rotm(const double *q, double *M) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    M[0] = 1.0 - 2.0 * (y * y + z * z); M[1] = 2.0 * (x * y - w * z);       M[2] = 2.0 * (x * z + w * y);
    M[3] = 2.0 * (x * y + w * z);       M[4] = 1.0 - 2.0 * (x * x + z * z); M[5] = 2.0 * (y * z - w * x);
    M[6] = 2.0 * (x * z - w * y);       M[7] = 2.0 * (y * z + w * x);       M[8] = 1.0 - 2.0 * (x * x + y * y);
}

// Y' = q_W^* (x) Y for the flipped Wahba quaternion Y of the weights (ka, km), in the reference
// frame's basis (z' the prediction in that basis): Y' = v * sc.  As rotm_to_quat_toward, with its
// |q.z| < 1/4 fallback taken in the world basis (R = Fw R', z = q_W (x) z') so that it is the
// reference's own branch formula and flip.  There is no near-identity fallback here: within
// ~1e-5 rad of the identity the reference's formula divides rounding noise by ~theta, so its
// result differs from ANY other evaluation of the same rotation by ~1e-16/theta (ours included,
// whatever formula we use: R' and numpy's SVD rotation differ in the last bits), and an exactly
// identity world rotation -- the one input where it is deterministic (NaN) -- does not arise from
// Fw R'.  The well-conditioned Q4 z value is returned instead.
struct NoPin {
    PEKF_DEV void operator()() const {}
};
// pin(): called after v = Q4 z and before the fallback branch (see ekf_record_step's PEKF_PIN_SCHUR)
// reload(acc, mag): the record's samples again, for a degenerate current frame only (a zero sample or acc
// parallel to mag, rank-1 B): V is NaN there, so is nv, and the fallback branch -- taken for NaN too --
// solves Wahba by wahba_current_rank1_quat with the reference's weights |acc_z|, 1 - |acc_z|
// (ExtendedKalmanFilter.py:71).  The caller re-reads them (memory, LDS) instead of holding six doubles
// in registers through the Wahba chain.
// wahba_quat_toward (below) in two halves, for ekf_record_step's HOIST schedule (the same arithmetic;
// the one-piece form is kept for every other kernel, whose schedule it fixes).
// The state-independent half: Wahba's rotation R' of the current frame in the reference basis (it
// depends on the record's samples only, not on the prediction z).
template <int F = 1, class RW, std::enable_if_t<RW::kRefBasis, int> = 0>
PEKF_DEV void wahba_rotation_ref(const RW &W, const Frame &V, double ka, double km, double *R) {
    const double kw = km * W.b2W, kb = km * W.b1W;
    double p = ka * W.aW * V.alpha + kb * V.beta1 + kw * V.beta2;
    double s = kw * V.beta1 - kb * V.beta2;
    const double ih = rsqrt<F>(p * p + s * s);
    p *= ih;
    s *= ih;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        R[j] = p * V.e1[j] - s * V.e2[j];
        R[3 + j] = s * V.e1[j] + p * V.e2[j];
        R[6 + j] = V.u3[j];
    }
}

// The z-dependent half: Q4 of R' flipped toward z, with the fallbacks.
template <int F = 1, class RW, class Reload, class Pin = NoPin, std::enable_if_t<RW::kRefBasis, int> = 0>
PEKF_DEV void wahba_toward_from_rotation(const RW &W, const double *R, const double *z, double *v, double &sc,
                                         const Reload &reload, const Pin &pin = Pin()) {
    double nv, t0;
    q4_times(R, z, v, nv, t0);
    sc = rsqrt<F>(nv);
    pin();
    if (PEKF_TAKEN(!(nv >= 1.0), false)) {  // (nv < 1, or NaN)
        double Fw[9], Rw[9], zw[4], vw[4], qw[4];
        W.quat(qw);
        quat_to_rotm(qw, Fw);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) Rw[3 * i + j] = Fw[3 * i] * R[j] + Fw[3 * i + 1] * R[3 + j] + Fw[3 * i + 2] * R[6 + j];
        qmul_left<false>(qw, z, zw);
        rotm_to_quat_flip_reference(Rw, zw, vw, sc);
        qmul_left<true>(qw, vw, v);
        // NaN: a degenerate current frame.  In this basis B' = Fw^T B pairs acc, mag with the reference
        // pair's own coordinates (aW, 0, 0), (b1W, b2W, 0); its shortest-arc attitude, flipped toward z
        // as ExtendedKalmanFilter.py:73-75 flips, replaces the NaN one.
        if (!(nv == nv)) {  // (it overwrites v and sc in place)
            double acc[3], mag[3];
            reload(acc, mag);
            const double a0[3] = {W.aW, 0.0, 0.0}, m0[3] = {W.b1W, W.b2W, 0.0}, kr = fabs(acc[2]);
            wahba_current_rank1_quat<1>(a0, m0, acc, mag, kr, 1.0 - kr, v);
            sc = v[0] * z[0] + v[1] * z[1] + v[2] * z[2] + v[3] * z[3] < 0.0 ? -1.0 : 1.0;
        }
    }
    (void)t0;
}

template <int F = 1, class RW, class Reload, class Pin = NoPin, std::enable_if_t<RW::kRefBasis, int> = 0>
PEKF_DEV void wahba_quat_toward(const RW &W, const Frame &V, double ka, double km, const double *z, double *v,
                                double &sc, const Reload &reload, const Pin &pin = Pin()) {
    const double kw = km * W.b2W, kb = km * W.b1W;
    double p = ka * W.aW * V.alpha + kb * V.beta1 + kw * V.beta2;
    double s = kw * V.beta1 - kb * V.beta2;
    const double ih = rsqrt<F>(p * p + s * s);
    p *= ih;
    s *= ih;
    double R[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        R[j] = p * V.e1[j] - s * V.e2[j];
        R[3 + j] = s * V.e1[j] + p * V.e2[j];
        R[6 + j] = V.u3[j];
    }
    double nv, t0;
    q4_times(R, z, v, nv, t0);
    sc = rsqrt<F>(nv);
    pin();
    if (PEKF_TAKEN(!(nv >= 1.0), false)) {  // (nv < 1, or NaN)
        double Fw[9], Rw[9], zw[4], vw[4], qw[4];
        W.quat(qw);
        quat_to_rotm(qw, Fw);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) Rw[3 * i + j] = Fw[3 * i] * R[j] + Fw[3 * i + 1] * R[3 + j] + Fw[3 * i + 2] * R[6 + j];
        qmul_left<false>(qw, z, zw);
        rotm_to_quat_flip_reference(Rw, zw, vw, sc);
        qmul_left<true>(qw, vw, v);
        // NaN: a degenerate current frame.  In this basis B' = Fw^T B pairs acc, mag with the reference
        // pair's own coordinates (aW, 0, 0), (b1W, b2W, 0); its shortest-arc attitude, flipped toward z
        // as ExtendedKalmanFilter.py:73-75 flips, replaces the NaN one.
        if (!(nv == nv)) {  // (it overwrites v and sc in place)
            double acc[3], mag[3];
            reload(acc, mag);
            const double a0[3] = {W.aW, 0.0, 0.0}, m0[3] = {W.b1W, W.b2W, 0.0}, kr = fabs(acc[2]);
            wahba_current_rank1_quat<1>(a0, m0, acc, mag, kr, 1.0 - kr, v);
            sc = v[0] * z[0] + v[1] * z[1] + v[2] * z[2] + v[3] * z[3] < 0.0 ? -1.0 : 1.0;
        }
    }
    (void)t0;
}

// Y = v * sc in the world basis (the per-record kernels)
template <int F = 1, class Reload, class Pin = NoPin>
PEKF_DEV void wahba_quat_toward(const Frame &W, const Frame &V, double ka, double km, const double *z, double *v,
                                double &sc, const Reload &reload, const Pin & = Pin()) {
    double R[9], nv, t0;
    wahba_rotation<true>(W, V, ka, km, R);
    q4_times(R, z, v, nv, t0);
    sc = rsqrt<true>(nv);
    // rotm_to_quat_toward's fallback, taken for NaN too (a degenerate current frame: rank-1 B)
    if (PEKF_TAKEN(!(nv >= 1.0) || t0 > 4.0 - 1e-10, false)) {
        rotm_to_quat_flip_reference(R, z, v, sc);
        // NaN: a degenerate current frame, solved from the re-read samples (see the reference-basis form)
        if (!(nv == nv)) {
            double acc[3], mag[3], a0[3], m0[3];
            reload(acc, mag);
            frame_pair(W, a0, m0);
            const double kr = fabs(acc[2]);
            wahba_current_rank1_quat<1>(a0, m0, acc, mag, kr, 1.0 - kr, v);
            sc = v[0] * z[0] + v[1] * z[1] + v[2] * z[2] + v[3] * z[3] < 0.0 ? -1.0 : 1.0;
        }
    }
}

// ------------------------------- fused-step forms --------------------------------------------
// With R = rI the reference recursion (ExtendedKalmanFilter.py:61-66,76-78) is, exactly in
// real arithmetic,
//   P-  = A P A^T + (q_scale / 4) (|X|^2 I - X X^T)
//   S   = P- + rI,   K = I - r S^-1,   P = P- - K P- = r I - r^2 S^-1,   X = z + K e = Y - r S^-1 e
// so only the symmetric S^-1 is formed (no general 4x4 products with K).

// Symmetric 4x4 stored as its upper triangle: 00 01 02 03 11 12 13 22 23 33
template <typename T>
struct Sym4T {
    T a00, a01, a02, a03, a11, a12, a13, a22, a23, a33;
};
using Sym4 = Sym4T<double>;

// M P M^T for M = L(q) (CONJ = false) or L(q)^T (CONJ = true): the covariance in the other basis
template <bool CONJ, typename T>
PEKF_DEV Sym4T<T> sym_rotate(const double *q, const Sym4T<T> &S) {
    const double p[4][4] = {{S.a00, S.a01, S.a02, S.a03}, {S.a01, S.a11, S.a12, S.a13},
                            {S.a02, S.a12, S.a22, S.a23}, {S.a03, S.a13, S.a23, S.a33}};
    double t[4][4], o[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // columns of M P (P symmetric: row j = column j)
        double c[4];
        qmul_left<CONJ>(q, p[j], c);
#pragma unroll
        for (int i = 0; i < 4; ++i) t[i][j] = c[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) qmul_left<CONJ>(q, t[i], o[i]);  // (M P) M^T: row i = M (row i of M P)
    return {(T)o[0][0], (T)o[0][1], (T)o[0][2], (T)o[0][3], (T)o[1][1],
            (T)o[1][2], (T)o[1][3], (T)o[2][2], (T)o[2][3], (T)o[3][3]};
}

// single-precision reciprocal for the opt-in mixed-precision covariance path: v_rcp_f32
// (1 ulp) + one Newton step
template <bool FAST>
PEKF_DEV float recip(float x) {
    if (!FAST) return 1.0f / x;
    float r = __builtin_amdgcn_rcpf(x);
    return fmaf(r, fmaf(-x, r, 1.0f), r);
}

// Innovation covariance S = A P A^T + g (|x|^2 I - x x^T) + rI, A = Omega(h), h = w/2
// (ExtendedKalmanFilter.py:44-47,52-55,61,63), returned DOUBLED: 2S, every entry exactly twice
// S's (a power-of-two factor commutes with rounding), so that the gyro enters only as w (the raw
// sample) and h -- S itself would need w/4 as well.  g2 = 2g, r2 = 2r; n2 = |x|^2 (shared with
// rk4_closed's normalisation); th2 = |h|^2; g2x = 2g / |x|^2 for an x that stands for the unit
// x / |x| (g2 otherwise).  The caller folds the factor into its constants:
// (2S)^-1 = S^-1 / 2 exactly, and the update (X normalised, P = rI - r^2 S^-1) is unchanged.
//
// Omega(h) is the matrix of right multiplication by the pure quaternion h, v -> v (x) h.  In the
// basis {I, L(e_a) R(e_b)} (a, b = 1..3) of symmetric 4x4 matrices, P = c0 I + sum C_ab L(e_a) R(e_b)
// with C_ab = tr(L(e_a) R(e_b) P) / 4, conjugation by R(h) maps e_b -> h e_b h^* = 2(h.e_b) h - |h|^2 e_b,
// so C -> 2 (C h) h^T - |h|^2 C and
//   A P A^T = 2 L(u) R(h) - |h|^2 P + 2 |h|^2 c0 I,   u = C h,
//   L(u) R(h) = [[-u.h, (u x h)^T], [u x h, (u.h) I - u h^T - h u^T]].
// u needs only the trace butterflies of P's diagonal and the sums / differences of its off-diagonal
// pairs: 71 FP64 operations for 2S against 96 for the direct Omega P Omega^T + Jb Q Jb^T + rI.
template <typename T>
PEKF_DEV Sym4T<T> innovation_cov2(const Sym4T<T> &P, const T *h, const T *w, T th2, const T *x, T n2, T g2, T r2,
                                  T g2x) {
    // U = 4u, U_a = D_aa h_a + sum_{b != a} D_ab h_b with D_ab = tr(L(e_a) R(e_b) P):
    //   D_11 = -P00 - P11 + P22 + P33, D_22 = -P00 + P11 - P22 + P33, D_33 = -P00 + P11 + P22 - P33,
    //   D_12 = 2(P03 - P12), D_21 = -2(P03 + P12), D_13 = -2(P02 + P13), D_31 = 2(P02 - P13),
    //   D_23 = 2(P01 - P23), D_32 = -2(P01 + P23)
    const T sp = P.a00 + P.a11, dp = P.a11 - P.a00, sq = P.a22 + P.a33, dq = P.a22 - P.a33;
    const T tr = sp + sq, d11 = sq - sp, d22 = dp - dq, d33 = dp + dq;
    const T u0 = fma(d11, h[0], fma(P.a03 - P.a12, w[1], -(P.a02 + P.a13) * w[2]));
    const T u1 = fma(d22, h[1], fma(P.a01 - P.a23, w[2], -(P.a03 + P.a12) * w[0]));
    const T u2 = fma(d33, h[2], fma(P.a02 - P.a13, w[0], -(P.a01 + P.a23) * w[1]));
    const T uh = fma(u0, h[0], fma(u1, h[1], u2 * h[2]));                   // 4u . h
    const T c0 = fma(u1, h[2], -u2 * h[1]), c1 = fma(u2, h[0], -u0 * h[2]);  // 4u x h
    const T c2 = fma(u0, h[1], -u1 * h[0]);
    const T nt = T(-2) * th2;
    // diagonal constant: 2 (2|h|^2 tr(P)/4 + g |x|^2 + r), -/+ 4u.h
    const T base = fma(th2, tr, fma(g2, n2, r2));
    const T b0 = base - uh, bk = base + uh;
    const T gx0 = g2x * x[0], gx1 = g2x * x[1], gx2 = g2x * x[2], gx3 = g2x * x[3];
    Sym4T<T> o;
    o.a00 = fma(nt, P.a00, fma(-gx0, x[0], b0));
    o.a01 = fma(nt, P.a01, fma(-gx0, x[1], c0));
    o.a02 = fma(nt, P.a02, fma(-gx0, x[2], c1));
    o.a03 = fma(nt, P.a03, fma(-gx0, x[3], c2));
    o.a11 = fma(nt, P.a11, fma(-gx1, x[1], fma(-u0, w[0], bk)));
    o.a22 = fma(nt, P.a22, fma(-gx2, x[2], fma(-u1, w[1], bk)));
    o.a33 = fma(nt, P.a33, fma(-gx3, x[3], fma(-u2, w[2], bk)));
    o.a12 = fma(nt, P.a12, fma(-gx1, x[2], -fma(u0, h[1], u1 * h[0])));
    o.a13 = fma(nt, P.a13, fma(-gx1, x[3], -fma(u0, h[2], u2 * h[0])));
    o.a23 = fma(nt, P.a23, fma(-gx2, x[3], -fma(u1, h[2], u2 * h[1])));
    return o;
}

// The same for the covariance carried as N, P = rI + beta D N D with beta = sqrt(2) r and
// D = diag(1, 1, -1, -1) (the multi-record stream loop): returns S^ = 2S / beta, for which
// spd_inverse_schur<NEG = true> gives the next record's N = -D (S^)^-1 D with no scaling at all
// (P+ = rI - r^2 S^-1 = rI - (2r^2/beta) (S^)^-1 = rI - beta (S^)^-1, since 2r^2 = beta^2), so the
// update P = rI - r^2 S^-1 costs nothing.  D flips the sign of the off-diagonal 2x2 block: in that
// form every entry of the negated inverse is a plain sum of products (no negations to
// materialise), and here the signs ride on the operand modifiers.  With A P A^T = r|h|^2 I + beta A N' A^T
// (N' = D N D):
//   S^ = 2 A N' A^T + (2/beta)(r|h|^2 + r) I + (2g/beta)(|x|^2 I - x x^T),
// innovation_cov2's algebra on N' with gb = 2g/beta, rb = 2r/beta (= sqrt 2) for 2g, 2r, and one
// operation more (tr N + rb); gbx = gb / |x|^2 as innovation_cov2's g2x.
template <typename T>
PEKF_DEV Sym4T<T> innovation_cov_n(const Sym4T<T> &N, const T *h, const T *w, T th2, const T *x, T n2, T gb, T rb,
                                   T gbx) {
    const T sp = N.a00 + N.a11, dp = N.a11 - N.a00, sq = N.a22 + N.a33, dq = N.a22 - N.a33;
    const T tr = sp + sq, d11 = sq - sp, d22 = dp - dq, d33 = dp + dq;
    const T u0 = fma(d11, h[0], fma(N.a12 - N.a03, w[1], (N.a02 + N.a13) * w[2]));
    const T u1 = fma(d22, h[1], fma(N.a01 - N.a23, w[2], (N.a03 + N.a12) * w[0]));
    const T u2 = fma(d33, h[2], fma(N.a13 - N.a02, w[0], -(N.a01 + N.a23) * w[1]));
    const T uh = fma(u0, h[0], fma(u1, h[1], u2 * h[2]));
    const T c0 = fma(u1, h[2], -u2 * h[1]), c1 = fma(u2, h[0], -u0 * h[2]);
    const T c2 = fma(u0, h[1], -u1 * h[0]);
    const T nt = T(-2) * th2;
    const T base = fma(th2, tr + rb, fma(gb, n2, rb));
    const T b0 = base - uh, bk = base + uh;
    const T gx0 = gbx * x[0], gx1 = gbx * x[1], gx2 = gbx * x[2], gx3 = gbx * x[3];
    Sym4T<T> o;
    o.a00 = fma(nt, N.a00, fma(-gx0, x[0], b0));
    o.a01 = fma(nt, N.a01, fma(-gx0, x[1], c0));
    o.a02 = fma(-nt, N.a02, fma(-gx0, x[2], c1));
    o.a03 = fma(-nt, N.a03, fma(-gx0, x[3], c2));
    o.a11 = fma(nt, N.a11, fma(-gx1, x[1], fma(-u0, w[0], bk)));
    o.a22 = fma(nt, N.a22, fma(-gx2, x[2], fma(-u1, w[1], bk)));
    o.a33 = fma(nt, N.a33, fma(-gx3, x[3], fma(-u2, w[2], bk)));
    o.a12 = fma(-nt, N.a12, fma(-gx1, x[2], -fma(u0, h[1], u1 * h[0])));
    o.a13 = fma(-nt, N.a13, fma(-gx1, x[3], -fma(u0, h[2], u2 * h[0])));
    o.a23 = fma(nt, N.a23, fma(-gx2, x[3], -fma(u1, h[2], u2 * h[1])));
    return o;
}

// innovation_cov_n in FP64 from the raw gyro sample w alone, for the omod build of the multi-record
// loop (OmodMode): every product with h = w/2 becomes the product with w halved by the instruction
// that forms it (omod div:2), and th2x2 = 2|h|^2 = |w|^2/2 replaces both |h|^2 and -2|h|^2 (the
// latter as a negated operand), so the gyro needs no scaling at all.  Every value equals
// innovation_cov_n's bit for bit: d_aa h_a = (d_aa/2) w_a, u.h = (u.w)/2 and u x h = (u x w)/2 with
// each rounding of a halved exact sum, |h|^2 (tr + rb) = th2x2 ((tr + rb)/2).  rbh = rb / 2.
PEKF_DEV Sym4 innovation_cov_n_w(const Sym4 &N, const double *w, double th2x2, const double *x, double n2, double gb,
                                 double rb, double rbh, double gbx) {
    const double sp = N.a00 + N.a11, dp = N.a11 - N.a00, sq = N.a22 + N.a33, dq = N.a22 - N.a33;
    const double trh = add_half(sp, sq) + rbh;  // (tr + rb) / 2
    const double d11h = sub_half(sq, sp), d22h = sub_half(dp, dq), d33h = add_half(dp, dq);
    const double u0 = fma(d11h, w[0], fma(N.a12 - N.a03, w[1], (N.a02 + N.a13) * w[2]));
    const double u1 = fma(d22h, w[1], fma(N.a01 - N.a23, w[2], (N.a03 + N.a12) * w[0]));
    const double u2 = fma(d33h, w[2], fma(N.a13 - N.a02, w[0], -(N.a01 + N.a23) * w[1]));
    const double uh = fma_half(u0, w[0], fma(u1, w[1], u2 * w[2]));
    const double c0 = fma_half_nc(u1, w[2], u2 * w[1]), c1 = fma_half_nc(u2, w[0], u0 * w[2]);
    const double c2 = fma_half_nc(u0, w[1], u1 * w[0]);
    const double base = fma(th2x2, trh, fma(gb, n2, rb));
    const double b0 = base - uh, bk = base + uh;
    const double gx0 = gbx * x[0], gx1 = gbx * x[1], gx2 = gbx * x[2], gx3 = gbx * x[3];
    Sym4 o;
    o.a00 = fma(-th2x2, N.a00, fma(-gx0, x[0], b0));
    o.a01 = fma(-th2x2, N.a01, fma(-gx0, x[1], c0));
    o.a02 = fma(th2x2, N.a02, fma(-gx0, x[2], c1));
    o.a03 = fma(th2x2, N.a03, fma(-gx0, x[3], c2));
    o.a11 = fma(-th2x2, N.a11, fma(-gx1, x[1], fma(-u0, w[0], bk)));
    o.a22 = fma(-th2x2, N.a22, fma(-gx2, x[2], fma(-u1, w[1], bk)));
    o.a33 = fma(-th2x2, N.a33, fma(-gx3, x[3], fma(-u2, w[2], bk)));
    o.a12 = fma(th2x2, N.a12, fma(-gx1, x[2], -fma_half(u0, w[1], u1 * w[0])));
    o.a13 = fma(th2x2, N.a13, fma(-gx1, x[3], -fma_half(u0, w[2], u2 * w[0])));
    o.a23 = fma(-th2x2, N.a23, fma(-gx2, x[3], -fma_half(u1, w[2], u2 * w[1])));
    return o;
}

// Inverse of an SPD 4x4 by 2x2 blocks, S = [[A, B], [B^T, D]]: A^-1 by its adjugate, the Schur
// complement C = D - B^T A^-1 B (SPD) likewise, then
//   S^-1 = [[A^-1 + X C^-1 X^T, -X C^-1], [-C^-1 X^T, C^-1]],  X = A^-1 B.
// Two reciprocals (an LDL^T factorisation needs four, and a v_rcp_f64 issues at 3x an FMA on
// gfx950, scripts/probe_rates.hip): 38 plain operations + 2 Newton-refined reciprocals.
// NEG = true returns -D S^-1 D, D = diag(1, 1, -1, -1), for the same work: with W = X (-C^-1) it is
// [[-A^-1 + W X^T, W], [W^T, -C^-1]], every entry a plain sum of products (the sign of -C^-1 rides on
// the second reciprocal, that of -A^-1 on an addend).
template <typename T, bool FAST = true, bool NEG = false>
PEKF_DEV Sym4T<T> spd_inverse_schur(const Sym4T<T> &S) {
    const T ia = recip<FAST>(S.a00 * S.a11 - S.a01 * S.a01);
    const T p00 = S.a11 * ia, p01 = -S.a01 * ia, p11 = S.a00 * ia;  // A^-1
    // X = A^-1 B, B = [[a02, a03], [a12, a13]]
    const T x00 = p00 * S.a02 + p01 * S.a12, x01 = p00 * S.a03 + p01 * S.a13;
    const T x10 = p01 * S.a02 + p11 * S.a12, x11 = p01 * S.a03 + p11 * S.a13;
    // C = D - B^T X
    const T c00 = S.a22 - S.a02 * x00 - S.a12 * x10;
    const T c01 = S.a23 - S.a02 * x01 - S.a12 * x11;
    const T c11 = S.a33 - S.a03 * x01 - S.a13 * x11;
    const T ic = NEG ? recip<FAST>(c01 * c01 - c00 * c11) : recip<FAST>(c00 * c11 - c01 * c01);
    const T q00 = c11 * ic, q01 = -c01 * ic, q11 = c00 * ic;        // C^-1 (NEG: -C^-1)
    Sym4T<T> o;
    if (NEG) {
        const T w00 = x00 * q00 + x01 * q01, w01 = x00 * q01 + x01 * q11;
        const T w10 = x10 * q00 + x11 * q01, w11 = x10 * q01 + x11 * q11;
        o.a00 = w00 * x00 + w01 * x01 - p00;
        o.a01 = w00 * x10 + w01 * x11 - p01;
        o.a11 = w10 * x10 + w11 * x11 - p11;
        o.a02 = w00; o.a03 = w01; o.a12 = w10; o.a13 = w11;
        o.a22 = q00; o.a23 = q01; o.a33 = q11;
        return o;
    }
    // off-diagonal block O = -X C^-1, top-left A^-1 - O X^T
    const T o00 = -(x00 * q00 + x01 * q01), o01 = -(x00 * q01 + x01 * q11);
    const T o10 = -(x10 * q00 + x11 * q01), o11 = -(x10 * q01 + x11 * q11);
    o.a00 = p00 - o00 * x00 - o01 * x01;
    o.a01 = p01 - o00 * x10 - o01 * x11;
    o.a11 = p11 - o10 * x10 - o11 * x11;
    o.a02 = o00;
    o.a03 = o01;
    o.a12 = o10;
    o.a13 = o11;
    o.a22 = q00;
    o.a23 = q01;
    o.a33 = q11;
    return o;
}

// Closed form of the classical RK4 step + normalisation (ExtendedKalmanFilter.py:25-41),
// h_w = w/2 (so Omega(h_w) = 0.5*Omega(w), the reference's W).  z = ca x + cb 0.5*Omega(w) x and,
// since 0.5*Omega(w) is skew with square -|h_w|^2 I, |z|^2 = (ca^2 + cb^2 |h_w|^2) |x|^2 exactly:
// the normalisation factor is known before z is formed and folds into ca and cb.  n2 = |x|^2.
// kk = ca^2 + cb^2 |h_w|^2 and in = 1 / sqrt(kk n2) are returned for callers that need 1/n2 = in^2 kk.
PEKF_DEV void rk4_closed(const double *x, double n2, double dt_ns, const double *hw, double th2, double *z,
                         double &kk, double &in) {
    const double h = dt_ns * kNsToS;
    const double xx = (h * h) * th2;
    const double ca = 1.0 - 0.5 * xx + xx * xx * (1.0 / 24.0);
    const double cb = h * (1.0 - xx * (1.0 / 6.0));
    kk = ca * ca + (cb * cb) * th2;
    in = rsqrt<true>(kk * n2);
    const double a = ca * in, c = cb * in;
    const double w0 = c * hw[0], w1 = c * hw[1], w2 = c * hw[2];
    // z = a x + Omega(c h_w) x, rows of Omega: [0,-w0,-w1,-w2] [w0,0,w2,-w1] [w1,-w2,0,w0] [w2,w1,-w0,0]
    z[0] = a * x[0] - w0 * x[1] - w1 * x[2] - w2 * x[3];
    z[1] = a * x[1] + w0 * x[0] + w2 * x[2] - w1 * x[3];
    z[2] = a * x[2] + w1 * x[0] - w2 * x[1] + w0 * x[3];
    z[3] = a * x[3] + w2 * x[0] + w1 * x[1] - w0 * x[2];
}

// rk4_closed from the raw gyro sample w and th2x2 = 2|h_w|^2 = |w|^2/2 (omod build, OmodMode): the
// same values bit for bit, every halving done by the instruction that forms the product.
PEKF_DEV void rk4_closed_w(const double *x, double n2, double dt_ns, const double *w, double th2x2, double *z,
                           double &kk, double &in) {
    const double h = dt_ns * kNsToS;
    const double xx = mul_half(h * h, th2x2);  // h^2 |h_w|^2
    const double ca = 1.0 - 0.5 * xx + xx * xx * (1.0 / 24.0);
    const double cb = h * (1.0 - xx * (1.0 / 6.0));
    kk = fma(ca, ca, mul_half(cb, cb) * th2x2);
    in = rsqrt<2>(kk * n2);
    const double a = ca * in, c = cb * in;
    const double w0 = mul_half(c, w[0]), w1 = mul_half(c, w[1]), w2 = mul_half(c, w[2]);
    z[0] = a * x[0] - w0 * x[1] - w1 * x[2] - w2 * x[3];
    z[1] = a * x[1] + w0 * x[0] + w2 * x[2] - w1 * x[3];
    z[2] = a * x[2] + w1 * x[0] - w2 * x[1] + w0 * x[3];
    z[3] = a * x[3] + w2 * x[0] + w1 * x[1] - w0 * x[2];
}

PEKF_DEV void rk4_closed(const double *x, double n2, double dt_ns, const double *hw, double th2, double *z) {
    double kk, in;
    rk4_closed(x, n2, dt_ns, hw, th2, z, kk, in);
}

PEKF_DEV void rk4_closed(const double *x, double n2, double dt_ns, const double *hw, double *z) {
    rk4_closed(x, n2, dt_ns, hw, hw[0] * hw[0] + hw[1] * hw[1] + hw[2] * hw[2], z);
}

}  // namespace pekf
