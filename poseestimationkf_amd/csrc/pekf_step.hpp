// pekf_step.hpp -- device code of the fused hot path shared by pekf_run.hip (one-record launches,
// the filter handle's update) and pekf_run_multi.hip (multi-record launches): the record layout, the
// state layouts, one record of main_file.py:42-45 on a lane's registers (ekf_record_step) and the
// fused stream kernel template k_run.  The two files instantiate disjoint sets of k_run variants
// and are compiled with different scheduling strategies (Makefile), never different arithmetic.
#pragma once

#include <type_traits>

#include "pekf_internal.hpp"
#include "pekf_math.hpp"
#include "pekf_tile.hpp"

namespace pekf {

constexpr int kRunBlock = 256;

// Cache policy of the record loads: nt (aux = 2), as each record is read once per launch.
// Same box, config 3: 136.8 / 137.7 ms against 137.8 / 138.8 with the default policy
// (profiles/r1/ab_nt_loads/); sc0 nt 137.0 / 137.9; nt sc1 and sc0 nt sc1 +0.2 % (profiles/r3/ab_rec_cache_policy/).
#ifndef PEKF_REC_AUX
#define PEKF_REC_AUX 2
#endif

// Filter state in HBM.  AoS (default, the ABI's natural layout): X[b][4], P[b][4][4].  SoA
// (PEKF_RUN_STATE_SOA): X[4][batch] and the 10 unique entries of P as P[10][batch]
// (00 01 02 03 11 12 13 22 23 33): every state load / store of a wave is one contiguous
// 512 B access, which matters when a launch covers few records (online serving).
template <bool SOA, typename PT>
__device__ __forceinline__ void load_state(const double *X, const double *P, int64_t b, int64_t batch,
                                           double *x, Sym4T<PT> &S) {
    if (SOA) {
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = X[k * batch + b];
        S = {(PT)P[0 * batch + b], (PT)P[1 * batch + b], (PT)P[2 * batch + b], (PT)P[3 * batch + b],
             (PT)P[4 * batch + b], (PT)P[5 * batch + b], (PT)P[6 * batch + b], (PT)P[7 * batch + b],
             (PT)P[8 * batch + b], (PT)P[9 * batch + b]};
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = X[4 * b + k];
        const double *pp = P + 16 * b;
        S = {(PT)pp[0], (PT)pp[1], (PT)pp[2], (PT)pp[3], (PT)pp[5],
             (PT)pp[6], (PT)pp[7], (PT)pp[10], (PT)pp[11], (PT)pp[15]};
    }
}

template <bool SOA, typename PT>
__device__ __forceinline__ void store_state(double *X, double *P, int64_t b, int64_t batch, const double *x,
                                            const Sym4T<PT> &S) {
    if (SOA) {
#pragma unroll
        for (int k = 0; k < 4; ++k) X[k * batch + b] = x[k];
        const double v[10] = {S.a00, S.a01, S.a02, S.a03, S.a11, S.a12, S.a13, S.a22, S.a23, S.a33};
#pragma unroll
        for (int k = 0; k < 10; ++k) P[k * batch + b] = v[k];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) X[4 * b + k] = x[k];
        double *po = P + 16 * b;
        po[0] = S.a00; po[1] = S.a01; po[2] = S.a02; po[3] = S.a03;
        po[4] = S.a01; po[5] = S.a11; po[6] = S.a12; po[7] = S.a13;
        po[8] = S.a02; po[9] = S.a12; po[10] = S.a22; po[11] = S.a23;
        po[12] = S.a03; po[13] = S.a13; po[14] = S.a23; po[15] = S.a33;
    }
}

// Buffer resource of one plane row (raw, byte-addressed; gfx9 DWORD3 0x00020000)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void *row, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(row), 0, (int)(uint32_t)bytes, 0x00020000);
}

// The rows of the three record planes a multi-record launch walks through (row r of a plane is
// batch x 16 B for gd / am, batch x 8 B for my; the window wraps).  Rows are read through buffer
// descriptors of a CHUNK of consecutive rows with the row's offset inside the chunk in the
// instruction's scalar offset (soffset), so moving to the next row is two scalar adds and a compare,
// and the descriptors are rebuilt only when a chunk ends: chunk offsets stay below 2^31 (128 rows at
// config 3, the whole 1,024-row window at config 2).  Each descriptor's record count is its chunk's
// byte size and the range check covers soffset (measured: scripts/buffer_range_probe.hip), so an
// offset past the chunk would read zeros, never another allocation.
struct RowCursor {
    const char *g, *a, *m;
    uint32_t row16, row8;
    int32_t window, chunk_rows;
    int32_t row = 0, end = 0;
    uint32_t s16 = 0, s8 = 0;
    __amdgpu_buffer_rsrc_t rg, ra, rm;

    __device__ __forceinline__ RowCursor(const float4 *gd, const float4 *am, const float2 *my, int64_t batch,
                                         int64_t win)
        : g(reinterpret_cast<const char *>(gd)), a(reinterpret_cast<const char *>(am)),
          m(reinterpret_cast<const char *>(my)), row16((uint32_t)batch * 16u), row8((uint32_t)batch * 8u),
          window((int32_t)win) {
        const uint32_t c = (1u << 31) / row16;
        chunk_rows = c ? (int32_t)c : 1;
    }
    __device__ __forceinline__ void start(int32_t r) {
        row = r;
        end = (window - r < chunk_rows) ? window : r + chunk_rows;
        const uint64_t n = (uint64_t)(end - r);
        rg = row_rsrc(g + (uint64_t)r * row16, (int64_t)(n * row16));
        ra = row_rsrc(a + (uint64_t)r * row16, (int64_t)(n * row16));
        rm = row_rsrc(m + (uint64_t)r * row8, (int64_t)(n * row8));
        s16 = 0;
        s8 = 0;
    }
    __device__ __forceinline__ void advance() {
        if (++row == end) {
            start(row == window ? 0 : row);
        } else {
            s16 += row16;
            s8 += row8;
        }
    }
    __device__ __forceinline__ Rec load(uint32_t off16, uint32_t off8) const {
        Rec v;
        v.gd = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rg, off16, s16, PEKF_REC_AUX));
        v.am = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, off16, s16, PEKF_REC_AUX));
        v.my = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rm, off8, s8, PEKF_REC_AUX));
        return v;
    }
};

// AoS P (full 4x4) <-> its upper triangle, for state moved through a WaveTile
template <typename PT>
__device__ __forceinline__ Sym4T<PT> sym_from16(const double (&p)[16]) {
    return {(PT)p[0], (PT)p[1], (PT)p[2], (PT)p[3], (PT)p[5], (PT)p[6], (PT)p[7], (PT)p[10], (PT)p[11], (PT)p[15]};
}
template <typename PT>
__device__ __forceinline__ void sym_to16(const Sym4T<PT> &S, double (&p)[16]) {
    p[0] = S.a00; p[1] = S.a01; p[2] = S.a02; p[3] = S.a03;
    p[4] = S.a01; p[5] = S.a11; p[6] = S.a12; p[7] = S.a13;
    p[8] = S.a02; p[9] = S.a12; p[10] = S.a22; p[11] = S.a23;
    p[12] = S.a03; p[13] = S.a13; p[14] = S.a23; p[15] = S.a33;
}

// |X|^2 of the state entering a launch.  After any record the state is unit (X /= |X|,
// ExtendedKalmanFilter.py:79, or X = z from the normalised RK4 step) to within ~40 ulp of the
// one-Newton-step rsqrt, and that is snapped to exactly 1: the stream kernel carries n2 = 1 as a
// constant after a launch's first record, and every launch shape (n records at once, one record
// per launch, the handle's per-record update) rounds identically.  A state that is not unit (a
// user's set_state) keeps its |X|^2, which the reference's Jb and RK4 use (:60-62).
__device__ __forceinline__ double state_norm2(const double *x) {
    const double n2 = x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
    return fabs(n2 - 1.0) < 1e-13 ? 1.0 : n2;
}

// One record of main_file.py:42-45 -- Prediction(gyro, T) then Correction(mag, acc) -- on the
// lane's state (x, P) in registers, in the world basis (Wf: the reference pair's Frame) or in the
// reference frame's own basis (Wf: a RefW, see pekf_math.hpp); n2 = state_norm2 of x (1 for every record after a launch's
// first).  gy = the gyro sample, dt_ns = T - previousT, missing: the record has no magnetometer
// sample (Wahba-skip, X = z, P = P-).  Shared by the fused stream kernel and the handle's
// per-record update, so both give bit-identical results for the same inputs.
// a * b - c as one three-address v_fma_f64 with a negated operand.  Left to itself the compiler
// picks the accumulating v_fmac_f64 for e = v sc - z and sets -z up in the accumulator registers
// ahead of the rare Wahba fallback branch (a negation and two register copies per component).
__device__ __forceinline__ double fma_sub(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, -%3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// c - a * b, likewise
__device__ __forceinline__ double fma_rsub(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, -%1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Per-launch constants of ekf_record_step.  MC = false: the covariance is carried as P itself;
// MC = true (the multi-record stream loop): as N with P = rI + beta D N D, beta = sqrt(2) r,
// D = diag(1, 1, -1, -1), so that the next N = -D (S^)^-1 D comes out of the Schur inverse of
// innovation_cov_n's S^ with no update arithmetic (pekf_math.hpp).
template <typename PT>
struct StepK {
    PT g2, r2;   // MC: 2g/beta, 2r/beta | P: 2g, 2r (innovation_cov_n / innovation_cov2)
    PT rp, rr;   // P: r, 2r^2 (P = rI - 2r^2 (2S)^-1) | MC: r2 / 2 (innovation_cov_n_w), unused
    double sy;   // Y's weight in the unnormalised X update: MC 1/sqrt(2), P 1/(2r)
};
template <typename PT, bool MC>
__device__ __forceinline__ StepK<PT> step_consts(double qs, double rs) {
    const double g = 0.25 * qs;  // Jb Q Jb^T = (q/4)(|X|^2 I - X X^T)
    if (MC) {
        const double ib = 1.0 / (kSqrt2 * rs);
        return {(PT)(2.0 * g * ib), (PT)(2.0 * rs * ib), (PT)(rs * ib), PT(0), 1.0 / kSqrt2};
    }
    return {(PT)(2.0 * g), (PT)(2.0 * rs), (PT)rs, (PT)(2.0 * (rs * rs)), 0.5 / rs};
}

// MC (the multi-record loop) also leaves X unnormalised, X = x / |x| with |x| ~ 0.7: its norm
// folds into the next record's RK4 normalisation (z = rk4(x) / |rk4(x)| whatever |x|) and Jb term
// (g (|X|^2 I - X X^T) = g I - (g / |x|^2) x x^T, |X|^2 = 1 as state_norm2 snaps it), and
// 1/|x|^2 = in^2 kk comes from RK4's own rsqrt: 8 operations instead of the 13 of normalising X.
// LAZY: x arrives that way (n2 ignored); the caller normalises once at the end of the launch.
// OM (the FP64 multi-record loop, inside OmodMode): the exact halvings fold into the instructions
// that form the products (omod, pekf_math.hpp) -- the gyro is never scaled to h = w/2, and the
// Newton steps of the rsqrt seeds need no separate multiply by 1/2: 9 VALU fewer per record, the
// same values bit for bit.
// reload(acc, mag) re-reads the record's samples for the rare degenerate-Wahba fallback
// (wahba_quat_toward); it is not called on the common path.
// Wahba-skip: no Correction for this record (X = z, P = P- = S - rI)
template <typename PT, bool MC>
__device__ __forceinline__ void record_skip(double *x, const double *z, Sym4T<PT> &P, const Sym4T<PT> &S2,
                                            const StepK<PT> &k) {
    x[0] = z[0]; x[1] = z[1]; x[2] = z[2]; x[3] = z[3];
    const PT hf = PT(0.5);
    if (MC)  // D N D = (S - 2r I) / beta = S^/2 - rb I
        P = {fma(hf, S2.a00, -k.r2), hf * S2.a01, -hf * S2.a02, -hf * S2.a03, fma(hf, S2.a11, -k.r2),
             -hf * S2.a12, -hf * S2.a13, fma(hf, S2.a22, -k.r2), hf * S2.a23, fma(hf, S2.a33, -k.r2)};
    else
        P = {fma(hf, S2.a00, -k.rp), hf * S2.a01, hf * S2.a02, hf * S2.a03, fma(hf, S2.a11, -k.rp),
             hf * S2.a12, hf * S2.a13, fma(hf, S2.a22, -k.rp), hf * S2.a23, fma(hf, S2.a33, -k.rp)};
}

// ---- Correction (ExtendedKalmanFilter.py:70-80) from S^-1 (Si) and Wahba's Y = v sc ----
template <typename PT, bool MC>
__device__ __forceinline__ void record_correct(double *x, const double *z, Sym4T<PT> &P, const Sym4T<PT> &Si,
                                               const double *v, double sc, const StepK<PT> &k) {
    // e = Y - z (MC: D e, whose last two components are z - Y)
    const PT e0 = (PT)fma_sub(v[0], sc, z[0]), e1 = (PT)fma_sub(v[1], sc, z[1]);
    const PT e2 = (PT)(MC ? fma_rsub(v[2], sc, z[2]) : fma_sub(v[2], sc, z[2]));
    const PT e3 = (PT)(MC ? fma_rsub(v[3], sc, z[3]) : fma_sub(v[3], sc, z[3]));
    // X = z + K e = Y - r S^-1 e (:77), normalised (:79): X ~ Y / (2r) - S^-1 e / 2, or (MC,
    // S^-1 = -(2/beta) D Si D) X ~ Y / sqrt(2) + D Si D e
    const double u0 = Si.a00 * e0 + Si.a01 * e1 + Si.a02 * e2 + Si.a03 * e3;
    const double u1 = Si.a01 * e0 + Si.a11 * e1 + Si.a12 * e2 + Si.a13 * e3;
    const double u2 = Si.a02 * e0 + Si.a12 * e1 + Si.a22 * e2 + Si.a23 * e3;
    const double u3 = Si.a03 * e0 + Si.a13 * e1 + Si.a23 * e2 + Si.a33 * e3;
    const double sr = sc * k.sy;
    const double x0 = fma(v[0], sr, MC ? u0 : -u0), x1 = fma(v[1], sr, MC ? u1 : -u1);
    const double x2 = fma(v[2], sr, -u2), x3 = fma(v[3], sr, -u3);
    if (MC) {
        x[0] = x0; x[1] = x1; x[2] = x2; x[3] = x3;
    } else {
        const double in = rsqrt<true>(x0 * x0 + x1 * x1 + x2 * x2 + x3 * x3);
        x[0] = x0 * in; x[1] = x1 * in; x[2] = x2 * in; x[3] = x3 * in;
    }
    // P = P- - K P- = r K = r I - r^2 S^-1 = r I - (2 r^2) Si (:78)
    if (MC) {
        P = Si;  // P = rI + beta D N D: nothing to compute
    } else {
        const PT rp = k.rp, rr = k.rr;
        P = {rp - rr * Si.a00, -rr * Si.a01, -rr * Si.a02, -rr * Si.a03, rp - rr * Si.a11,
             -rr * Si.a12, -rr * Si.a13, rp - rr * Si.a22, -rr * Si.a23, rp - rr * Si.a33};
    }
}

// HOIST (the FP64 multi-record loop only): the Correction's state-independent half -- S^-1, the
// current frame and Wahba's rotation R' -- is formed ahead of the missing-magnetometer branch, in the
// Prediction's basic block (held there by an empty asm), so one block carries two independent
// dependency chains (the Prediction's and the record's own); only Q4 z, its flip and the update stay
// behind the branch.  For launches of at most one wave per SIMD (config 2), where nothing else fills
// the chain's stalls (launch_run_multi selects it).  The same arithmetic, bit for bit.
template <typename PT, bool MC = false, bool LAZY = false, bool OM = false, bool PIN = false, bool HOIST = false,
          typename Ref, typename Reload>
__device__ __forceinline__ void ekf_record_step(double *x, double n2, Sym4T<PT> &P, const Ref &Wf, const StepK<PT> &k,
                                                const double *gy, double dt_ns, bool missing,
                                                const double *acc, const double *mag, const Reload &reload) {
    static_assert(!OM || (MC && std::is_same<PT, double>::value), "omod form: FP64 multi-record loop only");
    static_assert(!HOIST || OM, "hoisted form: FP64 multi-record loop only");
    constexpr int F = OM ? 2 : 1;  // rsqrt form
    // ---- Prediction (ExtendedKalmanFilter.py:58-68) ----
    const double n2x = LAZY ? x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3] : n2;
    double z[4], kk, irk;
    Sym4T<PT> S2;
    if constexpr (OM) {
        // th2x2 = 2 |h|^2 = |w|^2 / 2 (0.5*Omega(w) = Omega(h), h = w/2)
        const double th2x2 = fma_half(gy[2], gy[2], fma(gy[1], gy[1], gy[0] * gy[0]));
        rk4_closed_w(x, n2x, dt_ns, gy, th2x2, z, kk, irk);                  // (:62)
        const double g2x = LAZY ? ((irk * irk) * kk) * k.g2 : k.g2;           // 2g / |x|^2
        S2 = innovation_cov_n_w(P, gy, th2x2, x, LAZY ? 1.0 : n2, k.g2, k.r2, k.rp, g2x);
    } else {
        const double hw[3] = {0.5 * gy[0], 0.5 * gy[1], 0.5 * gy[2]};  // 0.5*Omega(w) = Omega(w/2)
        const double th2 = hw[0] * hw[0] + hw[1] * hw[1] + hw[2] * hw[2];
        const PT hp[3] = {(PT)hw[0], (PT)hw[1], (PT)hw[2]};
        const PT wp[3] = {(PT)gy[0], (PT)gy[1], (PT)gy[2]};
        const PT xp[4] = {(PT)x[0], (PT)x[1], (PT)x[2], (PT)x[3]};
        rk4_closed(x, n2x, dt_ns, hw, th2, z, kk, irk);                    // (:62)
        const PT g2x = LAZY ? (PT)((irk * irk) * kk) * k.g2 : k.g2;         // 2g / |x|^2
        const PT n2p = LAZY ? PT(1) : (PT)n2;
        // S2 = 2S, S = P- + rI with P- = A P A^T + Jb Q Jb^T, Jb from the prior X (:60-61, :63).
        // Exactly twice S (see innovation_cov2), so every result below is bit-identical to the
        // undoubled recursion: (2S)^-1 = S^-1/2, and the constants absorb the factor.
        S2 = MC ? innovation_cov_n<PT>(P, hp, wp, (PT)th2, xp, n2p, k.g2, k.r2, g2x)
                : innovation_cov2<PT>(P, hp, wp, (PT)th2, xp, n2p, k.g2, k.r2, g2x);
    }

    if constexpr (HOIST) {
        const Sym4T<PT> Si = spd_inverse_schur<PT, true, MC>(S2);
        const double ka = fabs(acc[2]);              // (:71)
        Frame Vf;
        make_frame<F>(acc, mag, Vf, 1.0 - ka);
        double R[9];
        wahba_rotation_ref<F>(Wf, Vf, ka, 1.0 - ka, R);
        asm volatile("" ::"v"(Si.a00), "v"(Si.a01), "v"(Si.a02), "v"(Si.a03), "v"(Si.a11), "v"(Si.a12),
                     "v"(Si.a13), "v"(Si.a22), "v"(Si.a23), "v"(Si.a33), "v"(R[0]), "v"(R[1]), "v"(R[2]),
                     "v"(R[3]), "v"(R[4]), "v"(R[5]), "v"(R[6]), "v"(R[7]), "v"(R[8]));
        if (missing) {
            record_skip<PT, MC>(x, z, P, S2, k);
        } else {
            double v[4], sc;
            wahba_toward_from_rotation<F>(Wf, R, z, v, sc, reload);  // Wahba.py:8-47 + the flip of :73-75
            record_correct<PT, MC>(x, z, P, Si, v, sc, k);
        }
        return;
    }
    if (missing) {
        // Wahba-skip: no Correction for this record (X = z, P = P- = S - rI)
        x[0] = z[0]; x[1] = z[1]; x[2] = z[2]; x[3] = z[3];
        const PT hf = PT(0.5);
        if (MC)  // D N D = (S - 2r I) / beta = S^/2 - rb I
            P = {fma(hf, S2.a00, -k.r2), hf * S2.a01, -hf * S2.a02, -hf * S2.a03, fma(hf, S2.a11, -k.r2),
                 -hf * S2.a12, -hf * S2.a13, fma(hf, S2.a22, -k.r2), hf * S2.a23, fma(hf, S2.a33, -k.r2)};
        else
            P = {fma(hf, S2.a00, -k.rp), hf * S2.a01, hf * S2.a02, hf * S2.a03, fma(hf, S2.a11, -k.rp),
                 hf * S2.a12, hf * S2.a13, fma(hf, S2.a22, -k.rp), hf * S2.a23, fma(hf, S2.a33, -k.rp)};
    } else {
        // K = P- S^-1 = I - r S^-1  (:64-66); Si = S^-1 / 2, or (MC) the next N = -D (S^)^-1 D
        const Sym4T<PT> Si = spd_inverse_schur<PT, true, MC>(S2);

        // ---- Correction (ExtendedKalmanFilter.py:70-80) ----
        const double ka = fabs(acc[2]);              // (:71)
        Frame Vf;
        // ka = |acc_z| >= 0, so wahba_sign(ka, km) is the sign of km = 1 - ka (never -0)
        make_frame<F>(acc, mag, Vf, 1.0 - ka);
        double v[4], sc;
        // PIN: S^-1 depends only on the Prediction; have it computed before the rare fallback branch,
        // in the basic block of the Wahba chain, so that the two independent chains interleave (left
        // to itself the compiler sinks it past the branch, behind the Wahba chain).  Worth it where a
        // SIMD has one wave and the record's dependency chain is exposed (config 2: -2.3 %); neutral at
        // 3 waves per SIMD (config 3), where the other waves fill those gaps anyway
        // (profiles/r2/ab_pin_schur/).  Scheduling only: the arithmetic is the same, bit for bit.
        auto pin = [&] {
            if constexpr (PIN && MC && OM)
                asm volatile("" ::"v"(Si.a00), "v"(Si.a01), "v"(Si.a02), "v"(Si.a03), "v"(Si.a11), "v"(Si.a12),
                             "v"(Si.a13), "v"(Si.a22), "v"(Si.a23), "v"(Si.a33));
        };
        wahba_quat_toward<F>(Wf, Vf, ka, 1.0 - ka, z, v, sc, reload, pin);  // Wahba.py:8-47 + the flip of :73-75: Y = v sc
        // e = Y - z (MC: D e, whose last two components are z - Y)
        const PT e0 = (PT)fma_sub(v[0], sc, z[0]), e1 = (PT)fma_sub(v[1], sc, z[1]);
        const PT e2 = (PT)(MC ? fma_rsub(v[2], sc, z[2]) : fma_sub(v[2], sc, z[2]));
        const PT e3 = (PT)(MC ? fma_rsub(v[3], sc, z[3]) : fma_sub(v[3], sc, z[3]));
        // X = z + K e = Y - r S^-1 e (:77), normalised (:79): X ~ Y / (2r) - S^-1 e / 2, or (MC,
        // S^-1 = -(2/beta) D Si D) X ~ Y / sqrt(2) + D Si D e
        const double u0 = Si.a00 * e0 + Si.a01 * e1 + Si.a02 * e2 + Si.a03 * e3;
        const double u1 = Si.a01 * e0 + Si.a11 * e1 + Si.a12 * e2 + Si.a13 * e3;
        const double u2 = Si.a02 * e0 + Si.a12 * e1 + Si.a22 * e2 + Si.a23 * e3;
        const double u3 = Si.a03 * e0 + Si.a13 * e1 + Si.a23 * e2 + Si.a33 * e3;
        const double sr = sc * k.sy;
        const double x0 = fma(v[0], sr, MC ? u0 : -u0), x1 = fma(v[1], sr, MC ? u1 : -u1);
        const double x2 = fma(v[2], sr, -u2), x3 = fma(v[3], sr, -u3);
        if (MC) {
            x[0] = x0; x[1] = x1; x[2] = x2; x[3] = x3;
        } else {
            const double in = rsqrt<true>(x0 * x0 + x1 * x1 + x2 * x2 + x3 * x3);
            x[0] = x0 * in; x[1] = x1 * in; x[2] = x2 * in; x[3] = x3 * in;
        }
        // P = P- - K P- = r K = r I - r^2 S^-1 = r I - (2 r^2) Si (:78)
        if (MC) {
            P = Si;  // P = rI + beta D N D: nothing to compute
        } else {
            const PT rp = k.rp, rr = k.rr;
            P = {rp - rr * Si.a00, -rr * Si.a01, -rr * Si.a02, -rr * Si.a03, rp - rr * Si.a11,
                 -rr * Si.a12, -rr * Si.a13, rp - rr * Si.a22, -rr * Si.a23, rp - rr * Si.a33};
        }
    }
}

// A multi-record launch runs the filter in its reference frame's own basis (RefW in pekf_math.hpp)
// with the covariance carried as N, P = rI + beta D N D (StepK).  to_ref_basis: the state entering
// the launch, x -> q_W^* x, P -> N of q_W^* P q_W; from_ref_basis: back at its end, X normalised.
template <typename PT>
__device__ __forceinline__ void to_ref_basis(const double *qw, double *x, Sym4T<PT> &P, double rs) {
    double xw[4];
    qmul_left<true>(qw, x, xw);
    x[0] = xw[0]; x[1] = xw[1]; x[2] = xw[2]; x[3] = xw[3];
    P = sym_rotate<true>(qw, P);
    const PT ib = (PT)(1.0 / (kSqrt2 * rs)), rp = (PT)rs;
    P = {(P.a00 - rp) * ib, P.a01 * ib, -P.a02 * ib, -P.a03 * ib, (P.a11 - rp) * ib,
         -P.a12 * ib, -P.a13 * ib, (P.a22 - rp) * ib, P.a23 * ib, (P.a33 - rp) * ib};
}
template <typename PT, typename RW>
__device__ __forceinline__ void from_ref_basis(const RW &Wr, double *x, Sym4T<PT> &P, double rs) {
    const PT be = (PT)(kSqrt2 * rs), rp = (PT)rs;
    P = {fma(be, P.a00, rp), be * P.a01, -be * P.a02, -be * P.a03, fma(be, P.a11, rp),
         -be * P.a12, -be * P.a13, fma(be, P.a22, rp), be * P.a23, fma(be, P.a33, rp)};
    const double in = rsqrt<true>(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
    const double xn[4] = {x[0] * in, x[1] * in, x[2] * in, x[3] * in};
    double xo[4], qw[4];
    Wr.quat(qw);
    qmul_left<false>(qw, xn, xo);
    x[0] = xo[0]; x[1] = xo[1]; x[2] = xo[2]; x[3] = xo[3];
    P = sym_rotate<false>(qw, P);
}

// Occupancy target of k_run in waves per SIMD (0: the compiler's choice)
#ifndef PEKF_RUN_WAVES
#define PEKF_RUN_WAVES 0
#endif
#if PEKF_RUN_WAVES
#define PEKF_RUN_ATTR __attribute__((amdgpu_waves_per_eu(PEKF_RUN_WAVES)))
#else
#define PEKF_RUN_ATTR
#endif

// MIXED = false: every operation in FP64 (the headline path).
// MIXED = true (opt-in, PEKF_RUN_MIXED_PRECISION): the covariance recursion (P-, S^-1, K, P)
// in FP32 while RK4, Wahba, R->q and the X update stay FP64 (~2e-8 vs FP64).
// COUNTS: filter b applies only its first counts[b] records of the launch (a separate
// instantiation so the uniform-length path carries no per-step lane predicate).
// PIN: the Schur-inverse-first schedule of the multi-record loop (ekf_record_step, launch_run_multi).
// LONGDT: the window has a dt side plane dtx[window][batch] (float64 ns): a record whose dt word is
// PEKF_DT_ESCAPE takes its dt from there -- gaps of 2^31 ns or more, negative or fractional ones, any
// T - previousT the reference accepts (ExtendedKalmanFilter.py:62).  A separate instantiation, so the
// windows without escapes (every synthetic and front-end stream but the rare long pause) pay nothing.
// HOIST: the Correction's state-independent half ahead of the missing branch (ekf_record_step).
template <bool TRAJ, bool MIXED, bool SOA, bool COUNTS, bool ONE, bool PIN = false, bool LONGDT = false,
          bool HOIST = false>
__global__ __launch_bounds__(kRunBlock) PEKF_RUN_ATTR void k_run(int64_t batch, int64_t n_steps, int64_t window,
                                                   int64_t step0, const float4 *__restrict__ gd,
                                                   const float4 *__restrict__ am,
                                                   const float2 *__restrict__ my,
                                                   const double *__restrict__ refs,
                                                   double *__restrict__ Xio, double *__restrict__ Pio,
                                                   double qs, double rs, double *__restrict__ traj,
                                                   const int32_t *__restrict__ counts,
                                                   const double *__restrict__ dtx) {
    using PT = typename std::conditional<MIXED, float, double>::type;
    if constexpr (ONE) {
        // one-record launch (online serving): the state and the reference pair are most of the
        // traffic.  The AoS state and the [batch][6] reference pairs move in coalesced wave tiles
        // (pekf_tile.hpp) instead of 128 / 48 B-strided per-lane accesses; the SoA state is read and
        // written per lane, one contiguous 512 B access per component and wave.
        constexpr int kTile = SOA ? 6 : 16;
        __shared__ double pool[kRunBlock / kWave * tile_doubles<kTile>()];
        const WaveTile t(pool, tile_doubles<kTile>(), batch);
        double cx[4], cp[16], cr[6];
        if constexpr (!SOA) {
            t.gather(Xio, cx);
            t.gather(Pio, cp);
        }
        t.gather(refs, cr);
        const bool act = t.active();
        const uint32_t lane = act ? (uint32_t)(t.first + t.lane) : 0u;  // idle lanes read a valid row
        const int64_t base = (step0 % window) * batch;
        const Rec cur = {(gd + base)[lane], (am + base)[lane], (my + base)[lane]};
        const bool run = act && (!COUNTS || counts[lane] > 0);
        double x[4], pv[16], rf[6];
        Sym4T<PT> P;
        if constexpr (SOA) {
            load_state<true>(Xio, Pio, lane, batch, x, P);
        } else {
            t.to_lanes(cx, x);
            t.to_lanes(cp, pv);
            P = sym_from16<PT>(pv);
        }
        t.to_lanes(cr, rf);
        Frame Wf;
        make_frame<true>(rf, rf + 3, Wf);
        if (run) {
            const double gy[3] = {cur.gd.x, cur.gd.y, cur.gd.z};
            const uint32_t word = __float_as_uint(cur.gd.w);
            const double acc[3] = {cur.am.x, cur.am.y, cur.am.z};
            const double mag[3] = {cur.am.w, cur.my.x, cur.my.y};
            double dtn = (double)(word & PEKF_DT_MASK);
            if constexpr (LONGDT) {
                if ((word & PEKF_DT_MASK) == PEKF_DT_ESCAPE) dtn = (dtx + base)[lane];
            }
            auto reload = [&](double *a, double *m) {  // rare: the degenerate-Wahba fallback
                const float4 va = (am + base)[lane];
                const float2 vm = (my + base)[lane];
                a[0] = va.x; a[1] = va.y; a[2] = va.z;
                m[0] = va.w; m[1] = vm.x; m[2] = vm.y;
            };
            ekf_record_step<PT>(x, state_norm2(x), P, Wf, step_consts<PT, false>(qs, rs), gy, dtn,
                                (word & PEKF_MISSING_MAG_BIT) != 0, acc, mag, reload);
        }
        if (TRAJ && act) {
            double2 *o = reinterpret_cast<double2 *>(traj) + 2 * (int64_t)lane;
            o[0] = make_double2(x[0], x[1]);
            o[1] = make_double2(x[2], x[3]);
        }
        if constexpr (SOA) {
            if (act) store_state<true>(Xio, Pio, lane, batch, x, P);
        } else {
            sym_to16(P, pv);
            t.store(Xio, x);
            t.store(Pio, pv);
        }
        return;
    }
    const int64_t b = (int64_t)blockIdx.x * kRunBlock + threadIdx.x;
    if (b >= batch) return;
    const int32_t my_steps = COUNTS ? (counts[b] < n_steps ? counts[b] : (int32_t)n_steps) : (int32_t)n_steps;

    // per-filter constants: the Wahba reference frame of (acc0, mag0) (Wahba.py:4-6)
    Frame Wf;
    {
        const double a0[3] = {refs[6 * b + 0], refs[6 * b + 1], refs[6 * b + 2]};
        const double m0[3] = {refs[6 * b + 3], refs[6 * b + 4], refs[6 * b + 5]};
        make_frame<true>(a0, m0, Wf);
    }
    double x[4];
    Sym4T<PT> P;
    load_state<SOA>(Xio, Pio, b, batch, x, P);

    // Record of stream row r: raw buffer loads whose lane offset is fixed and whose row offset is
    // the wave-uniform soffset within a chunk of rows (RowCursor), so a record costs two scalar adds
    // and a compare of address work, no per-step vector address arithmetic (batch < 2^28 is checked
    // on the host, so the offsets fit).
    const uint32_t lane = (uint32_t)b;
    const uint32_t off16 = lane * 16u, off8 = lane * 8u;
    RowCursor rows(gd, am, my, batch, window);
    // rows the cursor runs ahead of the record a step works on (ping-pong: one; deeper prefetch rings
    // were measured and not kept, profiles/r1/README.md)
    constexpr int32_t kLag = 1;
    // One record: Prediction + Correction (main_file.py:42-45) on (x, P) in registers.
    auto step = [&](const Rec &cur, int32_t t, double n2, const auto &ref, auto lazy) {
        // the multi-record loop (RefW) carries N and an unnormalised X, the one-record launch
        // (Frame) P and X; lazy: X arrives unnormalised (every multi-record step after the first)
        constexpr bool MC = !std::is_same<std::decay_t<decltype(ref)>, Frame>::value;
        if (!COUNTS || t < my_steps) {
            const double gy[3] = {cur.gd.x, cur.gd.y, cur.gd.z};
            const uint32_t word = __float_as_uint(cur.gd.w);
            const double acc[3] = {cur.am.x, cur.am.y, cur.am.z};
            const double mag[3] = {cur.am.w, cur.my.x, cur.my.y};
            double dtn = (double)(word & PEKF_DT_MASK);
            if constexpr (LONGDT) {  // the escaped record's row, (step0 + t) % window (rare: off the fast path)
                if ((word & PEKF_DT_MASK) == PEKF_DT_ESCAPE) dtn = dtx[((step0 + t) % window) * batch + b];
            }
            auto reload = [&](double *a, double *m) {  // rare: this record again; the cursor is kLag rows ahead
                int32_t r = rows.row - kLag;
                while (r < 0) r += rows.window;
                // through one-row descriptors and the lane offsets the loop holds anyway (no 64-bit
                // lane index is kept live for this)
                const float4 va = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                    row_rsrc(rows.a + (uint64_t)r * rows.row16, rows.row16), off16, 0, 0));
                const float2 vm = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(
                    row_rsrc(rows.m + (uint64_t)r * rows.row8, rows.row8), off8, 0, 0));
                a[0] = va.x; a[1] = va.y; a[2] = va.z;
                m[0] = va.w; m[1] = vm.x; m[2] = vm.y;
            };
            ekf_record_step<PT, MC, decltype(lazy)::value, MC && !MIXED, PIN, HOIST && MC && !MIXED>(
                x, n2, P, ref, step_consts<PT, MC>(qs, rs), gy, dtn, (word & PEKF_MISSING_MAG_BIT) != 0, acc, mag,
                reload);
        }
        if (TRAJ) {
            double xo[4] = {x[0], x[1], x[2], x[3]};
            // a filter with no records in this launch (COUNTS) repeats its stored X unchanged
            // (x was rotated by the identity, which is exact; it is not normalised or written back)
            if constexpr (MC) {
                if (!COUNTS || my_steps > 0) {
                    const double in = rsqrt<true>(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
                    const double xn[4] = {x[0] * in, x[1] * in, x[2] * in, x[3] * in};
                    double qw[4];
                    ref.quat(qw);
                    qmul_left<false>(qw, xn, xo);
                }
            }
            double2 *o = reinterpret_cast<double2 *>(traj + (int64_t)t * batch * 4) + 2 * (int64_t)lane;
            o[0] = make_double2(xo[0], xo[1]);
            o[1] = make_double2(xo[2], xo[3]);
        }
    };
    using eager = std::false_type;
    using lazy = std::true_type;

    // Time loop, unrolled by two with ping-pong records: the next row's record is always in
    // flight while the current one is processed, and no registers are copied between steps.
    // The prefetch is unconditional (the row wraps inside the resident window, so it is always
    // a valid address); n_steps >= 1 here.  One-record launches (online serving) use the ONE
    // instantiation, which has no prefetch: there its 40 B would be an eighth of the traffic.
    rows.start((int32_t)(step0 % window));
    Rec ra = rows.load(off16, off8), rb;
    // A multi-record launch runs the filter in its reference frame's own basis (RefW in
    // pekf_math.hpp: the same filter, with Wahba's rotation 24 operations cheaper per record);
    // the state is rotated in once and out once per launch.  A filter with no records in this
    // launch (COUNTS) rotates by the identity, which is exact, and its state is not written back.
    // Inside the loop the covariance is carried as N, P = rI + beta D N D (StepK).
    // Without trajectory output q_W is recomputed at the launch's end (and in the rare fallback)
    // rather than held through the loop (RefWLazy: 8 VGPRs).
    using RW = typename std::conditional<TRAJ, RefW, RefWLazy>::type;
    RW Wr;
    Wr.aW = Wf.alpha; Wr.b1W = Wf.beta1; Wr.b2W = Wf.beta2;
    {
        double qw[4];
        frame_quat(Wf, qw);
        if constexpr (TRAJ) {
            if (COUNTS && my_steps == 0) { qw[0] = 1.0; qw[1] = qw[2] = qw[3] = 0.0; }
            Wr.q[0] = qw[0]; Wr.q[1] = qw[1]; Wr.q[2] = qw[2]; Wr.q[3] = qw[3];
        } else {
            Wr.pair = refs + 6 * b;
        }
        to_ref_basis(qw, x, P, rs);
    }
    // The launch's first record takes |X|^2 from the loaded state; from then on the state is
    // unit and n2 = 1 is a compile-time constant (see state_norm2).  32-bit step counter
    // (n_steps < 2^31 is checked on the host).
    const int32_t n32 = (int32_t)n_steps;
    rows.advance();
    rb = rows.load(off16, off8);
    // the FP64 loop folds its exact halvings into output modifiers, which need this MODE
    OmodMode mode;
    if constexpr (!MIXED) mode.enter();
    step(ra, 0, state_norm2(x), Wr, eager{});
    for (int32_t t = 1; t < n32;) {
        rows.advance();
        ra = rows.load(off16, off8);
        step(rb, t, 1.0, Wr, lazy{});
        if (++t == n32) break;
        rows.advance();
        rb = rows.load(off16, off8);
        step(ra, t, 1.0, Wr, lazy{});
        ++t;
    }
    if constexpr (!MIXED) mode.leave();
    if (COUNTS && my_steps == 0) return;
    from_ref_basis(Wr, x, P, rs);
    store_state<SOA>(Xio, Pio, b, batch, x, P);
}


}  // namespace pekf
