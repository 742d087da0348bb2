// pekf_run_split.hip -- the multi-record fused kernel for SMALL batches (config 2: 65,536 filters =
// 1,024 waves, one per SIMD), where the one-lane-per-filter kernel leaves each SIMD a single wave and
// the ~300-instruction FP64 dependency chain of a record exposes its latencies (config 2 runs ~12 %
// below config 3's per-record rate).  Here each 64 filters get TWO waves: the MEASUREMENT wave
// computes the state-independent half of the Correction -- the current Gram-Schmidt frame of
// (acc, mag), Wahba's rotation R' in the reference frame's basis and the ten entries of Q4 = 4 q q^T
// (Wahba.py:8-47, ExtendedKalmanFilter.py:71) -- one record ahead, and hands them through LDS to
// the FILTER wave, which runs the Prediction, the Schur inverse and the update (ExtendedKalmanFilter.py
// :58-80) exactly as ekf_record_step<double, MC, LAZY, OM> does.  Each SIMD then interleaves two
// waves' independent instruction streams.  Same expressions, same contraction, same MODE in both
// waves: bit-identical to k_run<false, false, SOA, false, false> (tests/test_gpu_parity.py).
// Selected by launch_run_multi when the one-lane kernel would run < 2 waves per SIMD (PEKF_RUN_SPLIT
// overrides: 0 never, 1 always).
#include "pekf_step.hpp"

namespace pekf {

// A block covers kGroups groups of 64 filters with 2 kGroups waves: waves 0..3 are the groups'
// measurement waves, waves 4..7 their filter waves.  A block's waves go to the CU's SIMDs in turn, so
// each SIMD gets one wave of each kind (with a 2-wave block the two kinds would pair up per SIMD).
constexpr int kGroups = 4;
constexpr int kSplitBlock = 2 * kGroups * kWave;
constexpr int kQ4 = 10;                 // t0 t1 t2 t3 dw1 dw2 dw3 sxy sxz syz

// R' = diag(P2, 1) Fv^T of the record's (acc, mag) in the reference frame's basis: the first half
// of wahba_quat_toward<2, RW> with the frame of ekf_record_step (same expressions).
template <class RW>
__device__ __forceinline__ void wahba_rprime(const RW &W, const double *acc, const double *mag, double *R) {
    const double ka = fabs(acc[2]);
    Frame V;
    make_frame<2>(acc, mag, V, 1.0 - ka);
    const double km = 1.0 - ka;
    const double kw = km * W.b2W, kb = km * W.b1W;
    double p = ka * W.aW * V.alpha + kb * V.beta1 + kw * V.beta2;
    double s = kw * V.beta1 - kb * V.beta2;
    const double ih = rsqrt<2>(p * p + s * s);
    p *= ih;
    s *= ih;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        R[j] = p * V.e1[j] - s * V.e2[j];
        R[3 + j] = s * V.e1[j] + p * V.e2[j];
        R[6 + j] = V.u3[j];
    }
}

// the entries of Q4 of the rotation M (q4_times' first half, same expressions)
__device__ __forceinline__ void q4_entries(const double *M, double *q) {
    const double a = 1.0 + M[8], b = 1.0 - M[8], s = M[0] + M[4], d = M[0] - M[4];
    q[0] = a + s;
    q[1] = b + d;
    q[2] = b - d;
    q[3] = a - s;
    q[4] = M[7] - M[5];
    q[5] = M[2] - M[6];
    q[6] = M[3] - M[1];
    q[7] = M[1] + M[3];
    q[8] = M[2] + M[6];
    q[9] = M[5] + M[7];
}

// s_barrier after this wave's LDS accesses have completed; no wait on the record loads in flight
// (a workgroup-scope fence would also drain those)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One record of ekf_record_step<double, true, LAZY, true> with Wahba's Q4 entries supplied (qe);
// acc / mag are read only by the rare |q.z| < 1/4 fallback, which rebuilds R' from them.
template <bool LAZY, class RW>
__device__ __forceinline__ void filter_step_q4(double *x, double n2, Sym4T<double> &P, const RW &Wr,
                                               const StepK<double> &k, const double *gy, double dt_ns,
                                               bool missing, const double *qe, const double *acc,
                                               const double *mag) {
    const double n2x = LAZY ? x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3] : n2;
    double z[4], kk, irk;
    const double th2x2 = fma_half(gy[2], gy[2], fma(gy[1], gy[1], gy[0] * gy[0]));
    rk4_closed_w(x, n2x, dt_ns, gy, th2x2, z, kk, irk);                    // (:62)
    const double g2x = LAZY ? ((irk * irk) * kk) * k.g2 : k.g2;
    const Sym4T<double> S2 = innovation_cov_n_w(P, gy, th2x2, x, LAZY ? 1.0 : n2, k.g2, k.r2, k.rp, g2x);
    if (missing) {
        x[0] = z[0]; x[1] = z[1]; x[2] = z[2]; x[3] = z[3];
        const double hf = 0.5;
        P = {fma(hf, S2.a00, -k.r2), hf * S2.a01, -hf * S2.a02, -hf * S2.a03, fma(hf, S2.a11, -k.r2),
             -hf * S2.a12, -hf * S2.a13, fma(hf, S2.a22, -k.r2), hf * S2.a23, fma(hf, S2.a33, -k.r2)};
        return;
    }
    const Sym4T<double> Si = spd_inverse_schur<double, true, true>(S2);
    // v = Q4 z (q4_times' second half), Y = v sc
    double v[4];
    v[0] = fma(qe[0], z[0], fma(qe[4], z[1], fma(qe[5], z[2], qe[6] * z[3])));
    v[1] = fma(qe[4], z[0], fma(qe[1], z[1], fma(qe[7], z[2], qe[8] * z[3])));
    v[2] = fma(qe[5], z[0], fma(qe[7], z[1], fma(qe[2], z[2], qe[9] * z[3])));
    v[3] = fma(qe[6], z[0], fma(qe[8], z[1], fma(qe[9], z[2], qe[3] * z[3])));
    const double nv = fma(v[0], v[0], fma(v[1], v[1], fma(v[2], v[2], v[3] * v[3])));
    double sc = rsqrt<2>(nv);
    if (PEKF_TAKEN(nv < 1.0, false)) {  // wahba_quat_toward's fallback: the reference's own formula
        // opaque copies of the operands, so that none of the branch's state-independent work (R', the
        // reference frame's q_W) is speculated into the common path
        double ac[3] = {acc[0], acc[1], acc[2]}, mg[3] = {mag[0], mag[1], mag[2]};
        RW Wo = Wr;
        asm volatile("" : "+v"(ac[0]), "+v"(ac[1]), "+v"(ac[2]), "+v"(mg[0]), "+v"(mg[1]), "+v"(mg[2]), "+v"(Wo.pair));
        double R[9], Fw[9], Rw[9], zw[4], vw[4], qw[4];
        wahba_rprime(Wo, ac, mg, R);
        Wo.quat(qw);
        quat_to_rotm(qw, Fw);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) Rw[3 * i + j] = Fw[3 * i] * R[j] + Fw[3 * i + 1] * R[3 + j] + Fw[3 * i + 2] * R[6 + j];
        qmul_left<false>(qw, z, zw);
        rotm_to_quat_flip_reference(Rw, zw, vw, sc);
        qmul_left<true>(qw, vw, v);
    }
    const double e0 = fma_sub(v[0], sc, z[0]), e1 = fma_sub(v[1], sc, z[1]);
    const double e2 = fma_rsub(v[2], sc, z[2]);
    const double e3 = fma_rsub(v[3], sc, z[3]);
    const double u0 = Si.a00 * e0 + Si.a01 * e1 + Si.a02 * e2 + Si.a03 * e3;
    const double u1 = Si.a01 * e0 + Si.a11 * e1 + Si.a12 * e2 + Si.a13 * e3;
    const double u2 = Si.a02 * e0 + Si.a12 * e1 + Si.a22 * e2 + Si.a23 * e3;
    const double u3 = Si.a03 * e0 + Si.a13 * e1 + Si.a23 * e2 + Si.a33 * e3;
    const double sr = sc * k.sy;
    x[0] = fma(v[0], sr, u0); x[1] = fma(v[1], sr, u1);
    x[2] = fma(v[2], sr, -u2); x[3] = fma(v[3], sr, -u3);
    P = Si;
}

template <bool SOA>
__global__ __launch_bounds__(kSplitBlock) void k_run_split(int64_t batch, int64_t n_steps, int64_t window,
                                                          int64_t step0, const float4 *__restrict__ gd,
                                                          const float4 *__restrict__ am,
                                                          const float2 *__restrict__ my,
                                                          const double *__restrict__ refs,
                                                          double *__restrict__ Xio, double *__restrict__ Pio,
                                                          double qs, double rs) {
    __shared__ double q4b[kGroups][2][kQ4][kWave];  // per group, double buffer: record t's entries in slot t & 1
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave)), ln = threadIdx.x % kWave;
    const int grp = wave % kGroups;
    auto &q4s = q4b[grp];
    const int64_t b0 = ((int64_t)blockIdx.x * kGroups + grp) * kWave + ln;
    const bool act = b0 < batch;
    const int64_t b = act ? b0 : batch - 1;  // idle lanes compute on the last filter, store nothing
    const uint32_t off16 = (uint32_t)b * 16u, off8 = (uint32_t)b * 8u;
    const int32_t n32 = (int32_t)n_steps;

    Frame Wf;
    {
        const double a0[3] = {refs[6 * b + 0], refs[6 * b + 1], refs[6 * b + 2]};
        const double m0[3] = {refs[6 * b + 3], refs[6 * b + 4], refs[6 * b + 5]};
        make_frame<true>(a0, m0, Wf);
    }
    RefWLazy Wr;
    Wr.aW = Wf.alpha; Wr.b1W = Wf.beta1; Wr.b2W = Wf.beta2;
    Wr.pair = refs + 6 * b;
    RowCursor rows(gd, am, my, batch, window);
    rows.start((int32_t)(step0 % window));
    OmodMode mode;

    if (wave < kGroups) {  // wave-uniform: a measurement wave
        auto produce = [&](const Rec &rc, int slot) {
            const double acc[3] = {rc.am.x, rc.am.y, rc.am.z};
            const double mag[3] = {rc.am.w, rc.my.x, rc.my.y};
            double R[9], q[kQ4];
            wahba_rprime(Wr, acc, mag, R);
            q4_entries(R, q);
#pragma unroll
            for (int k = 0; k < kQ4; ++k) q4s[slot][k][ln] = q[k];
        };
        Rec ra = rows.load(off16, off8), rb;
        mode.enter();
        for (int32_t t = 0; t < n32; ++t) {
            rows.advance();
            rb = rows.load(off16, off8);  // always a valid row (the window wraps)
            produce(ra, t & 1);
            lds_barrier();  // B_t: record t's entries are in slot t & 1
            ra = rb;
        }
        lds_barrier();      // B_n
        mode.leave();
        return;
    }

    // the filter wave
    double x[4];
    Sym4T<double> P;
    load_state<SOA>(Xio, Pio, b, batch, x, P);
    {
        double qw[4];
        frame_quat(Wf, qw);
        to_ref_basis(qw, x, P, rs);
    }
    const StepK<double> kc = step_consts<double, true>(qs, rs);
    Rec ra = rows.load(off16, off8), rb;
    mode.enter();
    auto step = [&](const Rec &cur, int32_t t, auto lazy) {
        double qe[kQ4];
#pragma unroll
        for (int k = 0; k < kQ4; ++k) qe[k] = q4s[t & 1][k][ln];
        const double gy[3] = {cur.gd.x, cur.gd.y, cur.gd.z};
        const uint32_t word = __float_as_uint(cur.gd.w);
        const double acc[3] = {cur.am.x, cur.am.y, cur.am.z};
        const double mag[3] = {cur.am.w, cur.my.x, cur.my.y};
        filter_step_q4<decltype(lazy)::value>(x, decltype(lazy)::value ? 1.0 : state_norm2(x), P, Wr, kc, gy,
                                              (double)(word & 0x7FFFFFFFu), (word & PEKF_MISSING_MAG_BIT) != 0, qe,
                                              acc, mag);
    };
    lds_barrier();  // B_0
    rows.advance();
    rb = rows.load(off16, off8);
    step(ra, 0, std::false_type{});
    lds_barrier();  // B_1
    for (int32_t t = 1; t < n32;) {
        rows.advance();
        ra = rows.load(off16, off8);
        step(rb, t, std::true_type{});
        lds_barrier();  // B_{t+1}
        if (++t == n32) break;
        rows.advance();
        rb = rows.load(off16, off8);
        step(ra, t, std::true_type{});
        lds_barrier();
        ++t;
    }
    mode.leave();
    from_ref_basis(Wr, x, P, rs);
    if (act) store_state<SOA>(Xio, Pio, b, batch, x, P);
}

// true: launch_run_multi should use k_run_split for this batch (fewer than 2 waves per SIMD of the
// one-lane kernel); PEKF_RUN_SPLIT=0 / 1 forces the choice
bool run_split_wanted(int64_t batch) {
    const char *e = getenv("PEKF_RUN_SPLIT");
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return false;
    const int64_t waves = (batch + kWave - 1) / kWave;
    return waves < 2 * 4 * (int64_t)cus;
}

int launch_run_split(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const float4 *gd,
                     const float4 *am, const float2 *my, const double *refs, double *X, double *P, double q,
                     double r, bool soa, hipStream_t stream) {
    const dim3 grid(grid_for(batch, kGroups * kWave)), block(kSplitBlock);
    if (soa)
        hipLaunchKernelGGL(k_run_split<true>, grid, block, 0, stream, batch, n_steps, window, step0, gd, am, my,
                           refs, X, P, q, r);
    else
        hipLaunchKernelGGL(k_run_split<false>, grid, block, 0, stream, batch, n_steps, window, step0, gd, am, my,
                           refs, X, P, q, r);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_run_split");
    return PEKF_OK;
}

}  // namespace pekf
