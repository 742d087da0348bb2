// pekf_run64.hip -- the multi-record fused launch over FP64 records (recorded logs).
//
// The reference parses its logs into float64 (ReadFile.py:14-21) and main_file.py:38-47 feeds those
// doubles to Prediction / Correction.  The stream planes of pekf_run_dev hold the 40 B record (f32
// samples, a u32 ns dt word), which rounds such inputs to f32 (5.4e-8 on config 1's log).  Here the
// record is 80 B of doubles in three filter-minor planes [window][batch]:
//   GD double4 {gx, gy, gz, dt_ns}  AM double4 {ax, ay, az, mx}  MY double2 {my, mz}
// with dt the float64 T - previousT itself (ExtendedKalmanFilter.py:62): any pause, clock step or
// fraction, no escape word.  Every record carries a magnetometer sample (a log always does).
//
// The arithmetic is k_run's multi-record loop step for step -- reference-frame basis, covariance as
// N, lazy |X|, omod halvings (ekf_record_step<double, MC, LAZY, OM, PIN>, pekf_step.hpp) -- so a
// window of f32-representable values gives k_run's state bit for bit (tests/test_rec64.py).  Compiled
// with the same flags as pekf_run_multi.hip (Makefile RUNMULTIFLAGS).  Loads are plain global loads
// of the next record, one row ahead: at 80 B per record a log replay at scale is as much HBM as VALU.
#include "pekf_step.hpp"

namespace pekf {

struct Rec64 {
    double4 gd, am;
    double2 my;
};

template <bool TRAJ, bool COUNTS>
__global__ __launch_bounds__(kRunBlock) PEKF_RUN_ATTR void k_run64(
    int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const double4 *__restrict__ gd,
    const double4 *__restrict__ am, const double2 *__restrict__ my, const double *__restrict__ refs,
    double *__restrict__ Xio, double *__restrict__ Pio, double qs, double rs, double *__restrict__ traj,
    const int32_t *__restrict__ counts) {
    const int64_t b = (int64_t)blockIdx.x * kRunBlock + threadIdx.x;
    if (b >= batch) return;
    const int32_t n32 = (int32_t)n_steps;
    const int32_t my_steps = COUNTS ? (counts[b] < n32 ? counts[b] : n32) : n32;

    Frame Wf;  // the Wahba reference frame of (acc0, mag0) (Wahba.py:4-6)
    {
        const double a0[3] = {refs[6 * b + 0], refs[6 * b + 1], refs[6 * b + 2]};
        const double m0[3] = {refs[6 * b + 3], refs[6 * b + 4], refs[6 * b + 5]};
        make_frame<true>(a0, m0, Wf);
    }
    double x[4];
    Sym4T<double> P;
    load_state<false>(Xio, Pio, b, batch, x, P);
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
    const StepK<double> kc = step_consts<double, true>(qs, rs);

    auto load = [&](int64_t row) -> Rec64 {
        const int64_t i = row * batch + b;
        return {gd[i], am[i], my[i]};
    };
    int64_t row = step0 % window;
    Rec64 cur = load(row);
    OmodMode mode;
    mode.enter();
    for (int32_t t = 0; t < n32; ++t) {
        const int64_t next = row + 1 == window ? 0 : row + 1;
        const Rec64 nxt = load(next);  // in flight while this record is applied
        if (!COUNTS || t < my_steps) {
            const double gy[3] = {cur.gd.x, cur.gd.y, cur.gd.z};
            const double acc[3] = {cur.am.x, cur.am.y, cur.am.z};
            const double mag[3] = {cur.am.w, cur.my.x, cur.my.y};
            const int64_t r = row;
            auto reload = [&](double *a, double *m) {  // rare: the degenerate-Wahba fallback
                const double4 va = am[r * batch + b];
                const double2 vm = my[r * batch + b];
                a[0] = va.x; a[1] = va.y; a[2] = va.z;
                m[0] = va.w; m[1] = vm.x; m[2] = vm.y;
            };
            if (t == 0)
                ekf_record_step<double, true, false, true, true>(x, state_norm2(x), P, Wr, kc, gy, cur.gd.w, false, acc,
                                                                 mag, reload);
            else
                ekf_record_step<double, true, true, true, true>(x, 1.0, P, Wr, kc, gy, cur.gd.w, false, acc, mag,
                                                                reload);
        }
        if constexpr (TRAJ) {
            double xo[4] = {x[0], x[1], x[2], x[3]};
            if (!COUNTS || my_steps > 0) {  // (no record in this launch: the stored X, as k_run)
                const double in = rsqrt<true>(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]);
                const double xn[4] = {x[0] * in, x[1] * in, x[2] * in, x[3] * in};
                double qw[4];
                Wr.quat(qw);
                qmul_left<false>(qw, xn, xo);
            }
            double2 *o = reinterpret_cast<double2 *>(traj + (int64_t)t * batch * 4) + 2 * b;
            o[0] = make_double2(xo[0], xo[1]);
            o[1] = make_double2(xo[2], xo[3]);
        }
        cur = nxt;
        row = next;
    }
    mode.leave();
    if (COUNTS && my_steps == 0) return;
    from_ref_basis(Wr, x, P, rs);
    store_state<false>(Xio, Pio, b, batch, x, P);
}

}  // namespace pekf

using namespace pekf;

extern "C" int pekf_run_rec64_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                                  const void *plane_gd, const void *plane_am, const void *plane_my,
                                  const double *refs, double *X, double *P, double q, double r, double *traj,
                                  const int32_t *counts, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_steps >= 0, "negative size");
    if (batch == 0 || n_steps == 0) return PEKF_OK;
    PEKF_CHECK_ARG(window > 0 && step0 >= 0, "window must be > 0 and step0 >= 0");
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31), "n_steps must be < 2^31 records per launch");
    PEKF_CHECK_ARG(plane_gd && plane_am && plane_my && refs && X && P, "null pointer");
    PEKF_CHECK_ARG(((uintptr_t)plane_gd % 32 == 0) && ((uintptr_t)plane_am % 32 == 0) &&
                       ((uintptr_t)plane_my % 16 == 0) && ((uintptr_t)traj % 16 == 0),
                   "misaligned plane / traj pointer");
    PEKF_CHECK_ARG(r > 0.0, "r must be > 0 (S = P- + rI must be SPD)");
    const dim3 grid(grid_for(batch, kRunBlock)), block(kRunBlock);
    const auto *gd = static_cast<const double4 *>(plane_gd);
    const auto *am = static_cast<const double4 *>(plane_am);
    const auto *my = static_cast<const double2 *>(plane_my);
    const hipStream_t s = as_stream(stream);
#define PEKF_LAUNCH_RUN64(TR, CN)                                                                               \
    hipLaunchKernelGGL((k_run64<TR, CN>), grid, block, 0, s, batch, n_steps, window, step0, gd, am, my, refs, X, P, \
                       q, r, traj, counts)
    if (traj) {
        if (counts) PEKF_LAUNCH_RUN64(true, true); else PEKF_LAUNCH_RUN64(true, false);
    } else {
        if (counts) PEKF_LAUNCH_RUN64(false, true); else PEKF_LAUNCH_RUN64(false, false);
    }
#undef PEKF_LAUNCH_RUN64
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_run64");
    return PEKF_OK;
}
