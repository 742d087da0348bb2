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
// with the same flags as pekf_run_multi.hip (Makefile RUNMULTIFLAGS), and k_run's loop: rows through
// scalar-offset buffer descriptors (RowCursor64), the next record in flight one row ahead, unrolled by
// two so no record is copied between steps.  At 80 B per record a log replay at scale is as much HBM
// as VALU.
#include "pekf_step.hpp"

namespace pekf {

// k_run's RowCursor for the 80 B record: rows of batch x 32 B (gd, am) and batch x 16 B (my), read
// through buffer descriptors of a chunk of rows with the row's offset in the scalar offset, so the
// next row is two scalar adds and a compare and no vector address arithmetic is kept per record
// (the lane offsets are 32-bit: batch < 2^27, checked on the host).  A double4 is two 16 B loads
// (the second at the instruction's immediate offset).
struct RowCursor64 {
    const char *g, *a, *m;
    uint32_t row32, row16;
    int32_t window, chunk_rows;
    int32_t row = 0, end = 0;
    uint32_t s32 = 0, s16 = 0;
    __amdgpu_buffer_rsrc_t rg, ra, rm;

    __device__ __forceinline__ RowCursor64(const double4 *gd, const double4 *am, const double2 *my, int64_t batch,
                                           int64_t win)
        : g(reinterpret_cast<const char *>(gd)), a(reinterpret_cast<const char *>(am)),
          m(reinterpret_cast<const char *>(my)), row32((uint32_t)batch * 32u), row16((uint32_t)batch * 16u),
          window((int32_t)win) {
        const uint32_t c = (1u << 31) / row32;
        chunk_rows = c ? (int32_t)c : 1;
    }
    __device__ __forceinline__ void start(int32_t r) {
        row = r;
        end = (window - r < chunk_rows) ? window : r + chunk_rows;
        const uint64_t n = (uint64_t)(end - r);
        rg = row_rsrc(g + (uint64_t)r * row32, (int64_t)(n * row32));
        ra = row_rsrc(a + (uint64_t)r * row32, (int64_t)(n * row32));
        rm = row_rsrc(m + (uint64_t)r * row16, (int64_t)(n * row16));
        s32 = 0;
        s16 = 0;
    }
    __device__ __forceinline__ void advance() {
        if (++row == end) {
            start(row == window ? 0 : row);
        } else {
            s32 += row32;
            s16 += row16;
        }
    }
    template <int AUX>
    static __device__ __forceinline__ double4 load4(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t so) {
        const double2 lo = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, off, so, AUX));
        const double2 hi = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u, so, AUX));
        return make_double4(lo.x, lo.y, hi.x, hi.y);
    }
    __device__ __forceinline__ Rec64 load(uint32_t off32, uint32_t off16) const {
        Rec64 v;
        v.gd = load4<PEKF_REC_AUX>(rg, off32, s32);
        v.am = load4<PEKF_REC_AUX>(ra, off32, s32);
        v.my = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rm, off16, s16, PEKF_REC_AUX));
        return v;
    }
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

    const uint32_t lane = (uint32_t)b;
    const uint32_t off32 = lane * 32u, off16 = lane * 16u;
    RowCursor64 rows(gd, am, my, batch, window);
    rows.start((int32_t)(step0 % window));
    Rec64 ra = rows.load(off32, off16), rb;

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

    // One record (main_file.py:42-45) on (x, P) in registers; lazy: X arrives unnormalised (every
    // record after the launch's first)
    auto step = [&](const Rec64 &cur, int32_t t, auto lazy) {
        if (!COUNTS || t < my_steps) {
            const double gy[3] = {cur.gd.x, cur.gd.y, cur.gd.z};
            const double acc[3] = {cur.am.x, cur.am.y, cur.am.z};
            const double mag[3] = {cur.am.w, cur.my.x, cur.my.y};
            auto reload = [&](double *a, double *m) {  // rare: the degenerate-Wahba fallback; the cursor is a row ahead
                const int32_t r = rows.row == 0 ? rows.window - 1 : rows.row - 1;
                const double4 va = RowCursor64::load4<0>(row_rsrc(rows.a + (uint64_t)r * rows.row32, rows.row32), off32, 0);
                const double2 vm = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(
                    row_rsrc(rows.m + (uint64_t)r * rows.row16, rows.row16), off16, 0, 0));
                a[0] = va.x; a[1] = va.y; a[2] = va.z;
                m[0] = va.w; m[1] = vm.x; m[2] = vm.y;
            };
            if constexpr (decltype(lazy)::value)
                ekf_record_step<double, true, true, true, true>(x, 1.0, P, Wr, kc, gy, cur.gd.w, false, acc, mag,
                                                                reload);
            else
                ekf_record_step<double, true, false, true, true>(x, state_norm2(x), P, Wr, kc, gy, cur.gd.w, false, acc,
                                                                 mag, reload);
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
    };
    using eager = std::false_type;
    using lazy = std::true_type;

    // k_run's time loop: unrolled by two with ping-pong records, the next row always in flight and no
    // record copied between steps; the prefetch wraps inside the window, so it is always a valid row
    rows.advance();
    rb = rows.load(off32, off16);
    OmodMode mode;
    mode.enter();
    step(ra, 0, eager{});
    for (int32_t t = 1; t < n32;) {
        rows.advance();
        ra = rows.load(off32, off16);
        step(rb, t, lazy{});
        if (++t == n32) break;
        rows.advance();
        rb = rows.load(off32, off16);
        step(ra, t, lazy{});
        ++t;
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
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 27), "batch must be < 2^27 filters per launch (32-bit lane offsets of 32 B)");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31) && window < ((int64_t)1 << 31),
                   "n_steps and window must be < 2^31 (RowCursor64 holds the window as int32)");
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
