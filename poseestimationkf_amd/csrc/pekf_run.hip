// pekf_run.hip -- the fused hot path: main_file.py:38-47 (Prediction + Correction per record)
// for a whole batch of independent filters, n_steps records per launch.
//
// Mapping (DESIGN.md "Kernel"): one LANE owns one filter, so a wavefront advances 64
// filters in lock-step and every per-step input field is a coalesced 1 KiB (float4) or
// 512 B (float2) wave load from the filter-minor planes.  X (4 f64), the symmetric P
// (10 f64) and the filter's Wahba reference frame live in VGPRs for the whole launch;
// HBM traffic is the 40 B/filter-step input record plus, once per launch, the state
// and reference vectors.  The next step's record is loaded before the current step's
// arithmetic so its latency hides under ~400 VALU instructions of work.
// No MFMA: every contraction is 4x4 / 3x3 per lane.
#include "pekf_step.hpp"

namespace pekf {

// AoS <-> SoA state conversion (see load_state); P's 10 unique entries are the upper triangle.
// (the AoS side in coalesced wave tiles: this kernel is pure data movement)
__global__ __launch_bounds__(kRunBlock) void k_state_layout(int64_t batch, double *Xa, double *Pa,
                                                            double *Xs, double *Ps, int to_soa) {
    __shared__ double pool[kRunBlock / kWave * tile_doubles<16>()];
    const WaveTile tl(pool, tile_doubles<16>(), batch);
    const bool act = tl.active();
    const int64_t b = tl.first + tl.lane;
    double x[4], pv[16];
    if (to_soa) {  // uniform
        double cx[4], cp[16];
        tl.gather(Xa, cx);
        tl.gather(Pa, cp);
        tl.to_lanes(cx, x);
        tl.to_lanes(cp, pv);
        if (act) store_state<true>(Xs, Ps, b, batch, x, sym_from16<double>(pv));
    } else {
        Sym4T<double> S = {};
        x[0] = x[1] = x[2] = x[3] = 0.0;
        if (act) load_state<true>(Xs, Ps, b, batch, x, S);
        sym_to16(S, pv);
        tl.store(Xa, x);
        tl.store(Pa, pv);
    }
}

__global__ __launch_bounds__(kRunBlock) void k_reset(int64_t batch, double *X, double *P) {
    __shared__ double pool[kRunBlock / kWave * tile_doubles<16>()];
    const WaveTile tl(pool, tile_doubles<16>(), batch);
    const double x[4] = {1.0, 0.0, 0.0, 0.0};
    double pv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) pv[k] = (k % 5 == 0) ? 1.0 : 0.0;
    tl.store(X, x);
    tl.store(P, pv);
}

// One record per filter from FP64 arrays (the filter handle's online update,
// pekf_filter_update): dt = t - previousT per filter (ExtendedKalmanFilter.py:62,67), then the
// same ekf_record_step as the stream kernel.  Record arrays are filter-major ([batch][3]).
template <bool MIXED, bool SOA>
__global__ __launch_bounds__(kRunBlock) void k_update(int64_t batch, const double *__restrict__ gyro,
                                                      const int64_t *__restrict__ t_ns,
                                                      const double *__restrict__ acc,
                                                      const double *__restrict__ mag,
                                                      const uint8_t *__restrict__ missing,
                                                      const double *__restrict__ refs, int64_t *__restrict__ prev_t,
                                                      double *__restrict__ Xio, double *__restrict__ Pio, double qs,
                                                      double rs, double *__restrict__ x_out) {
    using PT = typename std::conditional<MIXED, float, double>::type;
    // the [batch][3] / [batch][6] operands (and AoS state) move in coalesced wave tiles
    constexpr int kW = SOA ? 6 : 16;
    __shared__ double pool[kRunBlock / kWave * tile_doubles<kW>()];
    const WaveTile tl(pool, tile_doubles<kW>(), batch);
    const bool act = tl.active();
    const int64_t b = act ? tl.first + tl.lane : 0;  // idle lanes compute on filter 0, store nothing
    double cr[6], cg[3], ca[3], cm[3];
    tl.gather(refs, cr);
    tl.gather(gyro, cg);
    tl.gather(acc, ca);
    tl.gather(mag, cm);
    double x[4];
    Sym4T<PT> P;
    double pv[16];
    if constexpr (SOA) {
        load_state<true>(Xio, Pio, b, batch, x, P);
    } else {
        double cx[4], cp[16];
        tl.gather(Xio, cx);
        tl.gather(Pio, cp);
        tl.to_lanes(cx, x);
        tl.to_lanes(cp, pv);
        P = sym_from16<PT>(pv);
    }
    const int64_t t = t_ns[b];
    const double dt_ns = (double)(t - prev_t[b]);
    const bool miss = missing && missing[b];
    double rf[6], g[3], a[3], m[3];
    tl.to_lanes(cr, rf);
    tl.to_lanes(cg, g);
    tl.to_lanes(ca, a);
    tl.to_lanes(cm, m);
    Frame Wf;
    make_frame<true>(rf, rf + 3, Wf);
    auto reload = [&](double *ra, double *rm) {  // rare: the degenerate-Wahba fallback
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            ra[i] = acc[3 * b + i];
            rm[i] = mag[3 * b + i];
        }
    };
    ekf_record_step<PT>(x, state_norm2(x), P, Wf, step_consts<PT, false>(qs, rs), g, dt_ns, miss, a, m, reload);
    if (act) prev_t[b] = t;
    if constexpr (SOA) {
        if (act) store_state<true>(Xio, Pio, b, batch, x, P);
    } else {
        sym_to16(P, pv);
        tl.store(Xio, x);
        tl.store(Pio, pv);
    }
    if (x_out) tl.store(x_out, x);
}

int launch_update(int64_t batch, const double *gyro, const int64_t *t_ns, const double *acc, const double *mag,
                  const uint8_t *missing, const double *refs, int64_t *prev_t, double *X, double *P, double q,
                  double r, double *x_out, uint32_t flags, hipStream_t stream) {
    const dim3 grid(grid_for(batch, kRunBlock)), block(kRunBlock);
    const bool mixed = flags & PEKF_RUN_MIXED_PRECISION, soa = flags & PEKF_RUN_STATE_SOA;
#define PEKF_LAUNCH_UPDATE(MX, SO)                                                                \
    hipLaunchKernelGGL((k_update<MX, SO>), grid, block, 0, stream, batch, gyro, t_ns, acc, mag, missing, \
                       refs, prev_t, X, P, q, r, x_out)
    if (mixed) {
        if (soa) PEKF_LAUNCH_UPDATE(true, true); else PEKF_LAUNCH_UPDATE(true, false);
    } else {
        if (soa) PEKF_LAUNCH_UPDATE(false, true); else PEKF_LAUNCH_UPDATE(false, false);
    }
#undef PEKF_LAUNCH_UPDATE
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_update");
    return PEKF_OK;
}

}  // namespace pekf

using namespace pekf;

extern "C" {

int pekf_run_ext_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                     const void *plane_gd, const void *plane_am, const void *plane_my, const double *dt_ext,
                     const double *refs, double *X, double *P, double q, double r, double *traj,
                     const int32_t *counts, uint32_t flags, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_steps >= 0, "negative size");
    PEKF_CHECK_ARG((flags & ~(uint32_t)(PEKF_RUN_MIXED_PRECISION | PEKF_RUN_STATE_SOA)) == 0, "unknown flags");
    if (batch == 0 || n_steps == 0) return PEKF_OK;
    PEKF_CHECK_ARG(window > 0 && step0 >= 0, "window must be > 0 and step0 >= 0");
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31), "n_steps must be < 2^31 records per launch");
    PEKF_CHECK_ARG(plane_gd && plane_am && plane_my && refs && X && P, "null pointer");
    PEKF_CHECK_ARG(((uintptr_t)plane_gd % 16 == 0) && ((uintptr_t)plane_am % 16 == 0) &&
                       ((uintptr_t)plane_my % 8 == 0) && ((uintptr_t)traj % 16 == 0) &&
                       ((uintptr_t)dt_ext % 8 == 0),
                   "misaligned plane / traj pointer");
    PEKF_CHECK_ARG(r > 0.0, "r must be > 0 (S = P- + rI must be SPD)");
    const dim3 grid(grid_for(batch, kRunBlock)), block(kRunBlock);
    const auto *gd = static_cast<const float4 *>(plane_gd);
    const auto *am = static_cast<const float4 *>(plane_am);
    const auto *my = static_cast<const float2 *>(plane_my);
    const bool mixed = flags & PEKF_RUN_MIXED_PRECISION, soa = flags & PEKF_RUN_STATE_SOA;
    if (n_steps > 1)  // the multi-record kernels live in pekf_run_multi.hip (its own scheduling strategy)
        return launch_run_multi(batch, n_steps, window, step0, gd, am, my, dt_ext, refs, X, P, q, r, traj, counts,
                                mixed, soa, as_stream(stream));
    // one-record launch (online serving)
#define PEKF_LAUNCH_ONE(TR, MX, SO, CN, LD)                                                                   \
    hipLaunchKernelGGL((k_run<TR, MX, SO, CN, true, false, LD>), grid, block, 0, as_stream(stream), batch, n_steps, \
                       window, step0, gd, am, my, refs, X, P, q, r, traj, counts, dt_ext)
#define PEKF_LAUNCH_ONE0(TR, MX, SO, CN) \
    do { if (dt_ext) PEKF_LAUNCH_ONE(TR, MX, SO, CN, true); else PEKF_LAUNCH_ONE(TR, MX, SO, CN, false); } while (0)
#define PEKF_LAUNCH_ONE1(TR, MX, SO) \
    do { if (counts) PEKF_LAUNCH_ONE0(TR, MX, SO, true); else PEKF_LAUNCH_ONE0(TR, MX, SO, false); } while (0)
#define PEKF_LAUNCH_ONE2(TR, MX) \
    do { if (soa) PEKF_LAUNCH_ONE1(TR, MX, true); else PEKF_LAUNCH_ONE1(TR, MX, false); } while (0)
    if (traj) {
        if (mixed) PEKF_LAUNCH_ONE2(true, true); else PEKF_LAUNCH_ONE2(true, false);
    } else {
        if (mixed) PEKF_LAUNCH_ONE2(false, true); else PEKF_LAUNCH_ONE2(false, false);
    }
#undef PEKF_LAUNCH_ONE2
#undef PEKF_LAUNCH_ONE1
#undef PEKF_LAUNCH_ONE0
#undef PEKF_LAUNCH_ONE
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_run");
    return PEKF_OK;
}

int pekf_run_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                 const void *plane_gd, const void *plane_am, const void *plane_my,
                 const double *refs, double *X, double *P, double q, double r, double *traj,
                 const int32_t *counts, uint32_t flags, void *stream) {
    return pekf_run_ext_dev(batch, n_steps, window, step0, plane_gd, plane_am, plane_my, nullptr, refs, X, P, q, r,
                            traj, counts, flags, stream);
}

int pekf_reset_state_dev(int64_t batch, double *X, double *P, void *stream) {
    PEKF_CHECK_ARG(batch >= 0, "negative size");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(X && P, "null pointer");
    hipLaunchKernelGGL(k_reset, dim3(grid_for(batch, kRunBlock)), dim3(kRunBlock), 0,
                       as_stream(stream), batch, X, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_reset");
    return PEKF_OK;
}

int pekf_state_layout_dev(int64_t batch, double *X_aos, double *P_aos, double *X_soa, double *P_soa,
                          int to_soa, void *stream) {
    PEKF_CHECK_ARG(batch >= 0, "negative size");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(X_aos && P_aos && X_soa && P_soa, "null pointer");
    hipLaunchKernelGGL(k_state_layout, dim3(grid_for(batch, kRunBlock)), dim3(kRunBlock), 0,
                       as_stream(stream), batch, X_aos, P_aos, X_soa, P_soa, to_soa);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_state_layout");
    return PEKF_OK;
}

}  // extern "C"
