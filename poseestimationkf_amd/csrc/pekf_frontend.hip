// pekf_frontend.hip -- the live server's pre-processing front-end on the device:
// raw phone events -> the 40 B records the filter consumes (what the server logs as gyro / T /
// Mag_1 / Acc_1).  One lane per filter walks its event stream through the state machine of
// Parser::WriteKalmanFilterMeasurement (KFS/Parser.cpp:148-219); when a gyro sample has both an
// accelerometer and a magnetometer sample after it, ExecuteKalmanFilter (Parser.cpp:229-257)
// interpolates both to the gyro time (:259-267), normalises them (:221-228) and low-pass filters
// them (alpha, from a zero state: KalmanFilter.cpp:16-18,21-24,279-303); the record's dt is the
// gyro time minus the previous record's (KalmanFilter.cpp:306-308).  Arithmetic in FP64 (one
// reciprocal / rsqrt with a Newton step instead of IEEE divisions: ~1e-15 relative), records
// rounded to f32 like every record of the stream.  Event plane: EV float4 {x, y, z, bits(word)},
// word = (ns gap to the previous event << 2) | type, [n_events][batch]: 16 B per event, coalesced.
#include "pekf_internal.hpp"
#include "pekf_math.hpp"

namespace pekf {

constexpr int kFeBlock = 256;
#ifndef PEKF_FE_RING
#define PEKF_FE_RING 9
#endif
enum : uint32_t { kEvAcc = 0, kEvGyro = 1, kEvMag = 2 };

struct V3 {
    double x, y, z;
};
struct F3 {
    float x, y, z;
};
__device__ __forceinline__ V3 widen(const F3 &f) { return {f.x, f.y, f.z}; }
// component-wise c ? a : b (a struct-valued ?: would go through scratch memory)
__device__ __forceinline__ V3 sel(bool c, const V3 &a, const V3 &b) {
    return {c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}
__device__ __forceinline__ F3 sel(bool c, const F3 &a, const F3 &b) {
    return {c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}

// Parser::NormalizeValues (:221-228) with one rsqrt instead of a sqrt and three divisions
__device__ __forceinline__ V3 normalised(const V3 &v) {
    const double in = rsqrt<true>((v.x * v.x + v.y * v.y) + v.z * v.z);
    return {v.x * in, v.y * in, v.z * in};
}

__global__ __launch_bounds__(kFeBlock) void k_frontend(int64_t batch, int64_t n_events,
                                                       const float4 *__restrict__ ev,
                                                       const double *__restrict__ init,
                                                       const int64_t *__restrict__ t_init, double alpha,
                                                       int64_t r_max, float4 *__restrict__ gd,
                                                       float4 *__restrict__ am, float2 *__restrict__ my,
                                                       int32_t *__restrict__ counts, double *__restrict__ refs,
                                                       int *__restrict__ err) {
    const int64_t b = (int64_t)blockIdx.x * kFeBlock + threadIdx.x;
    if (b >= batch) return;
    // phase-2 state: acc_0 / mag_0 = raw means at the initialisation time (Parser.cpp:44-53)
    V3 acc0 = {init[6 * b + 0], init[6 * b + 1], init[6 * b + 2]};
    V3 mag0 = {init[6 * b + 3], init[6 * b + 4], init[6 * b + 5]};
    const double t_start = (double)t_init[b];
    double t_acc0 = t_start, t_mag0 = t_start, prev_t = t_start;
    {   // the filter's reference vectors: normalised phase-2 means (Parser.cpp:48-49)
        const V3 a = normalised(acc0), m = normalised(mag0);
        refs[6 * b + 0] = a.x; refs[6 * b + 1] = a.y; refs[6 * b + 2] = a.z;
        refs[6 * b + 3] = m.x; refs[6 * b + 4] = m.y; refs[6 * b + 5] = m.z;
    }
    V3 acc1 = {0, 0, 0}, mag1 = {0, 0, 0};  // sensor samples (exact f32 values, kept widened)
    F3 gyro = {0, 0, 0};
    double t_acc1 = 0, t_mag1 = 0, t_gyro = 0;
    bool gyro_set = false, acc1_set = false, mag1_set = false;
    V3 lpf_acc = {0, 0, 0}, lpf_mag = {0, 0, 0};
    const double beta = 1.0 - alpha;
    int64_t r = 0;
    int bad = 0;

    // Emission is deferred: when a lane completes a record, only its inputs are copied aside
    // (pend), and the expensive part -- two interpolations with a reciprocal, two normalisations
    // with an rsqrt, the low-pass and the f32 packing -- runs for the whole wave once every
    // kFlush events instead of on every event some lane emits (which, with 64 lanes, is nearly
    // every event).  A lane needs at least 3 events (gyro, acc, mag) between two records, so
    // with kFlush = 3 it never has two pending.  Arithmetic is unchanged: the time differences
    // are formed at emission, exactly as lerp_to would form them.
    constexpr int kFlush = 3;
    bool pend = false;
    F3 p_gyro = {0, 0, 0};
    V3 p_acc0 = {0, 0, 0}, p_mag0 = {0, 0, 0}, p_acc1 = {0, 0, 0}, p_mag1 = {0, 0, 0};
    double p_dt = 0, p_an = 0, p_ad = 1, p_mn = 0, p_md = 1;  // dt, acc / mag lerp num and den
    auto flush = [&]() {
        if (!pend) return;
        pend = false;
        // Parser::LinearInterpolationSensor (:259-267): (y2 - y1) / (t2 - t1) * (t3 - t1) + y1, the
        // division taken as one reciprocal.  Timestamps are integer ns held in doubles (exact below
        // 2^53), so t3 - t1 and t2 - t1 are the exact differences (double)t3 - (double)t1 gives.
        const double fa = p_an * recip<true>(p_ad), fm = p_mn * recip<true>(p_md);
        const V3 a1 = p_acc1, m1 = p_mag1;
        const V3 a = normalised({(a1.x - p_acc0.x) * fa + p_acc0.x, (a1.y - p_acc0.y) * fa + p_acc0.y,
                                 (a1.z - p_acc0.z) * fa + p_acc0.z});
        const V3 m = normalised({(m1.x - p_mag0.x) * fm + p_mag0.x, (m1.y - p_mag0.y) * fm + p_mag0.y,
                                 (m1.z - p_mag0.z) * fm + p_mag0.z});
        lpf_mag = {alpha * m.x + beta * lpf_mag.x, alpha * m.y + beta * lpf_mag.y, alpha * m.z + beta * lpf_mag.z};
        lpf_acc = {alpha * a.x + beta * lpf_acc.x, alpha * a.y + beta * lpf_acc.y, alpha * a.z + beta * lpf_acc.z};
        if (!(p_dt >= 0.0 && p_dt < 2147483648.0)) bad |= 1;  // not representable in the 31-bit dt word
        if (r < r_max) {
            const int64_t o = r * batch + b;
            gd[o] = make_float4((float)p_gyro.x, (float)p_gyro.y, (float)p_gyro.z,
                                __uint_as_float((uint32_t)fmin(fmax(p_dt, 0.0), 2147483647.0)));
            am[o] = make_float4((float)lpf_acc.x, (float)lpf_acc.y, (float)lpf_acc.z, (float)lpf_mag.x);
            my[o] = make_float2((float)lpf_mag.y, (float)lpf_mag.z);
        } else {
            bad |= 2;  // more records than the output window holds
        }
        ++r;
    };

    // Events stream through a register ring of kFlush records loaded kFlush events ahead (the
    // loop is unrolled by kFlush so every ring index is static; the row is clamped to the last
    // event, so the loads past the end read a valid row and need no predicate).
    const uint32_t lane = (uint32_t)b;
    auto load = [&](int64_t e) -> float4 {
        const int64_t row = e < n_events ? e : n_events - 1;
        return (ev + row * batch)[lane];
    };
    double t = t_start;
    auto event = [&](const float4 v4) {
        const uint32_t word = __float_as_uint(v4.w);
        const uint32_t ty = word & 3u;
        t += (double)(word >> 2);  // the event word carries the ns gap to the previous event
        // Parser::WriteKalmanFilterMeasurement (Parser.cpp:148-219), branch-free: each state
        // variable is one select, so nothing is copied between divergent paths.
        //   before a gyro sample: acc -> acc_0, mag -> mag_0, gyro -> gyro (gyro_is_set);
        //   after it: acc -> acc_1, mag -> mag_1 (set); a new gyro replaces the gyro and shifts a set
        //   acc_1 -> acc_0 / mag_1 -> mag_0, clearing both flags.
        const bool isA = ty == kEvAcc, isM = ty == kEvMag, isG = ty == kEvGyro;
        const bool gs = gyro_set;
        const double vx = v4.x, vy = v4.y, vz = v4.z;
        const bool wA1 = isA && gs, wM1 = isM && gs;
        acc1 = sel(wA1, V3{vx, vy, vz}, acc1);
        t_acc1 = wA1 ? t : t_acc1;
        mag1 = sel(wM1, V3{vx, vy, vz}, mag1);
        t_mag1 = wM1 ? t : t_mag1;
        const bool a1s = wA1 || (acc1_set && !(isG && gs)), m1s = wM1 || (mag1_set && !(isG && gs));
        const bool sA = isG && gs && acc1_set, sM = isG && gs && mag1_set;  // gyro shift
        // ExecuteKalmanFilter (Parser.cpp:229-257) once acc_1 and mag_1 are both set: record its
        // inputs (pending until the next flush), then acc_0 <- acc_1, mag_0 <- mag_1, flags cleared
        const bool emit = a1s && m1s;
        if (emit) {
            pend = true;
            p_gyro = gyro; p_dt = t_gyro - prev_t;
            p_acc0 = acc0; p_acc1 = acc1; p_an = t_gyro - t_acc0; p_ad = t_acc1 - t_acc0;
            p_mag0 = mag0; p_mag1 = mag1; p_mn = t_gyro - t_mag0; p_md = t_mag1 - t_mag0;
            prev_t = t_gyro;
        }
        const bool wA0 = isA && !gs, wM0 = isM && !gs;
        const bool cA = sA || emit, cM = sM || emit;  // acc_0 <- acc_1 (shift or after a record)
        acc0 = sel(wA0, V3{vx, vy, vz}, sel(cA, acc1, acc0));
        t_acc0 = wA0 ? t : (cA ? t_acc1 : t_acc0);
        mag0 = sel(wM0, V3{vx, vy, vz}, sel(cM, mag1, mag0));
        t_mag0 = wM0 ? t : (cM ? t_mag1 : t_mag0);
        gyro = sel(isG, F3{v4.x, v4.y, v4.z}, gyro);
        t_gyro = isG ? t : t_gyro;
        gyro_set = (gs || isG) && !emit;
        acc1_set = a1s && !emit;
        mag1_set = m1s && !emit;
    };
    if (n_events > 0) {
        constexpr int kRing = PEKF_FE_RING;  // events in flight per lane (a multiple of kFlush)
        static_assert(kRing % kFlush == 0, "the ring depth must be a multiple of the flush period");
        float4 ring[kRing];
#pragma unroll
        for (int k = 0; k < kRing; ++k) ring[k] = load(k);
        for (int64_t e0 = 0; e0 < n_events; e0 += kRing) {
#pragma unroll
            for (int k = 0; k < kRing; ++k) {
                if (e0 + k >= n_events) break;  // uniform
                const float4 v4 = ring[k];
                ring[k] = load(e0 + k + kRing);
                event(v4);
                if ((k + 1) % kFlush == 0) flush();
            }
        }
        flush();  // a record completed in a trailing partial group
    }
    counts[b] = (int32_t)(r < r_max ? r : r_max);
    if (bad && err) atomicOr(err, bad);
}

// Phase 2 of the server's Parser (ProcessString, Parser.cpp:36-58; initialMeanAndCovariance,
// :84-140; InitialValues.cpp): the first n_avg samples of each sensor type are averaged (a
// sequential FP64 sum divided by n_avg) and their sample variance formed ((x - mean)^2 summed in
// order, divided by n_avg - 1).  A sensor counts as initialised at its first sample after those
// n_avg; the first event after all three are initialised builds the KalmanFilter (T0 = its time,
// acc_0 / mag_0 = the raw means at that time), and every later phase-2 event moves the acc_0 / mag_0
// time and previousT to its own (setAcc0 / setMag0, UpdateLatestPreviousTime).  So phase 3 starts
// from init = {mean acc, mean mag} at t_init = the last phase-2 event's time -- exactly the inputs of
// pekf_frontend_dev.  Same event planes as phase 3; two passes over them (the variance needs the
// mean first, as InitialValues::compute_mean_and_variance has it).
__global__ __launch_bounds__(kFeBlock) void k_frontend_init(int64_t batch, int64_t n_events, const float4 *__restrict__ ev,
                                                            const int64_t *__restrict__ t_start, int n_avg,
                                                            double *__restrict__ init, int64_t *__restrict__ t_init,
                                                            double *__restrict__ stats, int32_t *__restrict__ ready) {
    const int64_t b = (int64_t)blockIdx.x * kFeBlock + threadIdx.x;
    if (b >= batch) return;
    const uint32_t lane = (uint32_t)b;
    double sum[3][3] = {};  // [type][xyz]
    int cnt[3] = {0, 0, 0};
    bool done[3] = {false, false, false};  // Acc_ / Gyr_ / Mag_initialized
    bool kalman = false;
    int64_t t = t_start[b], t_last = t;
    // events come kInitRing rows at a time, all loads issued before the first is used (the loop body
    // is a few adds, so without it each wave would wait out one memory latency per event); rows past
    // the end are clamped to the last row and not processed
    constexpr int kInitRing = 8;
    auto row = [&](int64_t e) -> float4 { return (ev + (e < n_events ? e : n_events - 1) * batch)[lane]; };
    for (int64_t e0 = 0; e0 < n_events; e0 += kInitRing) {
        float4 r[kInitRing];
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) r[k] = row(e0 + k);
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) {
            if (e0 + k >= n_events) break;  // uniform
            const float4 v4 = r[k];
            const uint32_t word = __float_as_uint(v4.w);
            const int ty = (int)(word & 3u);
            t += (int64_t)(word >> 2);
            if (!(done[0] && done[1] && done[2])) {
                if (ty <= 2) {
                    if (cnt[ty] < n_avg) {
                        sum[ty][0] += (double)v4.x;
                        sum[ty][1] += (double)v4.y;
                        sum[ty][2] += (double)v4.z;
                        ++cnt[ty];
                    } else {
                        done[ty] = true;
                    }
                }
            } else {
                kalman = true;  // the KalmanFilter is built at the first such event, later ones move its time
                t_last = t;
            }
        }
    }
    double mean[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j) mean[k][j] = sum[k][j] / (double)n_avg;
    // second pass: the variance of the first n_avg samples of each type, in their order
    double var[3][3] = {};
    int c2[3] = {0, 0, 0};
    for (int64_t e0 = 0; e0 < n_events; e0 += kInitRing) {
        if (c2[0] >= n_avg && c2[1] >= n_avg && c2[2] >= n_avg) break;
        float4 r[kInitRing];
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) r[k] = row(e0 + k);
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) {
            if (e0 + k >= n_events) break;  // uniform
            const float4 v4 = r[k];
            const int ty = (int)(__float_as_uint(v4.w) & 3u);
            if (ty <= 2 && c2[ty] < n_avg) {
#pragma clang fp contract(off)
                const double d0 = (double)v4.x - mean[ty][0], d1 = (double)v4.y - mean[ty][1],
                             d2 = (double)v4.z - mean[ty][2];
                var[ty][0] += d0 * d0;
                var[ty][1] += d1 * d1;
                var[ty][2] += d2 * d2;
                ++c2[ty];
            }
        }
    }
    const double nan = __builtin_nan("");
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        init[6 * b + j] = kalman ? mean[kEvAcc][j] : nan;
        init[6 * b + 3 + j] = kalman ? mean[kEvMag][j] : nan;
    }
    t_init[b] = t_last;
    ready[b] = kalman ? 1 : 0;
    if (stats) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            stats[12 * b + j] = kalman ? mean[kEvGyro][j] : nan;
            stats[12 * b + 3 + j] = kalman ? var[kEvAcc][j] / (double)(n_avg - 1) : nan;
            stats[12 * b + 6 + j] = kalman ? var[kEvMag][j] / (double)(n_avg - 1) : nan;
            stats[12 * b + 9 + j] = kalman ? var[kEvGyro][j] / (double)(n_avg - 1) : nan;
        }
    }
}

}  // namespace pekf

using namespace pekf;

extern "C" int pekf_frontend_init_dev(int64_t batch, int64_t n_events, const void *ev_planes, const int64_t *t_start,
                                      int n_avg, double *init, int64_t *t_init, double *stats, int32_t *ready,
                                      void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_events >= 0, "negative size");
    PEKF_CHECK_ARG(n_avg >= 2, "n_avg must be >= 2 (the variance divides by n_avg - 1)");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(ev_planes && t_start && init && t_init && ready, "null pointer");
    hipLaunchKernelGGL(k_frontend_init, dim3(grid_for(batch, kFeBlock)), dim3(kFeBlock), 0, as_stream(stream), batch,
                       n_events, static_cast<const float4 *>(ev_planes), t_start, n_avg, init, t_init, stats, ready);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_frontend_init");
    return PEKF_OK;
}

extern "C" int pekf_frontend_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                                 const int64_t *t_init, double alpha, int64_t r_max, void *plane_gd, void *plane_am, void *plane_my, int32_t *counts, double *refs,
                                 int *dev_error, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_events >= 0 && r_max >= 0, "negative size");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(ev_planes && init && t_init && plane_gd && plane_am && plane_my && counts && refs,
                   "null pointer");
    hipLaunchKernelGGL(k_frontend, dim3(grid_for(batch, kFeBlock)), dim3(kFeBlock), 0, as_stream(stream), batch,
                       n_events, static_cast<const float4 *>(ev_planes), init, t_init, alpha, r_max,
                       static_cast<float4 *>(plane_gd), static_cast<float4 *>(plane_am),
                       static_cast<float2 *>(plane_my), counts, refs, dev_error);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_frontend");
    return PEKF_OK;
}
