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
#include "pekf_phase3.hpp"

namespace pekf {

constexpr int kFeBlock = 256;
// Non-temporal event loads (every event is read once per pass): k_frontend -1.7 %, phase 2's means
// -5 % (profiles/r4/ntload/).
#ifndef PEKF_FE_NTL
#define PEKF_FE_NTL 1
#endif
#ifndef PEKF_INIT_NTL
#define PEKF_INIT_NTL 1
#endif

// k_frontend's record queue: per group of kFeGroup lanes (one 128 B line of a gd / am row), a pool of
// kFePool LDS record slots and the ring of its free slot numbers.  A lane's record for a row in [base,
// base + kFeRows) of its group takes a free slot; the group writes row `base` as whole lines once every
// ready lane of the group has made it (round 5, profiles/r5/frontend_pool/: WRITE_SIZE 1.25x the record
// bytes, against 1.59x for 10 rows per lane and 2.6x storing each record where it is made; 56-78 slots
// and 16 / 32 rows swept).  64 slots x 8 groups + the tables = 23 KB per wave, 7 waves per CU, sized
// for gfx950's 160 KB of LDS (the library is built for gfx950 only).  The per-lane-row and wave-wide
// forms it replaced are in git history (round 5) and measured in profiles/r4/frontend_stage/.
constexpr int kFeGroup = 8;
constexpr int kFePool = 64;
constexpr int kFeRows = 32;
// FP64 events write 80 B FP64 records: PEKF_FE_POOL64 slots per group (32 = 20 KB per wave, the f32
// form's LDS footprint and waves per CU)
#ifndef PEKF_FE_POOL64
#define PEKF_FE_POOL64 32
#endif

// The pooled queue's LDS (one wave per block, so no barrier: a wave's LDS accesses complete in
// order): per group, P record slots and the ring of its free slot numbers; per lane, the slot of its
// record for each row base .. base + ROWS - 1 (row % ROWS).  R: the record (Rec, or Rec64 for FP64
// events), its three planes held as three arrays.
template <int P, int NG, int ROWS, typename R>
struct FePool {
    static_assert(P <= 255, "slot numbers are bytes");
    decltype(R::gd) gd[NG][P];
    decltype(R::am) am[NG][P];
    decltype(R::my) my[NG][P];
    uint8_t ring[NG][P];
    uint8_t slot[ROWS][64];
};
#ifndef PEKF_FE_RING
#define PEKF_FE_RING 9
#endif
#ifndef PEKF_FE_RING64
#define PEKF_FE_RING64 3  // FP64 events: 32 B each, so fewer in flight (registers)
#endif

// TE: the event planes may hold time events (Phase3::event).  dtx (may be null): the window's dt side
// plane [r_max][batch]; an escaped record's float64 dt goes there (err bit 4), else err bit 1.
//
// One wave per block.  Lanes' record rows drift apart (a wave's lanes span ~20 rows, p90 7.5 from its
// median, scripts/record_drift.py), so a record stored where it is made writes 16 / 16 / 8 B into its
// own row, and about one 32 B sector per store leaves L2 (profiles/r4/frontend_occ/).  Here each group
// keeps its records for rows [base, base + kFeRows) in its pool (the group's lanes that queue in one
// flush take consecutive entries of the free ring, in lane order); a record outside that range, or met
// by an empty pool, is stored directly.  Row base is written by every lane of the group holding it once
// all of the group's ready lanes have made it; its slots go back to the ring; the queue drains after
// the last event.  The records and their rows are unchanged; only the order of the stores differs.
//
// EV64: FP64 events (double4 planes, PEKF_EV_F64_EVENTS) -> FP64 records (Rec64: the planes of
// pekf_run_rec64_dev), every field FP64 and the dt any float64 (nothing escaped; dtx unused).
template <bool TE, bool EV64 = false>
__global__ __launch_bounds__(64) void k_frontend(int64_t batch, int64_t n_events,
                                                 const std::conditional_t<EV64, double4, float4> *__restrict__ ev,
                                                 const double *__restrict__ init, const int64_t *__restrict__ t_init,
                                                 double alpha, int64_t r_max,
                                                 decltype(std::conditional_t<EV64, Rec64, Rec>::gd) *__restrict__ gd,
                                                 decltype(std::conditional_t<EV64, Rec64, Rec>::am) *__restrict__ am,
                                                 decltype(std::conditional_t<EV64, Rec64, Rec>::my) *__restrict__ my,
                                                 double *__restrict__ dtx, int32_t *__restrict__ counts,
                                                 double *__restrict__ refs, int *__restrict__ err) {
    using EvT = std::conditional_t<EV64, double4, float4>;
    using RecT = std::conditional_t<EV64, Rec64, Rec>;
    const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (b >= batch) return;
    Phase3T<std::conditional_t<EV64, V3, F3>> fe;
    fe.start(init + 6 * b, t_init[b], alpha);
    const bool ready = init_is_finite(init + 6 * b);  // not ready (phase 2 unfinished): no records
    {
        double rf[6];
        fe.refs(rf);
#pragma unroll
        for (int k = 0; k < 6; ++k) refs[6 * b + k] = rf[k];
    }
    int32_t r = 0;  // this filter's records so far (r_max < 2^31, checked on the host)
    const int32_t rmax = (int32_t)r_max;
    int bad = 0;
    constexpr int POOL = EV64 ? PEKF_FE_POOL64 : kFePool, kG = kFeGroup, kRows = kFeRows;
    static_assert(kRows > 0 && kRows <= 32 && (kRows & (kRows - 1)) == 0, "a power-of-two row span of at most 32");
    __shared__ FePool<POOL, 64 / kG, kRows, RecT> st;
    const int col = threadIdx.x & 63;
    // the oldest row the group's queue holds (the same in each group of kG lanes)
    int32_t base = 0;
    uint32_t held = 0;  // bit row % kRows = this lane's record for that row is queued
    // this lane's group's bits of a wave ballot
    const int shift = col & ~(kG - 1);
    constexpr uint64_t kMask = (1ull << kG) - 1;
    const int grp = col / kG;                       // the group's pool
    const uint64_t below = (1ull << (col & (kG - 1))) - 1;  // the group's lanes before this one
    int head = 0, nfree = POOL;                     // the free ring's first entry and length (group-uniform)
    {  // the ring holds every slot; a group cut short by the batch's end has fewer lanes
        const uint64_t act = (__ballot(true) >> shift) & kMask;
        const int na = __popcll(act);
        for (int i = __popcll(act & below); i < POOL; i += na) st.ring[grp][i] = (uint8_t)i;
    }
    // the pending record (Phase3::pend) is emitted every kFlush events; a lane never has two
    constexpr int kFlush = 3;
    // flush with every lane active (the group's queueing lanes are ranked by a ballot)
    auto flush_pool = [&]() {
        const bool has = fe.pend;
        bool esc = false;
        RecT rc{};
        if (has) {
            if constexpr (EV64) {
                rc.gd = fe.emit64();
                rc.am = make_double4(fe.lpf_acc.x, fe.lpf_acc.y, fe.lpf_acc.z, fe.lpf_mag.x);
                rc.my = make_double2(fe.lpf_mag.y, fe.lpf_mag.z);
            } else {
                rc = fe.emit(esc);
            }
        }
        const bool live = has && ready;
        if (live && esc) bad |= dtx ? 4 : 1;
        const bool in = live && r < rmax;
        if (live && !in) bad |= 2;  // more records than the output window holds
        const bool want = in && r >= base && r < base + kRows;
        const uint64_t req = (__ballot(want) >> shift) & kMask;
        const int j = __popcll(req & below), k = __popcll(req);
        const int64_t o = (int64_t)r * batch + b;
        if (want && j < nfree) {
            int i = head + j;
            if (i >= POOL) i -= POOL;
            const int s = st.ring[grp][i];
            st.gd[grp][s] = rc.gd;
            st.am[grp][s] = rc.am;
            st.my[grp][s] = rc.my;
            const uint32_t sl = (uint32_t)r % kRows;
            st.slot[sl][col] = (uint8_t)s;
            held |= 1u << sl;
        } else if (in) {
            gd[o] = rc.gd;
            am[o] = rc.am;
            my[o] = rc.my;
        }
        if (!EV64 && in && esc && dtx) dtx[o] = fe.p.dt;
        const int t = k < nfree ? k : nfree;
        head += t;
        if (head >= POOL) head -= POOL;
        nfree -= t;
        if (live) ++r;
    };
    // write out row base while every ready lane of the group has made it (or, all, until no lane holds
    // any); its slots go back to the free ring
    auto drain_pool = [&](bool all) {
        for (;;) {
            bool go = ((__ballot(held != 0) >> shift) & kMask) != 0;
            if (!all) {
                const uint64_t behind = (__ballot(ready && r <= base && r < rmax) >> shift) & kMask;
                go = go && behind == 0;
            }
            if (!__any(go)) break;
            const uint32_t sl = (uint32_t)base % kRows;
            const bool mine = go && (held & (1u << sl));
            const uint64_t fm = (__ballot(mine) >> shift) & kMask;
            if (mine) {
                const int s = st.slot[sl][col];
                const int64_t o = (int64_t)base * batch + b;
                gd[o] = st.gd[grp][s];
                am[o] = st.am[grp][s];
                my[o] = st.my[grp][s];
                int i = head + nfree + __popcll(fm & below);
                if (i >= POOL) i -= POOL;
                st.ring[grp][i] = (uint8_t)s;
                held &= ~(1u << sl);
            }
            if (go) {
                nfree += __popcll(fm);
                ++base;
            }
        }
    };

    // Events stream through a register ring of kRing records loaded kRing events ahead (the loop is
    // unrolled by kRing so every ring index is static; the row is clamped to the last event, so the
    // loads past the end read a valid row and need no predicate).  32-bit event counters (n_events <
    // 2^30, checked on the host) keep the uniform tests scalar, and the last block is padded with null
    // events (a zero-step time event moves no state) so no exit sits inside the unrolled body; nothing
    // is pending after a whole block.
    const uint32_t lane = (uint32_t)b;
    const int32_t n_ev = (int32_t)n_events;
    auto load = [&](int32_t e) -> EvT {
        const int32_t row = e < n_ev ? e : n_ev - 1;
        return load_event<PEKF_FE_NTL>(ev + (int64_t)row * batch + lane);
    };
    if (n_ev > 0) {
        constexpr int kRing = EV64 ? PEKF_FE_RING64 : PEKF_FE_RING;  // events in flight per lane (a multiple of kFlush)
        static_assert(kRing % kFlush == 0, "the ring depth must be a multiple of the flush period");
        EvT ring[kRing];
#pragma unroll
        for (int k = 0; k < kRing; ++k) ring[k] = load(k);
        for (int32_t e0 = 0; e0 < n_ev; e0 += kRing) {
            if (e0 + kRing > n_ev) {  // uniform, once per launch
#pragma unroll
                for (int k = 0; k < kRing; ++k)
                    if (e0 + k >= n_ev) ring[k] = null_event<EvT>();
            }
#pragma unroll
            for (int k = 0; k < kRing; ++k) {
                const EvT v4 = ring[k];
                ring[k] = load(e0 + k + kRing);
                if constexpr (EV64)
                    fe.event64(v4);
                else
                    fe.template event<TE>(v4);
                if ((k + 1) % kFlush == 0) {
                    flush_pool();
                    drain_pool(false);
                }
            }
        }
    }
    drain_pool(true);
    counts[b] = r < rmax ? r : rmax;
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
// Every message counts, whatever its sensor type: one no sensor takes (type 3) adds no sample but, once
// all three are initialised, builds the filter or moves its time as any other (Parser.cpp:36-62).
// EV64: FP64 events (the server's stod doubles are what it averages, Parser.cpp:23-25,84-140); their
// times are absolute, and the no-message event (padding, ev64_none) is skipped.
template <bool EV64 = false>
__global__ __launch_bounds__(kFeBlock) void k_frontend_init(int64_t batch, int64_t n_events,
                                                            const std::conditional_t<EV64, double4, float4> *__restrict__ ev,
                                                            const int64_t *__restrict__ t_start, int n_avg,
                                                            double *__restrict__ init, int64_t *__restrict__ t_init,
                                                            double *__restrict__ stats, int32_t *__restrict__ ready) {
    using EvT = std::conditional_t<EV64, double4, float4>;
    const int64_t b = (int64_t)blockIdx.x * kFeBlock + threadIdx.x;
    if (b >= batch) return;
    const uint32_t lane = (uint32_t)b;
    double sum[3][3] = {};  // [type][xyz]
    int cnt[3] = {0, 0, 0};
    bool done[3] = {false, false, false};  // Acc_ / Gyr_ / Mag_initialized
    bool kalman = false;
    int64_t t = t_start[b], t_last = t;
    // events come kInitRing rows at a time, all loads issued before the first is used (the loop body
    // is a few adds, so without it each wave would wait out one memory latency per event).  32-bit
    // event counters (n_events < 2^30, checked on the host) keep the uniform bounds tests scalar; the
    // rows past the end of the last block are null events (a zero-step time event, which phase 2 skips
    // in both passes), so no exit sits inside the unrolled body.
    constexpr int kInitRing = 8;
    const int32_t n_ev = (int32_t)n_events;
    const EvT null_ev = null_event<EvT>();
    auto row = [&](int32_t e) -> EvT {
        return load_event<PEKF_INIT_NTL>(ev + (int64_t)(e < n_ev ? e : n_ev - 1) * batch + lane);
    };
    auto pad = [&](int32_t e0, EvT (&r)[kInitRing]) {
        if (e0 + kInitRing > n_ev) {  // uniform: the last block only
#pragma unroll
            for (int k = 0; k < kInitRing; ++k)
                if (e0 + k >= n_ev) r[k] = null_ev;
        }
    };
    for (int32_t e0 = 0; e0 < n_ev; e0 += kInitRing) {
        EvT r[kInitRing];
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) r[k] = row(e0 + k);
        pad(e0, r);
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) {
            const EvT v4 = r[k];
            int ty;
            if constexpr (EV64) {
                if (ev64_none(v4)) continue;  // no message
                ty = (int)ev64_type(v4);
                t = (int64_t)ev64_time(v4);
            } else {
                const uint32_t word = __float_as_uint(v4.w);
                ty = (int)(word & 3u);
                if (word == PEKF_EV_TIME) {  // a time event: the clock moves, nothing else happens
                    t += (int64_t)time_step(v4);
                    continue;
                }
                t += (int64_t)(word >> 2);
            }
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
    // second pass: the variance of the first n_avg samples of each type, in their order -- only when
    // it is asked for (stats; pekf_live's session path takes the means alone)
    double var[3][3] = {};
    int c2[3] = {0, 0, 0};
    for (int32_t e0 = 0; stats && e0 < n_ev; e0 += kInitRing) {
        // done once every type has its n_avg; a filter that never got ready reports NaN, so reads none
        if (!kalman || (c2[0] >= n_avg && c2[1] >= n_avg && c2[2] >= n_avg)) break;
        EvT r[kInitRing];
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) r[k] = row(e0 + k);
        pad(e0, r);
#pragma unroll
        for (int k = 0; k < kInitRing; ++k) {
            const EvT v4 = r[k];
            int ty;
            if constexpr (EV64)
                ty = (int)ev64_type(v4);
            else
                ty = (int)(__float_as_uint(v4.w) & 3u);
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

extern "C" int pekf_frontend_init_ext_dev(int64_t batch, int64_t n_events, const void *ev_planes,
                                          const int64_t *t_start, int n_avg, double *init, int64_t *t_init,
                                          double *stats, int32_t *ready, uint32_t flags, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_events >= 0, "negative size");
    PEKF_CHECK_ARG(n_avg >= 2, "n_avg must be >= 2 (the variance divides by n_avg - 1)");
    PEKF_CHECK_ARG(n_events < ((int64_t)1 << 30), "n_events must be < 2^30 per launch");
    PEKF_CHECK_ARG((flags & ~(PEKF_EV_TIME_EVENTS | PEKF_EV_F64_EVENTS)) == 0, "unknown flags");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(ev_planes && t_start && init && t_init && ready, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)ev_planes % 16 == 0, "misaligned event planes");
    const dim3 grid(grid_for(batch, kFeBlock)), block(kFeBlock);
    if (flags & PEKF_EV_F64_EVENTS)
        hipLaunchKernelGGL(k_frontend_init<true>, grid, block, 0, as_stream(stream), batch, n_events,
                           static_cast<const double4 *>(ev_planes), t_start, n_avg, init, t_init, stats, ready);
    else  // phase 2 always honours time events
        hipLaunchKernelGGL(k_frontend_init<false>, grid, block, 0, as_stream(stream), batch, n_events,
                           static_cast<const float4 *>(ev_planes), t_start, n_avg, init, t_init, stats, ready);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_frontend_init");
    return PEKF_OK;
}

extern "C" int pekf_frontend_init_dev(int64_t batch, int64_t n_events, const void *ev_planes, const int64_t *t_start,
                                      int n_avg, double *init, int64_t *t_init, double *stats, int32_t *ready,
                                      void *stream) {
    return pekf_frontend_init_ext_dev(batch, n_events, ev_planes, t_start, n_avg, init, t_init, stats, ready, 0u,
                                      stream);
}

extern "C" int pekf_frontend_ext_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                                     const int64_t *t_init, double alpha, int64_t r_max, void *plane_gd,
                                     void *plane_am, void *plane_my, double *dt_ext, int32_t *counts, double *refs,
                                     uint32_t flags, int *dev_error, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_events >= 0 && r_max >= 0, "negative size");
    PEKF_CHECK_ARG((flags & ~(PEKF_EV_TIME_EVENTS | PEKF_EV_F64_EVENTS)) == 0, "unknown flags");
    const bool ev64 = (flags & PEKF_EV_F64_EVENTS) != 0;
    PEKF_CHECK_ARG(!ev64 || ((flags & PEKF_EV_TIME_EVENTS) == 0 && !dt_ext),
                   "FP64 events carry their times and write FP64 records (no time events, no dt side plane)");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(n_events < ((int64_t)1 << 30), "n_events must be < 2^30 per launch");
    PEKF_CHECK_ARG(r_max < ((int64_t)1 << 31), "r_max must be < 2^31");
    PEKF_CHECK_ARG(ev_planes && init && t_init && plane_gd && plane_am && plane_my && counts && refs,
                   "null pointer");
    PEKF_CHECK_ARG((uintptr_t)ev_planes % 16 == 0 && (uintptr_t)plane_gd % 16 == 0 && (uintptr_t)plane_am % 16 == 0 &&
                       (uintptr_t)plane_my % 8 == 0,
                   "misaligned planes");
    const dim3 grid(grid_for(batch, 64)), block(64);
    if (ev64)
        hipLaunchKernelGGL((k_frontend<false, true>), grid, block, 0, as_stream(stream), batch, n_events,
                           static_cast<const double4 *>(ev_planes), init, t_init, alpha, r_max,
                           static_cast<double4 *>(plane_gd), static_cast<double4 *>(plane_am),
                           static_cast<double2 *>(plane_my), nullptr, counts, refs, dev_error);
    else if (flags & PEKF_EV_TIME_EVENTS)
        hipLaunchKernelGGL(k_frontend<true>, grid, block, 0, as_stream(stream), batch, n_events,
                           static_cast<const float4 *>(ev_planes), init, t_init, alpha, r_max,
                           static_cast<float4 *>(plane_gd), static_cast<float4 *>(plane_am),
                           static_cast<float2 *>(plane_my), dt_ext, counts, refs, dev_error);
    else
        hipLaunchKernelGGL(k_frontend<false>, grid, block, 0, as_stream(stream), batch, n_events,
                           static_cast<const float4 *>(ev_planes), init, t_init, alpha, r_max,
                           static_cast<float4 *>(plane_gd), static_cast<float4 *>(plane_am),
                           static_cast<float2 *>(plane_my), dt_ext, counts, refs, dev_error);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_frontend");
    return PEKF_OK;
}

extern "C" int pekf_frontend_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                                 const int64_t *t_init, double alpha, int64_t r_max, void *plane_gd, void *plane_am,
                                 void *plane_my, int32_t *counts, double *refs, int *dev_error, void *stream) {
    return pekf_frontend_ext_dev(batch, n_events, ev_planes, init, t_init, alpha, r_max, plane_gd, plane_am, plane_my,
                                 nullptr, counts, refs, 0u, dev_error, stream);
}
