// pekf_live.hip -- the live server's whole per-event loop on the device in one pass (SURVEY.md §8f-2:
// the front-end fused into the filter kernel): raw phone events -> phase-3 records (pekf_phase3.hpp,
// Parser::WriteKalmanFilterMeasurement / ExecuteKalmanFilter, KFS/Parser.cpp:148-267) -> Prediction +
// Correction of each record (pekf_step.hpp, ExtendedKalmanFilter.py:58-80 as main_file.py:42-45 calls
// them).  One lane per filter holds its front-end state, X and covariance in registers; records never
// touch memory.  A record's acc / mag stay the FP64 low-pass outputs (the server's filter input,
// KFS/KalmanFilter.cpp:279-303) in a 5-deep queue (20 KB per wave); PEKF_EV_F32_RECORDS rounds them to
// the f32 stream record in a 6-deep queue instead (18 KB) and then equals the split pipeline bit for
// bit.  FP64 costs +1.5-1.8 % at 1M filters x 1,024 events (same-box ABBA, profiles/r5/live_q5/): the
// shallower queue runs more filter steps with fewer lanes busy.  The split pipeline -- pekf_frontend_dev writing records to the stream planes, then
// pekf_run_dev with counts reading them back -- pays a 40 B record write that scatters into 96 B of
// sectors (each lane's record count drifts, so a wave's stores land in 64 different rows) plus the
// 40 B read; here the only HBM traffic is the 16 B event.
//
// Lanes complete records at different events (a record needs a gyro, an acc and a mag sample after the
// previous one: every ~10 events on the synthetic streams, never closer than 3), but a filter step is
// ~300 FP64 instructions that the wave executes for every lane at once.  Running it whenever some lane
// has a record would run it at nearly every emit with a few lanes active, so each lane queues its
// records (kQueue deep) and the wave runs one filter step -- the oldest queued record of every lane
// that has one -- at the end of a block of kRing events when at least kQuorum lanes have a record
// queued, or when some lane's queue could overflow within the next block, and until empty after the
// last event (scripts/live_queue_sim.py: 0.79 of the lanes busy per step at 3 / 6 / 56 against 0.28
// when every block drains).  Per lane the records apply in order with the same arithmetic as
// pekf_run_dev's multi-record kernel (reference basis, N, omod), so the final state equals the split
// pipeline's bit for bit (with f32 records; with FP64 ones, within FP64 rounding of the unrounded chain).
#include "pekf_phase3.hpp"
#include "pekf_step.hpp"

namespace pekf {

// Tuned on the box (scripts/ab_live.sh, profiles/r2/live/): the kernel is register-bound -- front-end
// state, filter state and a filter step's temporaries -- so the record queue lives in LDS and the
// launch is held to 2 waves per SIMD (252 registers) with a 3-event ring: 5.5 ms at 1M filters x
// 1,024 events, against 8.7 ms for 6 events and the queue in registers at 1 wave/SIMD.  Queueing the
// records' raw inputs instead (emit moved into the filter step, 104 B per slot, 3 deep) was slower:
// 5.9 ms (profiles/r2/live/variants/raw_queue.log).
#ifndef PEKF_LIVE_RING
#define PEKF_LIVE_RING 3  // event rows in flight per lane; a filter step may run after each block of them
#endif
#ifndef PEKF_LIVE_RING64
#define PEKF_LIVE_RING64 3  // the same for FP64 events (32 B each)
#endif
#ifndef PEKF_LIVE_NTL
#define PEKF_LIVE_NTL 1  // non-temporal event loads: each event is read once (-1.4 %, profiles/r4/ntload/)
#endif
#ifndef PEKF_LIVE_QUEUE
#define PEKF_LIVE_QUEUE 6  // records a lane can hold (48 B of LDS each: the 40 B record + its escaped dt)
#endif
#ifndef PEKF_LIVE_QUEUE64
#define PEKF_LIVE_QUEUE64 5  // the same with FP64 acc / mag (64 B each): 20 KB of LDS per wave, all of it
#endif
#ifndef PEKF_LIVE_QUEUE_EV64
#define PEKF_LIVE_QUEUE_EV64 4  // FP64 events: all-FP64 records (80 B each), 20 KB of LDS per wave
#endif
#ifndef PEKF_LIVE_QUORUM
#define PEKF_LIVE_QUORUM 56  // lanes of 64 with a queued record that trigger a filter step
#endif
#ifndef PEKF_LIVE_EV64_WAVES
#define PEKF_LIVE_EV64_WAVES 2
#endif

// A lane's records waiting for the wave's next filter step, oldest first: a ring of Q slots per lane in
// LDS, [slot][lane] so that a wave's accesses fall in distinct banks whatever slot each lane is at.  A
// push or pop is a few address operations and three LDS accesses.  (Held in registers -- slots as
// separate variables, a push selecting its slot -- the queue cost 40 selects per push and registers
// the kernel does not have: profiles/r2/live/variants/live_ab*.log.)
// A record whose dt does not fit its dt word (PEKF_DT_ESCAPE, a pause of 2^31 ns or more) keeps its
// float64 dt in the slot's side entry dt[slot][lane], written and read only for such a record.
template <int Q>
struct LdsQueue {
    static constexpr size_t kBytes = (sizeof(float4) * 2 + sizeof(float2) + sizeof(double)) * Q * kRunBlock;
    float4 (*gd)[kRunBlock];
    float4 (*am)[kRunBlock];
    float2 (*my)[kRunBlock];
    double (*dt)[kRunBlock];
    int head = 0, n = 0;
    __device__ __forceinline__ void bind(unsigned char *lds) {
        gd = reinterpret_cast<float4(*)[kRunBlock]>(lds);
        am = reinterpret_cast<float4(*)[kRunBlock]>(lds + sizeof(float4) * Q * kRunBlock);
        dt = reinterpret_cast<double(*)[kRunBlock]>(lds + 2 * sizeof(float4) * Q * kRunBlock);
        my = reinterpret_cast<float2(*)[kRunBlock]>(lds + (2 * sizeof(float4) + sizeof(double)) * Q * kRunBlock);
    }
    __device__ __forceinline__ int tail() const { return head + n < Q ? head + n : head + n - Q; }
    __device__ __forceinline__ bool esc_queued() const { return false; }  // escaped dts live in the dt plane
    __device__ __forceinline__ void push(const Rec &r, bool esc, double dtv) {
        const int slot = tail();
        gd[slot][threadIdx.x] = r.gd;
        am[slot][threadIdx.x] = r.am;
        my[slot][threadIdx.x] = r.my;
        if (esc) dt[slot][threadIdx.x] = dtv;
        ++n;
    }
    using Slot = Rec;
    // the oldest record and its dt in ns
    __device__ __forceinline__ Slot pop(double &dtv) {
        const Rec r = {gd[head][threadIdx.x], am[head][threadIdx.x], my[head][threadIdx.x]};
        const uint32_t word = __float_as_uint(r.gd.w) & PEKF_DT_MASK;
        dtv = (double)word;
        if (word == PEKF_DT_ESCAPE) dtv = dt[head][threadIdx.x];
        if (n > 0) {
            head = head + 1 < Q ? head + 1 : 0;
            --n;
        }
        return r;
    }
    static __device__ __forceinline__ void unpack(const Slot &r, double (&gy)[3], double (&acc)[3], double (&mag)[3]) {
        gy[0] = r.gd.x; gy[1] = r.gd.y; gy[2] = r.gd.z;
        acc[0] = r.am.x; acc[1] = r.am.y; acc[2] = r.am.z;
        mag[0] = r.am.w; mag[1] = r.my.x; mag[2] = r.my.y;
    }
    // the popped record's acc / mag again (it stays in its slot, the one before head, until a later push)
    __device__ __forceinline__ void reload(double *a, double *m) const {
        const int slot = head == 0 ? Q - 1 : head - 1;
        const float4 va = am[slot][threadIdx.x];
        const float2 vm = my[slot][threadIdx.x];
        a[0] = va.x; a[1] = va.y; a[2] = va.z;
        m[0] = va.w; m[1] = vm.x; m[2] = vm.y;
    }
};

// The queue with FP64 acc / mag: what the server's filter receives (KFS/KalmanFilter.cpp:279-303 hands
// the double low-pass outputs to Prediction / Correction), not the f32 stream record.  Per slot the
// gyro / dt word (16 B) and acc and mag as three double2 planes (48 B): 5 slots x 64 B x 64 lanes is
// 20 KB per wave, exactly the CU's 160 KB at 2 waves per SIMD, so there is no room for an escaped-dt
// plane.  A record whose dt does not fit the dt word keeps its float64 dt in a register instead
// (esc_dt), one per lane: k_live steps a wave while any lane still has such a record queued, so a lane
// never holds two (escapes are pauses of 2.1 s or more: rare, and cheap to drain for).
template <int Q>
struct LdsQueue64 {
    static constexpr size_t kBytes = (sizeof(float4) + 3 * sizeof(double2)) * Q * kRunBlock;
    float4 (*gd)[kRunBlock];
    double2 (*am)[3][kRunBlock];  // {acc.x, acc.y}, {acc.z, mag.x}, {mag.y, mag.z}
    double esc_dt = __builtin_nan("");  // the queued escaped record's dt (NaN: none queued)
    int head = 0, n = 0;
    __device__ __forceinline__ void bind(unsigned char *lds) {
        am = reinterpret_cast<double2(*)[3][kRunBlock]>(lds);
        gd = reinterpret_cast<float4(*)[kRunBlock]>(lds + 3 * sizeof(double2) * Q * kRunBlock);
    }
    // a lane has an escaped record queued (k_live then steps until it is applied)
    __device__ __forceinline__ bool esc_queued() const { return esc_dt == esc_dt; }
    __device__ __forceinline__ void push(const float4 &g, const V3 &a, const V3 &m, bool esc, double dtv) {
        const int slot = head + n < Q ? head + n : head + n - Q;
        gd[slot][threadIdx.x] = g;
        am[slot][0][threadIdx.x] = make_double2(a.x, a.y);
        am[slot][1][threadIdx.x] = make_double2(a.z, m.x);
        am[slot][2][threadIdx.x] = make_double2(m.y, m.z);
        if (esc) esc_dt = dtv;
        ++n;
    }
    struct Slot {
        float4 gd;
        double2 v[3];
    };
    __device__ __forceinline__ Slot pop(double &dtv) {
        const Slot r = {gd[head][threadIdx.x], {am[head][0][threadIdx.x], am[head][1][threadIdx.x], am[head][2][threadIdx.x]}};
        const uint32_t word = __float_as_uint(r.gd.w) & PEKF_DT_MASK;
        dtv = (double)word;
        if (n > 0 && word == PEKF_DT_ESCAPE) {
            dtv = esc_dt;
            esc_dt = __builtin_nan("");
        }
        if (n > 0) {
            head = head + 1 < Q ? head + 1 : 0;
            --n;
        }
        return r;
    }
    static __device__ __forceinline__ void unpack(const Slot &r, double (&gy)[3], double (&acc)[3], double (&mag)[3]) {
        gy[0] = r.gd.x; gy[1] = r.gd.y; gy[2] = r.gd.z;
        acc[0] = r.v[0].x; acc[1] = r.v[0].y; acc[2] = r.v[1].x;
        mag[0] = r.v[1].y; mag[1] = r.v[2].x; mag[2] = r.v[2].y;
    }
    __device__ __forceinline__ void reload(double *a, double *m) const {
        const int slot = head == 0 ? Q - 1 : head - 1;
        const double2 v0 = am[slot][0][threadIdx.x], v1 = am[slot][1][threadIdx.x], v2 = am[slot][2][threadIdx.x];
        a[0] = v0.x; a[1] = v0.y; a[2] = v1.x;
        m[0] = v1.y; m[1] = v2.x; m[2] = v2.y;
    }
};

// The queue of FP64-event launches: every field of the record in FP64 -- gyro and dt too, as the server's
// filter gets them (dt any float64, so no escape) -- 80 B per slot as five double2 planes [slot][lane]
// (16 B per lane and plane: conflict-free ds_*_b128), 4 deep = 20 KB per wave, the CU's 160 KB at 2
// waves per SIMD.
template <int Q>
struct LdsQueueF64 {
    static constexpr size_t kBytes = 5 * sizeof(double2) * Q * kRunBlock;
    double2 (*v)[5][kRunBlock];  // {gx, gy}, {gz, dt}, {ax, ay}, {az, mx}, {my, mz}
    int head = 0, n = 0;
    __device__ __forceinline__ void bind(unsigned char *lds) { v = reinterpret_cast<double2(*)[5][kRunBlock]>(lds); }
    __device__ __forceinline__ bool esc_queued() const { return false; }
    __device__ __forceinline__ void push(const double4 &g, const V3 &a, const V3 &m) {
        const int slot = head + n < Q ? head + n : head + n - Q;
        v[slot][0][threadIdx.x] = make_double2(g.x, g.y);
        v[slot][1][threadIdx.x] = make_double2(g.z, g.w);
        v[slot][2][threadIdx.x] = make_double2(a.x, a.y);
        v[slot][3][threadIdx.x] = make_double2(a.z, m.x);
        v[slot][4][threadIdx.x] = make_double2(m.y, m.z);
        ++n;
    }
    struct Slot {
        double2 v[5];
    };
    __device__ __forceinline__ Slot pop(double &dtv) {
        Slot r;
#pragma unroll
        for (int k = 0; k < 5; ++k) r.v[k] = v[head][k][threadIdx.x];
        dtv = r.v[1].y;
        if (n > 0) {
            head = head + 1 < Q ? head + 1 : 0;
            --n;
        }
        return r;
    }
    static __device__ __forceinline__ void unpack(const Slot &r, double (&gy)[3], double (&acc)[3], double (&mag)[3]) {
        gy[0] = r.v[0].x; gy[1] = r.v[0].y; gy[2] = r.v[1].x;
        acc[0] = r.v[2].x; acc[1] = r.v[2].y; acc[2] = r.v[3].x;
        mag[0] = r.v[3].y; mag[1] = r.v[4].x; mag[2] = r.v[4].y;
    }
    __device__ __forceinline__ void reload(double *a, double *m) const {
        const int slot = head == 0 ? Q - 1 : head - 1;
        const double2 v2 = v[slot][2][threadIdx.x], v3 = v[slot][3][threadIdx.x], v4 = v[slot][4][threadIdx.x];
        a[0] = v2.x; a[1] = v2.y; a[2] = v3.x;
        m[0] = v3.y; m[1] = v4.x; m[2] = v4.y;
    }
};

// TE: the event planes may hold time events (Phase3::event).  R64: records keep their FP64 acc / mag
// (LdsQueue64); otherwise they are the f32 stream records pekf_frontend_dev writes (LdsQueue).
// EV64: FP64 events (PEKF_EV_F64_EVENTS, double4 planes: the server's own sample values), records all
// FP64 (LdsQueueF64); TE and R64 do not apply.
template <bool TE, bool R64, bool EV64 = false>
__global__ __launch_bounds__(kRunBlock) __attribute__((amdgpu_waves_per_eu(EV64 ? PEKF_LIVE_EV64_WAVES : 2))) void k_live(
    int64_t batch, int64_t n_events, const std::conditional_t<EV64, double4, float4> *__restrict__ ev,
    const double *__restrict__ init, const int64_t *__restrict__ t_init, double alpha, double qs, double rs,
    double *__restrict__ Xio, double *__restrict__ Pio, int32_t *__restrict__ counts, double *__restrict__ refs) {
    using EvT = std::conditional_t<EV64, double4, float4>;
    constexpr int kRing = EV64 ? PEKF_LIVE_RING64 : PEKF_LIVE_RING, kFlush = 3, kQuorum = PEKF_LIVE_QUORUM;
    constexpr int kQueue = EV64 ? PEKF_LIVE_QUEUE_EV64 : R64 ? PEKF_LIVE_QUEUE64 : PEKF_LIVE_QUEUE;
    constexpr int kPush = kRing / kFlush;  // records a lane can complete within one block
    static_assert(kRing % kFlush == 0, "the ring depth must be a multiple of the emit period");
    static_assert(kQueue >= kPush, "the queue must hold a block's records");
    static_assert(!(EV64 && (TE || R64)), "FP64 events take their own record queue and carry their times");
    // LdsQueue64 keeps ONE escaped dt per lane (esc_dt) and want_step drains it before the next block,
    // which is safe only while a block completes at most one record per lane
    static_assert(!R64 || kPush == 1, "LdsQueue64's single escaped-dt register needs one record per lane per block");
    const int64_t b = (int64_t)blockIdx.x * kRunBlock + threadIdx.x;
    if (b >= batch) return;

    Phase3T<std::conditional_t<EV64, V3, F3>> fe;
    fe.start(init + 6 * b, t_init[b], alpha);
    // a filter that never finished phase 2 (non-finite init: pekf_frontend_init_dev's "not ready")
    // applies no record: its state is left as it was and counts[b] = 0
    const bool ready = init_is_finite(init + 6 * b);
    double rf[6];
    fe.refs(rf);
#pragma unroll
    for (int k = 0; k < 6; ++k) refs[6 * b + k] = rf[k];

    // the filter in its reference frame's basis, covariance as N (pekf_step.hpp), as k_run does it
    Frame Wf;
    make_frame<true>(rf, rf + 3, Wf);
    double x[4];
    Sym4T<double> P;
    load_state<false>(Xio, Pio, b, batch, x, P);
    RefWLazy Wr;
    Wr.aW = Wf.alpha; Wr.b1W = Wf.beta1; Wr.b2W = Wf.beta2;
    Wr.pair = refs + 6 * b;
    {
        double qw[4];
        frame_quat(Wf, qw);
        to_ref_basis(qw, x, P, rs);
    }
    const StepK<double> kc = step_consts<double, true>(qs, rs);

    using Queue = std::conditional_t<EV64, LdsQueueF64<kQueue>,
                                     std::conditional_t<R64, LdsQueue64<kQueue>, LdsQueue<kQueue>>>;
    __shared__ __attribute__((aligned(16))) unsigned char q_lds[Queue::kBytes];
    Queue queue;
    queue.bind(q_lds);
    int32_t applied = 0;
    // One filter step for every lane with a queued record: its oldest, Prediction + Correction with
    // the multi-record kernel's arithmetic (the first record of the launch from the loaded |X|^2,
    // every later one lazy; front-end records always carry a magnetometer sample).
    auto filter_step = [&]() {
        const bool has = queue.n > 0;
        double dt;
        const typename Queue::Slot cur = queue.pop(dt);
        auto reload = [&](double *a, double *m) { queue.reload(a, m); };  // rare: the degenerate-Wahba fallback
        OmodMode mode;
        mode.enter();
        if (has) {
            double gy[3], acc[3], mag[3];
            Queue::unpack(cur, gy, acc, mag);
            if (applied == 0)
                ekf_record_step<double, true, false, true>(x, state_norm2(x), P, Wr, kc, gy, dt, false, acc, mag,
                                                           reload);
            else
                ekf_record_step<double, true, true, true>(x, 1.0, P, Wr, kc, gy, dt, false, acc, mag, reload);
            ++applied;
        }
        mode.leave();
    };
    // the pending record (captured by Phase3::event) into the queue
    auto push_pending = [&](const auto &q) {
        bool esc;
        if constexpr (EV64) {
            const double4 g = fe.emit64(q);
            if (ready) queue.push(g, fe.lpf_acc, fe.lpf_mag);
        } else if constexpr (R64) {
            const float4 g = fe.emit_lpf(q, esc);
            if (ready) queue.push(g, fe.lpf_acc, fe.lpf_mag, esc, q.dt);
        } else {
            const Rec rc = fe.emit(q, esc);
            if (ready) queue.push(rc, esc, q.dt);
        }
    };
    auto on_event = [&](const EvT &v4) {
        if constexpr (EV64)
            fe.event64(v4);
        else
            fe.template event<TE>(v4);
    };
    auto flush = [&]() {
        if (fe.pend) {
            fe.pend = false;
            push_pending(fe.p);
        }
    };

    // Events stream through a register ring of kRing rows loaded kRing events ahead (the loop is
    // unrolled by kRing so every ring index is static; rows past the end are clamped to the last one).
    // 32-bit event counters (n_events < 2^30, checked on the host): the wave-uniform bounds tests are
    // then scalar compares, where 64-bit ones took a VALU move and compare each, twice per event.
    const uint32_t lane = (uint32_t)b;
    const int32_t n_ev = (int32_t)n_events;
    auto load = [&](int32_t e) -> EvT {
        const int32_t row = e < n_ev ? e : n_ev - 1;
#if PEKF_LIVE_NTL
        if constexpr (EV64) {
            typedef double nd2 __attribute__((ext_vector_type(2)));
            const nd2 *q = (const nd2 *)(ev + (int64_t)row * batch + lane);
            const nd2 lo = __builtin_nontemporal_load(q), hi = __builtin_nontemporal_load(q + 1);
            return make_double4(lo.x, lo.y, hi.x, hi.y);
        } else {
            typedef float nv4 __attribute__((ext_vector_type(4)));
            const nv4 v = __builtin_nontemporal_load((const nv4 *)(ev + (int64_t)row * batch + lane));
            return make_float4(v.x, v.y, v.z, v.w);
        }
#else
        return (ev + (int64_t)row * batch)[lane];
#endif
    };
    // wave-uniform: a step while some lane could overflow in the next block, then one more if a quorum
    // of lanes has a record; after the last event until every queue is empty; (R64) while some lane
    // still has an escaped record queued, so the next block cannot queue a second one on that lane
    auto want_step = [&](bool last) {
        const uint64_t queued = __ballot(queue.n > 0);
        return queued != 0 && (last || __any(queue.n > kQueue - kPush) || __popcll(queued) >= kQuorum ||
                               (R64 && !EV64 && __any(queue.esc_queued())));
    };
    auto steps = [&](bool last) {
        // tested before the loop, so a block that runs no step does not pass the loop's header
        if (want_step(last)) {
            do {
                filter_step();
            } while (want_step(last));
        }
    };
    if (n_ev > 0) {
        EvT ring[kRing];
#pragma unroll
        for (int k = 0; k < kRing; ++k) ring[k] = load(k);
        // No exit inside the unrolled body (one per event made the compiler copy the ring on the back
        // edge, behind a wait for the loads just issued): the last, partial block is padded with null
        // events -- a zero-step time event {0, 0, 0, word 3} moves no state, with or without TE -- so
        // every block runs whole, and nothing is pending after a whole block.
        for (int32_t e0 = 0; e0 < n_ev; e0 += kRing) {
            if (e0 + kRing > n_ev) {  // uniform, once per launch
#pragma unroll
                for (int k = 0; k < kRing; ++k)
                    if (e0 + k >= n_ev) {
                        if constexpr (EV64)
                            ring[k] = ev64_null();
                        else
                            ring[k] = make_float4(0.f, 0.f, 0.f, __uint_as_float(PEKF_EV_TIME));
                    }
            }
#pragma unroll
            for (int k = 0; k < kRing; ++k) {
                const EvT v4 = ring[k];
                ring[k] = load(e0 + k + kRing);
                on_event(v4);
                if ((k + 1) % kFlush == 0) flush();
            }
            steps(e0 + kRing >= n_ev);
        }
    }
    counts[b] = applied;
    if (applied == 0) return;  // no record: the state is left as it was (as pekf_run_dev with counts)
    from_ref_basis(Wr, x, P, rs);
    store_state<false>(Xio, Pio, b, batch, x, P);
}

}  // namespace pekf

using namespace pekf;

extern "C" int pekf_live_ext_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                                 const int64_t *t_init, double alpha, double *X, double *P, double q, double r,
                                 int32_t *counts, double *refs, uint32_t flags, int *dev_error, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_events >= 0, "negative size");
    PEKF_CHECK_ARG((flags & ~(PEKF_EV_TIME_EVENTS | PEKF_EV_F32_RECORDS | PEKF_EV_F64_EVENTS)) == 0, "unknown flags");
    const bool ev64 = (flags & PEKF_EV_F64_EVENTS) != 0;
    PEKF_CHECK_ARG(!ev64 || (flags & (PEKF_EV_TIME_EVENTS | PEKF_EV_F32_RECORDS)) == 0,
                   "PEKF_EV_F64_EVENTS takes no other flag (FP64 events carry their times; their records are FP64)");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(n_events < ((int64_t)1 << 30), "n_events must be < 2^30 per launch");
    PEKF_CHECK_ARG(ev_planes && init && t_init && X && P && counts && refs, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)ev_planes % 16 == 0, "misaligned event planes");
    PEKF_CHECK_ARG(r > 0.0, "r must be > 0 (S = P- + rI must be SPD)");
    (void)dev_error;  // every record's dt is applied (escaped ones from the queue's side entries)
    const auto *ev = static_cast<const float4 *>(ev_planes);
    const dim3 grid(grid_for(batch, kRunBlock)), block(kRunBlock);
    const bool te = (flags & PEKF_EV_TIME_EVENTS) != 0, r64 = (flags & PEKF_EV_F32_RECORDS) == 0;
    auto launch = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, grid, block, 0, as_stream(stream), batch, n_events, ev, init, t_init, alpha, q, r, X,
                           P, counts, refs);
    };
    if (ev64)
        hipLaunchKernelGGL((k_live<false, false, true>), grid, block, 0, as_stream(stream), batch, n_events,
                           static_cast<const double4 *>(ev_planes), init, t_init, alpha, q, r, X, P, counts, refs);
    else if (te)
        r64 ? launch(k_live<true, true>) : launch(k_live<true, false>);
    else
        r64 ? launch(k_live<false, true>) : launch(k_live<false, false>);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_live");
    return PEKF_OK;
}

extern "C" int pekf_live_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                             const int64_t *t_init, double alpha, double *X, double *P, double q, double r,
                             int32_t *counts, double *refs, int *dev_error, void *stream) {
    return pekf_live_ext_dev(batch, n_events, ev_planes, init, t_init, alpha, X, P, q, r, counts, refs, 0u, dev_error,
                             stream);
}
