// pekf_phase3.hpp -- phase 3 of the live server's front-end for one filter on one
// lane: raw phone events in, the 40 B records the filter consumes out.  Shared by k_frontend
// (pekf_frontend.hip: records written to the stream planes) and k_live (pekf_live.hip: records fed
// straight into the filter on the same lane), so both produce the same records bit for bit.
//
// The event step is Parser::WriteKalmanFilterMeasurement (KFS/Parser.cpp:148-219); a record is
// ExecuteKalmanFilter (Parser.cpp:229-257): acc / mag interpolated to the gyro time (:259-267),
// normalised (:221-228), low-pass filtered (alpha, from a zero state: KalmanFilter.cpp:16-18,21-24,
// 279-303), dt = gyro time - the previous record's (KalmanFilter.cpp:306-308).  FP64 arithmetic (one
// reciprocal / rsqrt with a Newton step instead of IEEE divisions: ~1e-15 relative).  Records for the
// stream planes are rounded to f32 like every record of the stream (emit); k_live can take the low-pass
// outputs in FP64 instead (emit_lpf + lpf_acc / lpf_mag), as the server hands them to its filter.  The arithmetic is contracted as the compiler's default
// (fp contract fast) whatever the including file is compiled with: every function with arithmetic
// opens with that pragma, so k_live's records are k_frontend's.
//
// Two event forms (Phase3T<S>): f32 events (S = F3, 16 B: float4 {x, y, z, bits(gap << 2 | type)}) and
// FP64 events (S = V3, 32 B: double4 {x, y, z, bits(t) | type}, PEKF_EV_F64_EVENTS).  The server parses
// each sample from the phone's text with std::stod (Parser.cpp:23-25) -- the double nearest the
// decimal Float.toString printed (MessageSender.java:222-227), in general not the f32 itself -- so only
// the FP64 form carries the server's own input values; the state machine and the record arithmetic are
// the same code for both.
#pragma once

#include "pekf_internal.hpp"
#include "pekf_math.hpp"

namespace pekf {

enum : uint32_t { kEvAcc = 0, kEvGyro = 1, kEvMag = 2 };

// The clock step of a time event (word == PEKF_EV_TIME): an integer ns count held as a float64 whose low
// and high halves are the event's x and y bits.
__device__ __forceinline__ double time_step(const float4 v4) {
    return __hiloint2double(__float_as_int(v4.y), __float_as_int(v4.x));
}

// phase 2's result for a filter is usable (pekf_frontend_init_dev writes NaN for one that never got ready)
__device__ __forceinline__ bool init_is_finite(const double *init6) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 6; ++k) ok = ok && isfinite(init6[k]);
    return ok;
}

struct V3 {
    double x, y, z;
};
struct F3 {
    float x, y, z;
};
__device__ __forceinline__ V3 widen(const F3 &f) { return {f.x, f.y, f.z}; }
__device__ __forceinline__ V3 widen(const V3 &v) { return v; }
// component-wise c ? a : b (a struct-valued ?: would go through scratch memory)
__device__ __forceinline__ V3 sel(bool c, const V3 &a, const V3 &b) {
    return {c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}
__device__ __forceinline__ F3 sel(bool c, const F3 &a, const F3 &b) {
    return {c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z};
}

// Parser::NormalizeValues (:221-228) with one rsqrt instead of a sqrt and three divisions
__device__ __forceinline__ V3 normalised(const V3 &v) {
#pragma clang fp contract(fast)
    const double in = rsqrt<true>((v.x * v.x + v.y * v.y) + v.z * v.z);
    return {v.x * in, v.y * in, v.z * in};
}
// The same with the sum of squares fused explicitly, fma(z, z, fma(y, y, x x)): which product of a sum of
// products the compiler contracts depends on the code around it, and the FP64-event records of k_live and
// k_frontend must round identically (normalised keeps the f32 form's rounding as it was)
__device__ __forceinline__ V3 normalised_fma(const V3 &v) {
    const double in = rsqrt<true>(__builtin_fma(v.z, v.z, __builtin_fma(v.y, v.y, v.x * v.x)));
    return {v.x * in, v.y * in, v.z * in};
}

// A completed record's inputs, captured when the state machine completes it (its state moves on at
// once) and turned into the record by Phase3::emit: the gyro sample, acc_0 / acc_1 / mag_0 / mag_1
// (f32 samples; *_mean: acc_0 / mag_0 is still the phase-2 mean) and the time differences of
// LinearInterpolationSensor and of the record's dt.
template <typename S>
struct RawRecT {
    S gyro, acc0, acc1, mag0, mag1;
    bool acc0_mean, mag0_mean;
    double dt, an, ad, mn, md;  // dt, acc / mag lerp num and den
};
using RawRec = RawRecT<F3>;
// FP64 events: the record waits with its interpolations already formed, each scaled by |t2 - t1| (A, M:
// Phase3T::lerp_scaled), so a pending record is 10 doubles instead of 20 -- the registers that keep
// k_live's FP64-event form at two waves per SIMD -- and its emit needs no reciprocal.
template <>
struct RawRecT<V3> {
    V3 A, M, gyro;
    double dt;
};

// An FP64 event {x, y, z, w}: w's bits are those of the event's time in ns as a float64 (an integer of
// magnitude < 2^51, so its two lowest mantissa bits are zero) with the type in those two bits (3: a
// message no sensor takes).  Absolute times: any gap or clock step is just the next event's time.  No
// message at all (padding) is w = the bits of -0.0 with type 3, which no time packs to.
__device__ __forceinline__ uint32_t ev64_type(const double4 &e) {
    return (uint32_t)__double_as_longlong(e.w) & 3u;
}
__device__ __forceinline__ double ev64_time(const double4 &e) {
    return __longlong_as_double(__double_as_longlong(e.w) & ~3ll);
}
// no message (padding: moves nothing in either phase)
constexpr unsigned long long kEv64None = 0x8000000000000003ull;
__device__ __forceinline__ double4 ev64_null() { return make_double4(0.0, 0.0, 0.0, __longlong_as_double((long long)kEv64None)); }
__device__ __forceinline__ bool ev64_none(const double4 &e) {
    return (unsigned long long)__double_as_longlong(e.w) == kEv64None;
}

// The padding event of either form: f32 -- a zero-step time event {0, 0, 0, word 3}; FP64 -- ev64_null.
template <typename EvT>
__device__ __forceinline__ EvT null_event() {
    if constexpr (std::is_same<EvT, double4>::value)
        return ev64_null();
    else
        return make_float4(0.f, 0.f, 0.f, __uint_as_float(PEKF_EV_TIME));
}

// One event of a plane, non-temporal (NT: each event is read once per pass) or plain.
template <bool NT>
__device__ __forceinline__ float4 load_event(const float4 *q) {
    if constexpr (NT) {
        typedef float nv4 __attribute__((ext_vector_type(4)));
        const nv4 v = __builtin_nontemporal_load((const nv4 *)q);
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *q;
    }
}
template <bool NT>
__device__ __forceinline__ double4 load_event(const double4 *q) {
    if constexpr (NT) {
        typedef double nd2 __attribute__((ext_vector_type(2)));
        const nd2 lo = __builtin_nontemporal_load((const nd2 *)q), hi = __builtin_nontemporal_load((const nd2 *)q + 1);
        return make_double4(lo.x, lo.y, hi.x, hi.y);
    } else {
        return *q;
    }
}

// With f32 events (S = F3) the state machine moves samples as f32 (one select per component instead
// of two, no conversions per event); they are widened only when a record is emitted.  With FP64 events
// (S = V3) they are the server's doubles throughout.  acc_0 / mag_0 start as the phase-2 means (FP64,
// not samples): a flag says a slot still holds the mean.
template <typename S>
struct Phase3T {
    using Raw = RawRecT<S>;
    static constexpr bool kLean = std::is_same<S, V3>::value;  // FP64 events: the lean capture (RawRecT<V3>)
    // phase-2 state: acc_0 / mag_0 = raw means at the initialisation time (Parser.cpp:44-53)
    V3 mean_acc, mean_mag;
    S acc0, mag0;
    bool acc0_mean, mag0_mean;  // acc_0 / mag_0 is still the phase-2 mean
    double t_acc0, t_mag0, prev_t, t;  // t: the f32 events' running clock (FP64 events carry their time)
    // The latest acc / mag sample and its time.  The Parser's acc_1 / mag_1 is always the latest sample
    // while it is set (it is written by every sample after the gyro, and nothing else moves until the
    // record completes or the next gyro shifts it to acc_0 / mag_0), so it is not held separately: each
    // event updates the latest sample once and acc_0 / mag_0 copy it when the Parser would, 10 VALU
    // per event fewer than moving acc_1 / mag_1 and acc_0 / mag_0 through two selects each.
    S acc1, mag1;
    S gyro;
    double t_acc1, t_mag1, t_gyro;
    bool gyro_set, acc1_set, mag1_set;
    V3 lpf_acc, lpf_mag;
    double alpha, beta;

    // Emission is deferred: when a lane completes a record, only its inputs are captured (RawRec),
    // and the expensive part -- two interpolations with a reciprocal, two normalisations with an
    // rsqrt, the low-pass and the f32 packing (emit) -- runs for the whole wave later, not on every
    // event some lane completes one (which, with 64 lanes, is nearly every event).  The deferring
    // form of event() keeps one captured record in p (pend): a lane needs at least 3 events (gyro,
    // acc, mag) between two records, so when emit runs every 3 events it never has two pending.
    // Arithmetic is unchanged: the time differences are formed at capture, exactly as lerp_to would.
    bool pend;
    Raw p;
    const double *init;  // kLean: the phase-2 means are re-read from here in the (rare) capture that needs them

    __device__ __forceinline__ void start(const double *init6, int64_t t_start, double a) {
        init = init6;
        mean_acc = {init6[0], init6[1], init6[2]};
        mean_mag = {init6[3], init6[4], init6[5]};
        acc0 = mag0 = acc1 = mag1 = gyro = {0, 0, 0};
        acc0_mean = mag0_mean = true;
        t = t_acc0 = t_mag0 = prev_t = (double)t_start;
        lpf_acc = lpf_mag = {0, 0, 0};
        t_acc1 = t_mag1 = t_gyro = 0;
        gyro_set = acc1_set = mag1_set = false;
        alpha = a;
        beta = 1.0 - a;
        pend = false;
        if constexpr (kLean) {
            p.A = p.M = p.gyro = {0, 0, 0};
            p.dt = 0;
        } else {
            p.gyro = p.acc0 = p.mag0 = p.acc1 = p.mag1 = {0, 0, 0};
            p.acc0_mean = p.mag0_mean = true;
            p.dt = p.an = p.mn = 0;
            p.ad = p.md = 1;
        }
    }

    // kLean: Parser::LinearInterpolationSensor (:259-267), y1 + (y2 - y1) / (t2 - t1) * (t3 - t1), formed
    // times d = |t2 - t1| as (y2 - y1) * s + y1 * d with s = sign(t2 - t1) (t3 - t1) -- equal in real
    // arithmetic, and normalisation removes the positive scale d.  d = 0 gives NaN, as the reference's
    // division by zero does (every component inf or NaN, normalised to NaN).
    __device__ __forceinline__ static V3 lerp_scaled(const V3 &y1, const V3 &y2, double num, double den) {
#pragma clang fp contract(fast)
        const double d = fabs(den), sn = den < 0.0 ? -num : num;
        // explicit fmas: the contraction of a sum of two products is the compiler's choice, and k_live and
        // k_frontend must round their records identically
        V3 r = {__builtin_fma(y2.x - y1.x, sn, y1.x * d), __builtin_fma(y2.y - y1.y, sn, y1.y * d),
                __builtin_fma(y2.z - y1.z, sn, y1.z * d)};
        if (d == 0.0) r.x = __builtin_nan("");
        return r;
    }

    // the filter's reference vectors: the normalised phase-2 means (Parser.cpp:48-49); call after start
    __device__ __forceinline__ void refs(double (&r)[6]) const {
        const V3 a = normalised(mean_acc), m = normalised(mean_mag);
        r[0] = a.x; r[1] = a.y; r[2] = a.z;
        r[3] = m.x; r[4] = m.y; r[5] = m.z;
    }

    // One event {x, y, z, bits(word)}: the word carries the type and the ns gap to the previous event.
    // Parser::WriteKalmanFilterMeasurement (Parser.cpp:148-219), branch-free: each state variable is
    // one select, so nothing is copied between divergent paths (step).
    // on_done(const Raw &) runs for a lane whose event completes a record.
    // TE: the stream may hold time events (word == PEKF_EV_TIME: no sample, the clock moves by the
    // float64 in the x / y bits -- a pause of 2^30 ns or more, or a clock stepping back); without TE
    // such an event moves nothing.  Either way type 3 matches no sensor, so the state machine skips it.
    template <bool TE = false, typename F>
    __device__ __forceinline__ void event(const float4 v4, F &&on_done) {
#pragma clang fp contract(fast)
        const uint32_t word = __float_as_uint(v4.w);
        const uint32_t ty = word & 3u;
        if constexpr (TE)
            t += word == PEKF_EV_TIME ? time_step(v4) : (double)(word >> 2);
        else
            t += (double)(word >> 2);
        step(S{v4.x, v4.y, v4.z}, ty, t, on_done);
    }
    // One FP64 event {x, y, z, bits(t) | type} (PEKF_EV_F64_EVENTS): the sample is the server's double.
    template <typename F>
    __device__ __forceinline__ void event64(const double4 &e, F &&on_done) {
        step(S{e.x, e.y, e.z}, ev64_type(e), ev64_time(e), on_done);
    }

    // The state machine for a sample v of type ty at time tn:
    //   before a gyro sample: acc -> acc_0, mag -> mag_0, gyro -> gyro (gyro_is_set);
    //   after it: acc -> acc_1, mag -> mag_1 (set); a new gyro replaces the gyro and shifts a set
    //   acc_1 -> acc_0 / mag_1 -> mag_0, clearing both flags.
    template <typename F>
    __device__ __forceinline__ void step(const S &v, const uint32_t ty, const double tn, F &&on_done) {
        const bool isA = ty == kEvAcc, isM = ty == kEvMag, isG = ty == kEvGyro;
        const bool gs = gyro_set;
        const bool wA1 = isA && gs, wM1 = isM && gs;
        // acc1 / mag1: the latest sample (equal to the Parser's acc_1 / mag_1 whenever that is set)
        if constexpr (kLean) {
            // FP64 samples: a masked 64-bit move per double (a branch) instead of two selects
            if (isA) {
                asm volatile("");
                acc1 = v;
                t_acc1 = tn;
            }
            if (isM) {
                asm volatile("");
                mag1 = v;
                t_mag1 = tn;
            }
        } else {
            acc1 = sel(isA, v, acc1);
            t_acc1 = isA ? tn : t_acc1;
            mag1 = sel(isM, v, mag1);
            t_mag1 = isM ? tn : t_mag1;
        }
        const bool a1s = wA1 || (acc1_set && !(isG && gs)), m1s = wM1 || (mag1_set && !(isG && gs));
        const bool sA = isG && gs && acc1_set, sM = isG && gs && mag1_set;  // gyro shift
        // ExecuteKalmanFilter (Parser.cpp:229-257) once acc_1 and mag_1 are both set: record its
        // inputs, then acc_0 <- acc_1, mag_0 <- mag_1, flags cleared
        const bool done = a1s && m1s;
        if (done) {
            asm volatile("");  // keeps this a branch: masked 64-bit moves, not two selects per double
            Raw r;
            r.gyro = gyro; r.dt = t_gyro - prev_t;
            if constexpr (kLean) {
                V3 a0 = acc0, m0 = mag0;
                // acc_0 / mag_0 can still be the phase-2 means only up to a lane's first record
                if (__builtin_expect(__any(acc0_mean || mag0_mean), 0)) {
                    a0 = sel(acc0_mean, V3{init[0], init[1], init[2]}, a0);
                    m0 = sel(mag0_mean, V3{init[3], init[4], init[5]}, m0);
                }
                r.A = lerp_scaled(a0, acc1, t_gyro - t_acc0, t_acc1 - t_acc0);
                r.M = lerp_scaled(m0, mag1, t_gyro - t_mag0, t_mag1 - t_mag0);
            } else {
                r.acc0 = acc0; r.acc0_mean = acc0_mean; r.acc1 = acc1; r.an = t_gyro - t_acc0; r.ad = t_acc1 - t_acc0;
                r.mag0 = mag0; r.mag0_mean = mag0_mean; r.mag1 = mag1; r.mn = t_gyro - t_mag0; r.md = t_mag1 - t_mag0;
            }
            on_done(r);
            prev_t = t_gyro;
        }
        // acc_0 <- the sample before any gyro (then acc1 = v), or acc_1 on a shift or after a record
        const bool cA = (isA && !gs) || sA || done, cM = (isM && !gs) || sM || done;
        if constexpr (kLean) {
            if (cA) {
                asm volatile("");
                acc0 = acc1;
                t_acc0 = t_acc1;
            }
            if (cM) {
                asm volatile("");
                mag0 = mag1;
                t_mag0 = t_mag1;
            }
            if (isG) {
                asm volatile("");
                gyro = v;
                t_gyro = tn;
            }
            acc0_mean = acc0_mean && !cA;
            mag0_mean = mag0_mean && !cM;
        } else {
            acc0 = sel(cA, acc1, acc0);
            acc0_mean = acc0_mean && !cA;
            t_acc0 = cA ? t_acc1 : t_acc0;
            mag0 = sel(cM, mag1, mag0);
            mag0_mean = mag0_mean && !cM;
            t_mag0 = cM ? t_mag1 : t_mag0;
            gyro = sel(isG, v, gyro);
            t_gyro = isG ? tn : t_gyro;
        }
        gyro_set = (gs || isG) && !done;
        acc1_set = a1s && !done;
        mag1_set = m1s && !done;
    }

    // the deferring form: the completed record's inputs wait in p (pend) for emit(esc)
    template <bool TE = false>
    __device__ __forceinline__ void event(const float4 v4) {
        event<TE>(v4, [&](const Raw &r) {
            pend = true;
            p = r;
        });
    }
    __device__ __forceinline__ void event64(const double4 &e) {
        event64(e, [&](const Raw &r) {
            pend = true;
            p = r;
        });
    }
    // the pending record; its dt stays in p.dt (the float64 an escaped record needs)
    __device__ __forceinline__ Rec emit(bool &esc) {
        pend = false;
        return emit(p, esc);
    }
    // the same with the low-pass outputs left in FP64 (lpf_acc / lpf_mag)
    __device__ __forceinline__ float4 emit_lpf(bool &esc) {
        pend = false;
        return emit_lpf(p, esc);
    }

    // The low-pass step l <- alpha x + beta l (KalmanFilter.cpp:285,298), rounded as fma(beta, l, alpha x)
    // -- the contraction the compiler chose for the expression -- but written into l's own register: the
    // compiler's accumulating v_fmac form left the result in the product's register and copied it back
    // (6 moves per emit).
    __device__ __forceinline__ void lpf_step(double &l, double x) const {
        const double ax = alpha * x;
        asm("v_fma_f64 %0, %1, %0, %2" : "+v"(l) : "v"(beta), "v"(ax));
    }

    // A captured record, in the order they complete: interpolation, normalisation, low-pass (the FP64
    // results stay in lpf_acc / lpf_mag).
    __device__ __forceinline__ void lpf_record(const Raw &q) {
#pragma clang fp contract(fast)
        // Parser::LinearInterpolationSensor (:259-267): (y2 - y1) / (t2 - t1) * (t3 - t1) + y1, the
        // division taken as one reciprocal.  Timestamps are integer ns held in doubles (exact below
        // 2^53), so t3 - t1 and t2 - t1 are the exact differences (double)t3 - (double)t1 gives.
        const double fa = q.an * recip<true>(q.ad), fm = q.mn * recip<true>(q.md);
        V3 a0 = widen(q.acc0), m0 = widen(q.mag0);
        const V3 a1 = widen(q.acc1), m1 = widen(q.mag1);
        // acc_0 / mag_0 can still be the phase-2 mean only up to a lane's first record, so the wave
        // selects it behind a wave-uniform test that is false for all but its first few emits
        if (__builtin_expect(__any(q.acc0_mean || q.mag0_mean), 0)) {
            a0 = sel(q.acc0_mean, mean_acc, a0);
            m0 = sel(q.mag0_mean, mean_mag, m0);
        }
        const V3 a = normalised({(a1.x - a0.x) * fa + a0.x, (a1.y - a0.y) * fa + a0.y, (a1.z - a0.z) * fa + a0.z});
        const V3 m = normalised({(m1.x - m0.x) * fm + m0.x, (m1.y - m0.y) * fm + m0.y, (m1.z - m0.z) * fm + m0.z});
        lpf_step(lpf_mag.x, m.x); lpf_step(lpf_mag.y, m.y); lpf_step(lpf_mag.z, m.z);
        lpf_step(lpf_acc.x, a.x); lpf_step(lpf_acc.y, a.y); lpf_step(lpf_acc.z, a.z);
    }

    // lpf_record, and the gyro / dt half of the 40 B record, which is returned (f32 events).
    // esc: its dt does not fit the dt word (not in [0, 2^31 - 1) ns): the word is PEKF_DT_ESCAPE and
    // the caller keeps q.dt beside the record (pekf.h).
    __device__ __forceinline__ float4 emit_lpf(const Raw &q, bool &esc) {
        lpf_record(q);
        esc = !(q.dt >= 0.0 && q.dt < (double)PEKF_DT_ESCAPE);
        return make_float4((float)q.gyro.x, (float)q.gyro.y, (float)q.gyro.z,
                           __uint_as_float(esc ? PEKF_DT_ESCAPE : (uint32_t)q.dt));
    }

    // lpf_record, and the record's gyro and dt in FP64 (FP64 events: {gx, gy, gz, dt_ns}, the GD half of
    // an 80 B record; the dt is any float64, so nothing is escaped).
    __device__ __forceinline__ double4 emit64(const Raw &q) {
        static_assert(kLean, "FP64 records come from FP64 events");
        // the captured interpolations normalised (their scale d drops out), then the low-pass
        const V3 a = normalised_fma(q.A), m = normalised_fma(q.M);
        lpf_step(lpf_mag.x, m.x); lpf_step(lpf_mag.y, m.y); lpf_step(lpf_mag.z, m.z);
        lpf_step(lpf_acc.x, a.x); lpf_step(lpf_acc.y, a.y); lpf_step(lpf_acc.z, a.z);
        return make_double4(q.gyro.x, q.gyro.y, q.gyro.z, q.dt);
    }
    __device__ __forceinline__ double4 emit64() {
        pend = false;
        return emit64(p);
    }

    // The 40 B stream record (acc / mag rounded to f32, as every record of the stream planes).
    __device__ __forceinline__ Rec emit(const Raw &q, bool &esc) {
        Rec r;
        r.gd = emit_lpf(q, esc);
        r.am = make_float4((float)lpf_acc.x, (float)lpf_acc.y, (float)lpf_acc.z, (float)lpf_mag.x);
        r.my = make_float2((float)lpf_mag.y, (float)lpf_mag.z);
        return r;
    }
};
using Phase3 = Phase3T<F3>;    // f32 events
using Phase3_64 = Phase3T<V3>; // FP64 events (the server's stod values)

}  // namespace pekf
