// pekf_wire_dev.hip -- the phone -> server wire on the device (the step before phase 2
// and phase 3): the clients' 100-byte text frames in, the FP64 event planes of pekf_frontend_init_ext_dev /
// pekf_live_ext_dev out, with no host parse between the socket and the filter.
//
// Each message the Android client sends is one 100-byte frame: "#<phase>,<type>:<x>,<y>,<z>,t:<ns>" padded
// with spaces to 99 characters plus println's newline (ASC/MessageSender.java:217-233); the server reads
// exactly such frames (recv of messageSize = 100, KFS/Server.cpp:35,84), keeps those that start with '#'
// (Parser::run, KFS/Parser.cpp:357-363) and parses them in ProcessString (:12-26): phase = the first
// character, Type = the first character before the first ':', each value std::stod of the text before the
// next ',', the time std::stoll of the text after "t:".  One lane per phone walks its frames in order
// ([n_frames][batch][100] bytes: a wave's 64 frames of one index are 6,400 contiguous bytes, staged
// through LDS with coalesced dword loads, the next index's in flight while this one is parsed), and
// appends each phase-2 / phase-3 message to that phase's plane as the FP64 event {x, y, z, bits(t) |
// type} (type 3 for a Type no sensor takes); the rows after a phone's last message get the no-message
// event.
//
// The values are std::stod's -- strtod's correctly rounded double of the decimal -- bit for bit: a
// decimal of at most 19 significant digits m and exponent e with m <= 2^53 and |e| <= 22 is one IEEE
// multiply or divide of two exact doubles (the case of every sensor reading); any other m < 2^64 with
// |e| <= 80 (Float.toString's extremes: 1.4E-45, 3.4028235E38) takes an exact big-integer path;
// "NaN", "Infinity" and "-Infinity" are Float.toString's non-finite forms.  A frame in any other form
// (a number strtod would read but the client never prints: blanks, hex, more than 19 digits; or text
// std::stod / std::stoll would throw on) is not parsed here: the phone's first such frame is reported
// (bad_frame, *dev_error bit 1) and pekf_wire_parse on the host takes it.
#include "pekf_internal.hpp"
#include "pekf_phase3.hpp"

namespace pekf {

constexpr int kWireFrame = 100;  // bytes per message, as sent and as received
constexpr int kWireBlock = 64;   // one wave per block: 6,400 B of frames in LDS
constexpr int kWireDwords = kWireFrame * kWireBlock / 4;  // 1,600

__constant__ double kWirePow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// ---- exact decimal -> double for the cases one IEEE operation cannot do (rare: off the common path) ----
// Unsigned big integers as 12 little-endian 32-bit limbs (384 bits: m < 2^64 times 10^80 < 2^266 fits).
constexpr int kLimbs = 12;

__device__ void big_mul10(uint32_t (&a)[kLimbs]) {
    uint64_t carry = 0;
    for (int i = 0; i < kLimbs; ++i) {
        const uint64_t v = (uint64_t)a[i] * 10u + carry;
        a[i] = (uint32_t)v;
        carry = v >> 32;
    }
}
__device__ int big_bitlen(const uint32_t (&a)[kLimbs]) {
    for (int i = kLimbs - 1; i >= 0; --i)
        if (a[i]) return 32 * i + 32 - __clz(a[i]);
    return 0;
}
__device__ bool big_bit(const uint32_t (&a)[kLimbs], int b) { return b >= 0 && ((a[b >> 5] >> (b & 31)) & 1u); }
__device__ void big_shl(uint32_t (&a)[kLimbs], int s) {  // a <<= s (0 <= s, result < 2^384)
    const int w = s >> 5, r = s & 31;
    for (int i = kLimbs - 1; i >= 0; --i) {
        const uint32_t hi = i - w >= 0 ? a[i - w] : 0u, lo = i - w - 1 >= 0 ? a[i - w - 1] : 0u;
        a[i] = r ? (hi << r) | (lo >> (32 - r)) : hi;
    }
}
__device__ bool big_ge(const uint32_t (&a)[kLimbs], const uint32_t (&b)[kLimbs]) {
    for (int i = kLimbs - 1; i >= 0; --i)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}
__device__ void big_sub(uint32_t (&a)[kLimbs], const uint32_t (&b)[kLimbs]) {  // a -= b (a >= b)
    uint64_t borrow = 0;
    for (int i = 0; i < kLimbs; ++i) {
        const uint64_t v = (uint64_t)a[i] - b[i] - borrow;
        a[i] = (uint32_t)v;
        borrow = (v >> 63) & 1u;
    }
}
// q (of 54..64 bits) times 2^e2, rounded to 53 bits to nearest-even with `sticky` for the bits below q
__device__ double round_scaled(uint64_t q, bool sticky, int e2) {
    const int s = 64 - __clzll(q) - 53;
    uint64_t qm = q >> s;
    const uint64_t rem = q & ((1ull << s) - 1), half = 1ull << (s - 1);
    if (rem > half || (rem == half && (sticky || (qm & 1u)))) {
        if (++qm == (1ull << 53)) return ldexp((double)(qm >> 1), e2 + s + 1);
    }
    return ldexp((double)qm, e2 + s);
}
// m * 10^e10 correctly rounded (m > 0, |e10| <= 80): the value strtod gives the decimal
__device__ double decimal_exact(uint64_t m, int e10) {
    uint32_t n[kLimbs] = {(uint32_t)m, (uint32_t)(m >> 32)};
    if (e10 >= 0) {
        for (int i = 0; i < e10; ++i) big_mul10(n);
        const int L = big_bitlen(n);
        if (L <= 64) {
            const uint64_t v = ((uint64_t)n[1] << 32) | n[0];
            return L <= 53 ? (double)v : round_scaled(v, false, 0);
        }
        // the top 64 bits and a sticky bit for the rest
        const int s = L - 64;
        uint64_t q = 0;
        for (int b = 63; b >= 0; --b) q |= (uint64_t)big_bit(n, s + b) << b;
        bool sticky = false;
        for (int b = 0; b < s; ++b) sticky |= big_bit(n, b);
        return round_scaled(q, sticky, s);
    }
    uint32_t d[kLimbs] = {1u};
    for (int i = 0; i < -e10; ++i) big_mul10(d);
    // scale so that q = floor(n / d) has 55 or 56 bits: n * 2^k (k >= 0) or d * 2^-k
    const int k = big_bitlen(d) - big_bitlen(n) + 55;
    if (k >= 0)
        big_shl(n, k);
    else
        big_shl(d, -k);
    uint64_t q = 0;
    for (int i = 55; i >= 0; --i) {  // restoring division, one quotient bit per step
        uint32_t t[kLimbs];
        for (int j = 0; j < kLimbs; ++j) t[j] = d[j];
        big_shl(t, i);
        if (big_ge(n, t)) {
            big_sub(n, t);
            q |= 1ull << i;
        }
    }
    bool sticky = false;
    for (int j = 0; j < kLimbs; ++j) sticky |= n[j] != 0;
    return round_scaled(q, sticky, -k);
}

// ---- one frame ----
// A number token at fr[i..], up to the ',' that must follow it: Float.toString's forms (and plain
// decimals).  Returns false for any other form; i is left on the ','.
__device__ bool wire_number(const uint8_t *fr, int &i, double &out) {
    auto ch = [&](int j) -> unsigned {  // past the frame: none (the address clamped into it)
        const unsigned c = fr[j < kWireFrame ? j : kWireFrame - 1];
        return j < kWireFrame ? c : 0u;
    };
    bool neg = false;
    if (ch(i) == '-' || ch(i) == '+') neg = ch(i++) == '-';
    if (ch(i) == 'N' || ch(i) == 'I') {  // "NaN" (strtod: the positive quiet NaN), "[-]Infinity"
        const bool nan = ch(i) == 'N';
        const char *w = nan ? "NaN," : "Infinity,";
        if (nan && neg) return false;
        int j = 0;
        for (; w[j]; ++j)
            if (ch(i + j) != (uint8_t)w[j]) return false;
        i += j - 1;
        out = nan ? __longlong_as_double(0x7ff8000000000000ll) : (neg ? -__builtin_huge_val() : __builtin_huge_val());
        return true;
    }
    // the digits and one '.': a loop whose body has no branch (the lanes of a wave run it together);
    // leading zeros are not significant digits; more than 19 of them is not the client's form (m wraps
    // then, and the token is refused below)
    uint64_t m = 0;
    int nd = 0, nf = 0;
    bool any = false, frac = false, act = true;
    for (;;) {  // until no lane of the wave is in its digits: the exit is wave-uniform, not per lane
        const unsigned c = ch(i), d = c - '0';
        const bool dig = d < 10u, pt = c == '.' && !frac;
        act = act && (dig || pt);
        if (!__any(act)) break;
        const bool sig = act && dig && (m != 0 || d != 0);
        m = sig ? m * 10 + d : m;
        nd += sig;
        nf += act && dig && frac;
        any |= act && dig;
        frac |= act && pt;
        i += act;
    }
    if (!any || nd > 19) return false;
    int e10 = -nf;
    if (ch(i) == 'e' || ch(i) == 'E') {
        ++i;
        bool eneg = false;
        if (ch(i) == '+' || ch(i) == '-') eneg = ch(i++) == '-';
        unsigned e = 0;  // (wraps past 9 digits: refused below)
        int ne = 0;
        bool eact = true;
        for (;;) {
            const unsigned d = ch(i) - '0';
            eact = eact && d < 10u;
            if (!__any(eact)) break;
            e = eact ? e * 10 + d : e;
            ne += eact;
            i += eact;
        }
        if (ne == 0 || ne > 4) return false;
        e10 += eneg ? -(int)e : (int)e;
    }
    if (ch(i) != ',') return false;
    double v;
    if (m == 0) {
        v = 0.0;  // any exponent: strtod's zero
    } else if (m <= (1ull << 53) && e10 >= -22 && e10 <= 22) {
        v = e10 < 0 ? (double)m / kWirePow10[-e10] : (double)m * kWirePow10[e10];
    } else if (e10 >= -80 && e10 <= 80) {
        v = decimal_exact(m, e10);
    } else {
        return false;
    }
    out = neg ? -v : v;
    return true;
}

struct WireMsg {
    uint8_t phase, type;  // characters
    double v[3];
    long long t;
};

// 0: a message (m filled); 1: no message (no '#': Parser::run skips it); 2: not parsed here (see above)
__device__ int wire_frame(const uint8_t *fr, WireMsg &m) {
    auto ch = [&](int j) -> unsigned {
        const unsigned c = fr[j < kWireFrame ? j : kWireFrame - 1];
        return j < kWireFrame ? c : 0u;
    };
    if (fr[0] != '#') return 1;
    m.phase = fr[1];
    int i = 3;  // str.substr(2) of the text after '#'
    bool cact = true, nul = false;
    for (;;) {  // to the first ':' (a NUL before it: strchr's end, not the server's message)
        const unsigned c = ch(i);
        nul |= cact && c == 0 && i < kWireFrame;
        cact = cact && i < kWireFrame && c != ':' && c != 0;
        if (!__any(cact)) break;
        i += cact;
    }
    if (nul || i >= kWireFrame) return 2;
    m.type = i > 3 ? fr[3] : 0;  // FindValues(str, ":")[0]
    ++i;
    for (int k = 0; k < 3; ++k) {
        if (!wire_number(fr, i, m.v[k])) return 2;
        ++i;  // past the ','
    }
    if (ch(i) != 't' || ch(i + 1) != ':') return 2;
    i += 2;
    const bool neg = ch(i) == '-';
    if (neg) ++i;
    uint64_t t = 0;
    int nd = 0;
    bool tact = true;
    for (;;) {
        const unsigned d = ch(i) - '0';
        tact = tact && d < 10u;
        if (!__any(tact)) break;
        t = tact ? t * 10 + d : t;  // (wraps past 19 digits: refused below)
        nd += tact;
        i += tact;
    }
    if (!nd || nd > 19 || t > (neg ? (1ull << 63) : (1ull << 63) - 1)) return 2;  // std::stoll: ERANGE throws
    m.t = neg ? (long long)(0 - t) : (long long)t;
    return 0;
}

// Held to 3 waves per SIMD (168 VGPRs, 4 of them spilled on the rare big-integer path; the compiler's
// choice was 201 = 2 waves): the parse is a chain of dependent LDS reads and divergent branches, and the
// third wave hides part of it.  262,144 phones x 1,024 frames, same box (profiles/r6/wire_dev/): 29.8 ms
// (byte loops with early exits, 2 waves) -> 27.5 (branch-free digit loops) -> 25.4 ms (and 3 waves) ->
// 23.6 ms (the character loops exit when no lane of the wave is still in them, __any, instead of lane by
// lane).  Measured and not kept: a dword-window reader instead of byte reads (36.6 against 29.8 ms), and
// every check of a token as a status flag instead of an exit (35.2 against 23.7 ms: the division and the
// big-integer path then run for every lane, and the registers spill).
__global__ __launch_bounds__(kWireBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_wire_events(
    int64_t batch, int64_t n_frames, const uint32_t *__restrict__ frames, int64_t e2_max, int64_t e3_max,
    double4 *__restrict__ ev2, double4 *__restrict__ ev3, int64_t *__restrict__ first_t2, int32_t *__restrict__ n2,
    int32_t *__restrict__ n3, int32_t *__restrict__ bad_frame, int *__restrict__ err) {
    __shared__ uint32_t lds[kWireDwords];
    const int lane = threadIdx.x;
    const int64_t k0 = (int64_t)blockIdx.x * kWireBlock;
    const int64_t b = k0 + lane;
    const int nk = batch - k0 < kWireBlock ? (int)(batch - k0) : kWireBlock;  // phones in this block
    const int nd = nk * (kWireFrame / 4);  // dwords of one frame index
    // dword j of frame index f of this block's phones (frames of one index are contiguous across phones)
    auto load = [&](int64_t f, uint32_t (&r)[kWireDwords / kWireBlock]) {
        const uint32_t *src = frames + (f * batch + k0) * (kWireFrame / 4);
#pragma unroll
        for (int c = 0; c < kWireDwords / kWireBlock; ++c) {
            const int j = c * kWireBlock + lane;
            r[c] = j < nd ? __builtin_nontemporal_load(src + j) : 0u;
        }
    };
    const uint8_t *fr = reinterpret_cast<const uint8_t *>(lds) + lane * kWireFrame;
    int32_t c2 = 0, c3 = 0, bad = -1;
    int64_t t2 = 0;
    const double4 none = ev64_null();
    uint32_t cur[kWireDwords / kWireBlock];
    if (n_frames > 0) load(0, cur);
    for (int64_t f = 0; f < n_frames; ++f) {
        __syncthreads();  // the previous index's frames are parsed
#pragma unroll
        for (int c = 0; c < kWireDwords / kWireBlock; ++c) lds[c * kWireBlock + lane] = cur[c];
        __syncthreads();
        if (f + 1 < n_frames) load(f + 1, cur);  // in flight while this index is parsed
        if (b >= batch || bad >= 0) continue;
        WireMsg m;
        const int st = wire_frame(fr, m);
        if (st == 2) {
            bad = (int32_t)f;
            continue;
        }
        if (st != 0 || (m.phase != '2' && m.phase != '3')) continue;  // phase 1 (calibration) and others: skipped
        const double td = (double)m.t;
        if (!(fabs(td) < 2251799813685248.0)) {  // the FP64 event's time limit, 2^51 ns
            bad = (int32_t)f;
            continue;
        }
        const uint32_t ty = (m.type >= '0' && m.type <= '2') ? (uint32_t)(m.type - '0') : 3u;
        const double4 e = make_double4(m.v[0], m.v[1], m.v[2],
                                       __longlong_as_double(__double_as_longlong(td) | (long long)ty));
        if (m.phase == '2') {
            if (c2 == 0) t2 = m.t;
            if (c2 < e2_max) ev2[(int64_t)c2 * batch + b] = e;
            ++c2;
        } else {
            if (c3 < e3_max) ev3[(int64_t)c3 * batch + b] = e;
            ++c3;
        }
    }
    if (b >= batch) return;
    for (int64_t e = c2; e < e2_max; ++e) ev2[e * batch + b] = none;
    for (int64_t e = c3; e < e3_max; ++e) ev3[e * batch + b] = none;
    n2[b] = c2;
    n3[b] = c3;
    first_t2[b] = t2;
    if (bad_frame) bad_frame[b] = bad;
    const int flags = (bad >= 0 ? 1 : 0) | (c2 > e2_max || c3 > e3_max ? 2 : 0);
    if (flags && err) atomicOr(err, flags);
}

}  // namespace pekf

using namespace pekf;

extern "C" int pekf_wire_events_dev(int64_t batch, int64_t n_frames, const void *frames, int64_t e2_max,
                                    int64_t e3_max, void *ev2, void *ev3, int64_t *first_t2, int32_t *n2,
                                    int32_t *n3, int32_t *bad_frame, int *dev_error, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_frames >= 0 && e2_max >= 0 && e3_max >= 0, "negative size");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(frames || n_frames == 0, "null pointer");
    PEKF_CHECK_ARG((ev2 || e2_max == 0) && (ev3 || e3_max == 0) && first_t2 && n2 && n3, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)frames % 4 == 0 && (uintptr_t)ev2 % 16 == 0 && (uintptr_t)ev3 % 16 == 0,
                   "misaligned buffers");
    PEKF_CHECK_ARG(n_frames < ((int64_t)1 << 31) && e2_max < ((int64_t)1 << 31) && e3_max < ((int64_t)1 << 31),
                   "n_frames and e_max must be < 2^31");
    hipLaunchKernelGGL(k_wire_events, dim3(grid_for(batch, kWireBlock)), dim3(kWireBlock), 0, as_stream(stream),
                       batch, n_frames, static_cast<const uint32_t *>(frames), e2_max, e3_max,
                       static_cast<double4 *>(ev2), static_cast<double4 *>(ev3), first_t2, n2, n3, bad_frame,
                       dev_error);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_wire_events");
    return PEKF_OK;
}
