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
// ([n_frames][batch][100] bytes: a wave's 64 frames of one index are 6,400 contiguous bytes, brought
// into LDS by buffer loads to LDS, the next index's in flight while this one is parsed), and
// appends each phase-2 / phase-3 message to that phase's plane as the FP64 event {x, y, z, bits(t) |
// type} (type 3 for a Type no sensor takes); the rows after a phone's last message get the no-message
// event.  With PEKF_WIRE_FRAME_ROWS a message goes to row f, its frame's index, instead (the no-message
// event to row f of the other plane): every lane of a wave stores one row however far the phones' message
// counts drift apart, and since no row depends on the frames before it, a small batch's frames are split
// into chunks over several waves, their counts combined by k_wire_rows_finalize.
//
// Frames in the client's own form are parsed without a character loop (wire_frame_fast: digit masks of
// 16-byte windows, 8 digits per SWAR conversion); any other frame by wire_frame, the general parser.
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
// The fast form reads at most a frame's first 76 bytes: tokens of at most 16 bytes from byte 5, the time's
// window of 20 from at most byte 53 (see wire_frame_fast)
constexpr int kFastDwords = 19;
constexpr int kFastSlot = kFastDwords * kWireBlock;  // 1,216 dwords: 64 frames' first 76 bytes

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

// ---- the client's own form, without a character loop ----
// Every frame the client prints has one shape: "#p,T:" then three Float.toString numbers
// ([-]D+.D+ or [-]D.D+E[-]D+, at most 9 significant digits) and "t:" with the decimal time.  Each
// token is classified from a window of its bytes at once -- a 16- or 20-bit mask of the digit bytes,
// found 4 bytes per dword operation -- and its digit runs converted 8 at a time (SWAR: 4-digit groups by
// two byte dot products and a 24-bit multiply-add each).  A token in any other form, or longer than
// the window, sends the frame to wire_frame, which decides it; where this path accepts a frame,
// wire_frame would produce the same message bit for bit: the same integer mantissa m < 10^15 and
// exponent, and the same one IEEE multiply or divide.

// bit 7 of byte j: byte j of x is not a decimal digit
__device__ __forceinline__ uint32_t other_flags(uint32_t x) {
    const uint32_t y = x ^ 0x30303030u;                              // a digit: a byte below 10
    return (((y & 0x7f7f7f7fu) + 0x76767676u) | y) & 0x80808080u;   // bit 7: y >= 10
}
// the flags of 8 bytes (two dwords) as bits 7..14 (dot products with 1, 2, 4, ... 128: 4 bytes an op)
__device__ __forceinline__ uint32_t other_bits8(uint32_t x0, uint32_t x1) {
    return __builtin_amdgcn_udot4(other_flags(x1), 0x80402010u,
                                  __builtin_amdgcn_udot4(other_flags(x0), 0x08040201u, 0u, false), false);
}

// the value of 8 decimal digits, byte 0 of lo the most significant (each byte 0..9)
__device__ __forceinline__ uint32_t swar8(uint32_t lo, uint32_t hi) {
    // (the masks only tell the compiler that the products are 24-bit: full-rate multiplies)
    auto quad = [](uint32_t x) {  // 100 (10 a + b) + 10 c + d: two dot products of the bytes, a 24-bit mad
        return (__builtin_amdgcn_udot4(x, 0x0000010au, 0u, false) & 0xffu) * 100u +
               __builtin_amdgcn_udot4(x, 0x010a0000u, 0u, false);
    };
    return (quad(lo) & 0x3fffu) * 10000u + quad(hi);
}

// the value of the L (1..8) digit characters in bytes 0..L-1 of (hi:lo)
__device__ __forceinline__ uint32_t digits_value(uint32_t lo, uint32_t hi, int L) {
    // per dword: a byte below the digits never borrows (each digit byte is >= '0')
    uint64_t v = ((uint64_t)(hi - 0x30303030u) << 32) | (uint32_t)(lo - 0x30303030u);
    v <<= 8 * (8 - L);  // the bytes past the digits leave at the top, leading zeros come in below
    return swar8((uint32_t)v, (uint32_t)(v >> 32));
}

// 8 bytes of the frame from byte pos (fr32: the frame's dwords in LDS)
__device__ __forceinline__ void wire_rd64(const uint32_t *fr32, int pos, uint32_t &lo, uint32_t &hi) {
    const int a = pos >> 2, s = pos & 3;
    const uint32_t d0 = fr32[a], d1 = fr32[a + 1], d2 = fr32[a + 2];
    lo = __builtin_amdgcn_alignbyte(d1, d0, s);
    hi = __builtin_amdgcn_alignbyte(d2, d1, s);
}

// A number at byte i of the form [-]D{1,8}.D{1,15}(E[-]D{1,2})? with at most 15 digits, all within 16
// bytes including the ',' after it, and |e10| <= 22.  i moves past the ','.  False: not this form.
__device__ __forceinline__ bool wire_number_fast(const uint32_t *fr32, const double *p10, int &i, double &out) {
    const int a = i >> 2, s = i & 3;
    const uint32_t d0 = fr32[a], d1 = fr32[a + 1], d2 = fr32[a + 2], d3 = fr32[a + 3], d4 = fr32[a + 4];
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, s), w1 = __builtin_amdgcn_alignbyte(d2, d1, s),
                   w2 = __builtin_amdgcn_alignbyte(d3, d2, s), w3 = __builtin_amdgcn_alignbyte(d4, d3, s);
    // bit j: byte j is not a digit (every bit from 16 up is set: past the window)
    const uint32_t nd = (other_bits8(w0, w1) >> 7) | (other_bits8(w2, w3) << 1) | 0xffff0000u;
    const int o = (w0 & 0xffu) == '-';
    const int p = __builtin_ctz(nd >> o << o);                 // the '.'
    const int q = __builtin_ctz(nd >> (p + 1) << (p + 1));     // past the fraction: 'E' or ','
    const int nI = p - o, nF = q - p - 1;
    const uint32_t wp = p < 4 ? w0 : (p < 8 ? w1 : w2);        // (p <= 9 where nI <= 8)
    bool ok = nI >= 1 && nI <= 8 && ((wp >> (8 * (p & 3))) & 0xffu) == '.' && nF >= 1 && nI + nF <= 15;
    uint32_t elo, ehi;
    wire_rd64(fr32, i + q, elo, ehi);
    const uint64_t ev = ((uint64_t)ehi << 32) | elo;
    const bool has_e = (elo & 0xffu) == 'E';
    const int eneg = has_e && ((elo >> 8) & 0xffu) == '-';
    const int r0 = q + 1 + eneg;
    const int r = has_e ? __builtin_ctz(nd >> r0 << r0) : q;   // the ','
    const int ne = r - r0;
    const uint64_t ex = ev >> (8 * (r0 - q));
    const int x0 = (int)(ex & 0xffu) - '0', x1 = (int)((ex >> 8) & 0xffu) - '0';
    const int e = ne == 2 ? x0 * 10 + x1 : x0;
    const int rq = r - q < 7 ? r - q : 7;
    ok = ok && ((ev >> (8 * rq)) & 0xffu) == ',' && r <= 15 && (!has_e || (ne >= 1 && ne <= 2));
    const int e10 = (has_e ? (eneg ? -e : e) : 0) - nF;
    ok = ok && e10 >= -22 && e10 <= 22;
    // m = I 10^nF + FA 10^(nF - 8) + FB: the integer digits, the first 8 and the rest of the fraction
    auto clamp = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
    const uint32_t I = digits_value(__builtin_amdgcn_alignbyte(w1, w0, o), __builtin_amdgcn_alignbyte(w2, w1, o),
                                    clamp(nI, 1, 8));
    uint32_t flo, fhi, glo, ghi;
    wire_rd64(fr32, i + p + 1, flo, fhi);
    wire_rd64(fr32, i + p + 9, glo, ghi);
    const int LB = clamp(nF - 8, 0, 8);
    const uint32_t FA = digits_value(flo, fhi, clamp(nF, 1, 8));
    const uint32_t FB = LB > 0 ? digits_value(glo, ghi, LB) : 0u;
    const double F = fma((double)FA, p10[LB], (double)FB);      // exact: integers below 10^15
    const double m = fma((double)I, p10[clamp(nF, 0, 22)], F);
    const double v = e10 < 0 ? m / p10[clamp(-e10, 0, 22)] : m * p10[clamp(e10, 0, 22)];
    out = o ? -v : v;
    i += (r < 15 ? r : 15) + 1;
    return ok;
}

// "t:" and 1..16 digits at byte i, then any non-digit
__device__ __forceinline__ bool wire_time_fast(const uint32_t *fr32, int i, long long &t) {
    const int a = i >> 2, s = i & 3;
    const uint32_t d0 = fr32[a], d1 = fr32[a + 1], d2 = fr32[a + 2], d3 = fr32[a + 3], d4 = fr32[a + 4],
                   d5 = fr32[a + 5];
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, s), w1 = __builtin_amdgcn_alignbyte(d2, d1, s),
                   w2 = __builtin_amdgcn_alignbyte(d3, d2, s), w3 = __builtin_amdgcn_alignbyte(d4, d3, s),
                   w4 = __builtin_amdgcn_alignbyte(d5, d4, s);
    const uint32_t nd = (other_bits8(w0, w1) >> 7) | (other_bits8(w2, w3) << 1) |
                        (__builtin_amdgcn_udot4(other_flags(w4), 0x08040201u, 0u, false) << 9) | 0xfff00000u;
    const int n = __builtin_ctz(nd & ~3u) - 2;  // digits from byte 2
    const bool ok = (w0 & 0xffffu) == ('t' | ':' << 8) && n >= 1 && n <= 16;
    // the last min(n, 8) digits and those before them
    const int LA = n - 8 > 0 ? n - 8 : 0, LB = n < 8 ? (n > 0 ? n : 1) : 8;
    uint32_t lo, hi;
    wire_rd64(fr32, i + 2 + LA, lo, hi);
    const uint32_t B = digits_value(lo, hi, LB);
    wire_rd64(fr32, i + 2, lo, hi);
    const uint32_t A = LA > 0 ? digits_value(lo, hi, LA < 8 ? LA : 8) : 0u;
    t = (long long)((uint64_t)A * 100000000ull + B);
    return ok;
}

// 0: a message; 1: no message (no '#'); 3: not the client's own form: wire_frame decides
__device__ __forceinline__ int wire_frame_fast(const uint32_t *fr32, const double *p10, WireMsg &m) {
    const uint32_t h0 = fr32[0], h1 = fr32[1];
    if ((h0 & 0xffu) != '#') return 1;
    m.phase = (uint8_t)(h0 >> 8);
    m.type = (uint8_t)(h0 >> 24);
    bool ok = (h1 & 0xffu) == ':' && m.type != ':' && m.type != 0;  // one Type character, the first ':'
    int i = 5;
    ok = wire_number_fast(fr32, p10, i, m.v[0]) && ok;
    ok = wire_number_fast(fr32, p10, i, m.v[1]) && ok;
    ok = wire_number_fast(fr32, p10, i, m.v[2]) && ok;
    ok = wire_time_fast(fr32, i, m.t) && ok;
    return ok ? 0 : 3;
}

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

// Two loops over the frame indices: the client's own form (wire_frame_fast) for every phone, then, for the
// phones that met a frame in another form, wire_frame from that frame on.  Held to 4 waves per SIMD
// (128 VGPRs: the fast loop needs 126 and does not spill; the second loop's big-integer path does).
// 262,144 phones x 1,024 frames, same box (profiles/r6/wire_dev/): the character loops of wire_frame
// alone took 29.8 ms (byte loops with early exits, 2 waves) -> 27.5 (branch-free digit loops) -> 25.4 ms
// (3 waves) -> 23.6 ms (loop exits wave-uniform, __any); the fast form, 7.9 ms (800 VALU per wave and frame
// against 1,302 VALU + 1,352 SALU, and no chain of dependent one-byte LDS reads), 7.8 ms with dot products
// for the mask gathers and SWAR steps (656 VALU), 7.7 ms with the frames' first 76 bytes brought into a
// two-slot LDS ring by buffer loads to LDS (no registers for the frame in flight; parsing without loads
// at all takes 5.4 ms).  Not kept: the frame's commas found first so the four token windows are
// independent (+90 VALU, 1 % slower); two frames per lane and step at low occupancy (no gain); a
// dword-window reader instead of byte reads (36.6 against 29.8 ms), and every check of a token as a
// status flag instead of an exit (35.2 against 23.7 ms: the division and the big-integer path then run for
// every lane, and the registers spill).
// ROWS (PEKF_WIRE_FRAME_ROWS): frame f's message goes to row f of its phase's plane and the no-message
// event to row f of the other, so every lane of a wave stores the same row (see pekf.h).
template <bool ROWS>
__global__ __launch_bounds__(kWireBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_wire_events(
    int64_t batch, int64_t n_frames, const uint32_t *__restrict__ frames, int64_t e2_max, int64_t e3_max,
    double4 *__restrict__ ev2, double4 *__restrict__ ev3, int64_t *__restrict__ first_t2, int32_t *__restrict__ n2,
    int32_t *__restrict__ n3, int32_t *__restrict__ bad_frame, int *__restrict__ err, int64_t f_per_chunk,
    int4 *__restrict__ part, int64_t *__restrict__ part_t2, int32_t *__restrict__ bounds) {
    // (ROWS, f_per_chunk > 0: block row blockIdx.y parses frames [fb, fe) and leaves its counts, first
    // phase-2 time and refused frame in part / part_t2 [chunk][batch] for k_wire_rows_finalize)
    const int64_t fb = f_per_chunk > 0 ? (int64_t)blockIdx.y * f_per_chunk : 0;
    const int64_t fe = f_per_chunk > 0 && fb + f_per_chunk < n_frames ? fb + f_per_chunk : n_frames;
    // One LDS array (a second __shared__ object can make the compiler drain the DMA ring, vmcnt(0)):
    // the fast loop's ring of two slots of 64 frames' first 76 bytes, written by buffer loads to LDS; the
    // second loop's 64 whole frames; the powers of ten at the end.
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * kFastSlot + 46];
    double *p10 = reinterpret_cast<double *>(lds + 2 * kFastSlot);
    const int lane = threadIdx.x;
    if (lane < 23) p10[lane] = kWirePow10[lane];
    const int64_t k0 = (int64_t)blockIdx.x * kWireBlock;
    const int64_t b = k0 + lane;
    const int nk = batch - k0 < kWireBlock ? (int)(batch - k0) : kWireBlock;  // phones in this block
    const int nd = nk * (kWireFrame / 4);  // dwords of one frame index
    // dword j of frame index f of this block's phones (frames of one index are contiguous across phones),
    // through a buffer resource of exactly those frames: a lane past the block's last phone reads 0
    // (6 x 16 bytes per lane, 1 KiB per wave-instruction, and one dword: the 6,400 bytes of a frame index)
    auto load = [&](int64_t f, uint32_t (&r)[kWireDwords / kWireBlock]) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(frames + (f * batch + k0) * (kWireFrame / 4)), 0, nd * 4, 0x00020000);
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const uint4 v = __builtin_bit_cast(
                uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, c * 1024 + lane * 16, 0, 2));
            r[4 * c] = v.x, r[4 * c + 1] = v.y, r[4 * c + 2] = v.z, r[4 * c + 3] = v.w;
        }
        r[24] = __builtin_amdgcn_raw_buffer_load_b32(rs, 6144 + lane * 4, 0, 2);
    };
    auto stage = [&](const uint32_t (&r)[kWireDwords / kWireBlock]) {
#pragma unroll
        for (int c = 0; c < 6; ++c)
            *reinterpret_cast<uint4 *>(lds + 256 * c + 4 * lane) = make_uint4(r[4 * c], r[4 * c + 1], r[4 * c + 2],
                                                                              r[4 * c + 3]);
        lds[1536 + lane] = r[24];
    };
    // The fast loop's DMA: dword j (j < 64 x 19) of a slot is dword j % 19 of the block's frame j / 19
    uint32_t off[kFastDwords];
#pragma unroll
    for (int c = 0; c < kFastDwords; ++c) {
        const int j = c * kWireBlock + lane;
        off[c] = (uint32_t)((j / kFastDwords) * kWireFrame + (j % kFastDwords) * 4);
    }
    auto dma = [&](int64_t f, int slot) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint32_t *>(frames + (f * batch + k0) * (kWireFrame / 4)), 0, nd * 4, 0x00020000);
#pragma unroll
        for (int c = 0; c < kFastDwords; ++c)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void *)(lds + slot * kFastSlot + c * kWireBlock), 4, off[c],
                0, 0, 2);
    };
    const uint8_t *fr = reinterpret_cast<const uint8_t *>(lds) + lane * kWireFrame;
    int32_t c2 = 0, c3 = 0, bad = -1, resume = -1;
    int32_t end2 = 0, from3 = 0;  // (ROWS, bounds) 1 + the last phase-2 row, n_frames - the first phase-3 row
    int64_t t2 = 0;
    const double4 none = ev64_null();
    // One parsed frame: a message to its phase's next row (ROWS: to row f, and the no-message event to
    // row f of the other plane); a refused frame ends the phone
    auto take = [&](int st, const WireMsg &m, int64_t f) {
        double4 e2r = none, e3r = none;  // (ROWS) row f of each plane
        if (st == 2) {
            bad = (int32_t)f;
        } else if (st == 0 && (m.phase == '2' || m.phase == '3')) {  // phase 1 (calibration), others: skipped
            const double td = (double)m.t;
            if (!(fabs(td) < 2251799813685248.0)) {  // the FP64 event's time limit, 2^51 ns
                bad = (int32_t)f;
            } else {
                const uint32_t ty = (m.type >= '0' && m.type <= '2') ? (uint32_t)(m.type - '0') : 3u;
                const double4 e = make_double4(m.v[0], m.v[1], m.v[2],
                                               __longlong_as_double(__double_as_longlong(td) | (long long)ty));
                if (m.phase == '2') {
                    if (c2 == 0) t2 = m.t;
                    if constexpr (ROWS) {
                        e2r = e;
                        end2 = (int32_t)f + 1;
                    }
                    else if (c2 < e2_max)
                        ev2[(int64_t)c2 * batch + b] = e;
                    ++c2;
                } else {
                    if constexpr (ROWS) {
                        e3r = e;
                        if (from3 == 0) from3 = (int32_t)(n_frames - f);
                    }
                    else if (c3 < e3_max)
                        ev3[(int64_t)c3 * batch + b] = e;
                    ++c3;
                }
            }
        }
        if constexpr (ROWS) {
            if (bad < 0) {  // (a stopped phone's rows are filled at the end)
                ev2[f * batch + b] = e2r;
                ev3[f * batch + b] = e3r;
            }
        }
    };
    // One wave per block: no barrier (its fence would wait for the ring, vmcnt(0)); the wave's own waits
    // order its DMA and its LDS reads.  Frame index f + 1's DMA is in flight while f is parsed; loads
    // return in order, so at most 19 outstanding vector memory operations (whatever event stores are among
    // them) means that all of f's have landed.
    static_assert(kFastDwords == 19, "the vmcnt below counts one frame index's DMA instructions");
    if (fb < fe) dma(fb, (int)(fb & 1));
    for (int64_t f = fb; f < fe; ++f) {
        if (f + 1 < fe) {
            dma(f + 1, (int)((f + 1) & 1));
            asm volatile("s_waitcnt vmcnt(19)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (b >= batch || bad >= 0 || resume >= 0) continue;
        WireMsg m;
        const int st = wire_frame_fast(lds + (f & 1) * kFastSlot + lane * kFastDwords, p10, m);
        if (st == 3) {
            resume = (int32_t)f;  // a frame in another form: this phone goes on below
            continue;
        }
        take(st, m, f);
    }
    // The phones that met a frame in another form go on from it with wire_frame, the block's frames from
    // the first such index staged again (a separate loop: the two parsers' registers are not live at once)
    int f0 = resume >= 0 ? resume : INT_MAX;
    for (int d = 1; d < kWireBlock; d <<= 1) f0 = min(f0, __shfl_xor(f0, d));
    uint32_t cur[kWireDwords / kWireBlock];
    for (int64_t f = f0; f < fe; ++f) {
        __syncthreads();
        load(f, cur);
        stage(cur);
        __syncthreads();
        if (b >= batch || bad >= 0 || resume < 0 || f < resume) continue;
        WireMsg m;
        const int st = wire_frame(fr, m);
        take(st, m, f);
    }
    if (ROWS && bounds) {  // the rows the planes' consumers need: max over the wave, one atomic per wave
        for (int d = 1; d < kWireBlock; d <<= 1) {
            end2 = max(end2, __shfl_xor(end2, d));
            from3 = max(from3, __shfl_xor(from3, d));
        }
        if (lane == 0) {
            atomicMax(bounds, end2);
            atomicMax(bounds + 1, from3);
        }
    }
    if (b >= batch) return;
    if (part) {
        part[(int64_t)blockIdx.y * batch + b] = make_int4(c2, c3, bad, 0);
        part_t2[(int64_t)blockIdx.y * batch + b] = t2;
        return;
    }
    if constexpr (ROWS) {  // rows from the frame that stopped the phone, or past the last frame
        const int64_t r0 = bad >= 0 ? bad : n_frames;
        for (int64_t e = r0; e < e2_max; ++e) ev2[e * batch + b] = none;
        for (int64_t e = r0; e < e3_max; ++e) ev3[e * batch + b] = none;
    } else {
        for (int64_t e = c2; e < e2_max; ++e) ev2[e * batch + b] = none;
        for (int64_t e = c3; e < e3_max; ++e) ev3[e * batch + b] = none;
    }
    n2[b] = c2;
    n3[b] = c3;
    first_t2[b] = t2;
    if (bad_frame) bad_frame[b] = bad;
    const int flags = (bad >= 0 ? 1 : 0) | (c2 > e2_max || c3 > e3_max ? 2 : 0);
    if (flags && err) atomicOr(err, flags);
}

// A phone's chunks in frame order: its counts up to its first refused frame, its first phase-2 time,
// and no-message rows from the refused frame (or the last frame) on.
__global__ __launch_bounds__(256) void k_wire_rows_finalize(int64_t batch, int64_t n_frames, int64_t n_chunks,
                                                            const int4 *__restrict__ part,
                                                            const int64_t *__restrict__ part_t2, int64_t e2_max,
                                                            int64_t e3_max, double4 *__restrict__ ev2,
                                                            double4 *__restrict__ ev3, int64_t *__restrict__ first_t2,
                                                            int32_t *__restrict__ n2, int32_t *__restrict__ n3,
                                                            int32_t *__restrict__ bad_frame, int *__restrict__ err) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    int32_t c2 = 0, c3 = 0, bad = -1;
    int64_t t2 = 0;
    for (int64_t ch = 0; ch < n_chunks; ++ch) {
        const int4 p = part[ch * batch + b];
        if (c2 == 0 && p.x > 0) t2 = part_t2[ch * batch + b];
        c2 += p.x;
        c3 += p.y;
        if (p.z >= 0) {  // the phone stopped here: later chunks' frames are not its messages
            bad = p.z;
            break;
        }
    }
    const double4 none = ev64_null();
    const int64_t r0 = bad >= 0 ? bad : n_frames;
    for (int64_t e = r0; e < e2_max; ++e) ev2[e * batch + b] = none;
    for (int64_t e = r0; e < e3_max; ++e) ev3[e * batch + b] = none;
    n2[b] = c2;
    n3[b] = c3;
    first_t2[b] = t2;
    if (bad_frame) bad_frame[b] = bad;
    if (bad >= 0 && err) atomicOr(err, 1);
}

}  // namespace pekf

using namespace pekf;

extern "C" int pekf_wire_events_ext_dev(int64_t batch, int64_t n_frames, const void *frames, int64_t e2_max,
                                        int64_t e3_max, void *ev2, void *ev3, int64_t *first_t2, int32_t *n2,
                                        int32_t *n3, int32_t *bad_frame, int *dev_error, int32_t *row_bounds,
                                        uint32_t flags, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_frames >= 0 && e2_max >= 0 && e3_max >= 0, "negative size");
    PEKF_CHECK_ARG((flags & ~(uint32_t)PEKF_WIRE_FRAME_ROWS) == 0, "unknown flags");
    const bool rows = flags & PEKF_WIRE_FRAME_ROWS;
    PEKF_CHECK_ARG(!rows || (e2_max >= n_frames && e3_max >= n_frames),
                   "PEKF_WIRE_FRAME_ROWS: the planes need a row per frame index (e_max >= n_frames)");
    if (batch == 0) return PEKF_OK;
    PEKF_CHECK_ARG(frames || n_frames == 0, "null pointer");
    PEKF_CHECK_ARG((ev2 || e2_max == 0) && (ev3 || e3_max == 0) && first_t2 && n2 && n3, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)frames % 4 == 0 && (uintptr_t)ev2 % 16 == 0 && (uintptr_t)ev3 % 16 == 0,
                   "misaligned buffers");
    PEKF_CHECK_ARG(n_frames < ((int64_t)1 << 31) && e2_max < ((int64_t)1 << 31) && e3_max < ((int64_t)1 << 31),
                   "n_frames and e_max must be < 2^31");
    // Frame rows need no count before a frame's store: where the grid leaves SIMDs short of 4 waves, the
    // frames are split into chunks parsed by separate waves (PEKF_WIRE_CHUNKS=n forces n) and their
    // counts combined after.
    const int64_t waves = grid_for(batch, kWireBlock);
    int64_t chunks = 1;
    if (rows) {
        const char *ec = getenv("PEKF_WIRE_CHUNKS");
        if (ec && atoi(ec) > 0) {
            chunks = atoi(ec);
        } else {
            int dev = 0, cus = 0;
            if (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
                chunks = ((int64_t)cus * 16 + waves - 1) / waves;
            const int64_t most = n_frames / 128;  // chunks of at least 128 frame indices
            chunks = chunks < most ? chunks : most;
            chunks = chunks < 16 ? chunks : 16;
        }
        chunks = chunks < n_frames ? chunks : n_frames;
        if (chunks < 1) chunks = 1;
    }
    const int64_t per = chunks > 1 ? (n_frames + chunks - 1) / chunks : 0;
    if (per) chunks = (n_frames + per - 1) / per;
    int4 *part = nullptr;
    int64_t *part_t2 = nullptr;
    hipStream_t st = as_stream(stream);
    if (rows && row_bounds) {
        hipError_t z = hipMemsetAsync(row_bounds, 0, 2 * sizeof(int32_t), st);
        if (z != hipSuccess) return hip_fail(z, "k_wire_events row bounds");
    }
    if (per) {
        hipError_t a = hipMallocAsync(reinterpret_cast<void **>(&part), (size_t)(chunks * batch) * 24, st);
        if (a != hipSuccess) return hip_fail(a, "k_wire_events chunk counts");
        part_t2 = reinterpret_cast<int64_t *>(part + chunks * batch);
    }
    auto launch = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(waves, per ? chunks : 1), dim3(kWireBlock), 0, st, batch, n_frames,
                           static_cast<const uint32_t *>(frames), e2_max, e3_max, static_cast<double4 *>(ev2),
                           static_cast<double4 *>(ev3), first_t2, n2, n3, bad_frame, dev_error, per, part, part_t2,
                           rows ? row_bounds : nullptr);
    };
    if (rows)
        launch(k_wire_events<true>);
    else
        launch(k_wire_events<false>);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_wire_events");
    if (per) {
        hipLaunchKernelGGL(k_wire_rows_finalize, dim3(grid_for(batch, 256)), dim3(256), 0, st, batch, n_frames, chunks,
                           part, part_t2, e2_max, e3_max, static_cast<double4 *>(ev2), static_cast<double4 *>(ev3),
                           first_t2, n2, n3, bad_frame, dev_error);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_wire_rows_finalize");
        e = hipFreeAsync(part, st);
        if (e != hipSuccess) return hip_fail(e, "k_wire_events chunk counts");
    }
    return PEKF_OK;
}

extern "C" int pekf_wire_events_dev(int64_t batch, int64_t n_frames, const void *frames, int64_t e2_max,
                                    int64_t e3_max, void *ev2, void *ev3, int64_t *first_t2, int32_t *n2,
                                    int32_t *n3, int32_t *bad_frame, int *dev_error, void *stream) {
    return pekf_wire_events_ext_dev(batch, n_frames, frames, e2_max, e3_max, ev2, ev3, first_t2, n2, n3, bad_frame,
                                    dev_error, nullptr, 0u, stream);
}
