// pekf_wire.cpp -- host side of the phone -> server link: the sample values the
// server actually computes with.  Host code, no device work; it packs the FP64 event planes
// (PEKF_EV_F64_EVENTS, include/pekf.h) of pekf_live_ext_dev / pekf_frontend_ext_dev /
// pekf_frontend_init_ext_dev.
//
// The Android client sends every sample as text: Float.toString(f) for each of the three values
// (ASC/MessageSender.java:217-233, ConvertSensorMsg: "#<phase>,<type>:<x>,<y>,<z>,t:<ns>" padded with
// spaces to 99 characters, println'ed), and the server parses each value with std::stod into a double
// (KFS/Parser.cpp:12-26, ProcessString) -- the double nearest the printed decimal, which in general is
// not the float itself (e.g. "0.1" is 0.1, not 0.100000001490116...).
//
//  * pekf_wire_parse: the server's own parse of such text (Parser::run's '#' test and ProcessString's
//    length test and field splitting, strtod / strtoll as std::stod / std::stoll call them, strtod in the
//    "C" locale, pekf_cnum.hpp).
//  * pekf_f32_wire_values: for samples known only as floats, the double the server would parse from
//    Float.toString(f).  Float.toString prints the shortest decimal that rounds to f, the closest to f
//    among those (JDK 19+ specification; for a float whose shortest decimal has one digit it picks the
//    closest decimal of one or two digits); std::to_chars gives the shortest closest digits, and the
//    two-digit case is to_chars with precision 1 (correctly rounded from f's exact value).
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/pekf.h"
#include "pekf_cnum.hpp"

namespace pekf {
int set_error(int code, const char *fmt, ...);  // pekf_capi.hip
}

namespace {

// One parsed message: the phase and type characters, the three stod values and the stoll time.
struct Message {
    char ph, ty;
    double v[3];
    long long t;
};

// The powers of ten a double holds exactly
constexpr double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                               1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// A plain decimal [+-]digits[.digits][(e|E)[+-]digits] at p, immediately followed by `term` (',' in a
// message; '\0': the decimal ends at mend):
// true with its value when one IEEE multiply or divide of two exact doubles gives it -- at most 19
// significant digits with a mantissa <= 2^53 and a decimal exponent within +-22 -- which is then the
// correctly rounded decimal, strtod's own result; false for anything else (the caller's strtod path).
// p is left on the terminator.
bool fast_decimal(const char *&p, const char *mend, double &out, char term = ',') {
    const char *q = p;
    bool neg = false;
    if (q < mend && (*q == '+' || *q == '-')) neg = *q++ == '-';
    uint64_t m = 0;
    int nd = 0, exp10 = 0;
    bool any = false;
    for (; q < mend && (unsigned)(*q - '0') < 10u; ++q) {
        any = true;
        if (m || *q != '0') {
            if (++nd > 19) return false;
            m = m * 10 + (uint64_t)(*q - '0');
        }
    }
    if (q < mend && *q == '.') {
        for (++q; q < mend && (unsigned)(*q - '0') < 10u; ++q) {
            any = true;
            if (m || *q != '0') {
                if (++nd > 19) return false;
                m = m * 10 + (uint64_t)(*q - '0');
            }
            --exp10;
        }
    }
    if (!any) return false;
    if (q < mend && (*q == 'e' || *q == 'E')) {
        ++q;
        bool eneg = false;
        if (q < mend && (*q == '+' || *q == '-')) eneg = *q++ == '-';
        int e = 0, ne = 0;
        for (; q < mend && (unsigned)(*q - '0') < 10u; ++q) {
            if (++ne > 4) return false;
            e = e * 10 + (*q - '0');
        }
        if (!ne) return false;
        exp10 += eneg ? -e : e;
    }
    if (term ? (q >= mend || *q != term) : q != mend) return false;
    if (m > (1ull << 53) || exp10 < -22 || exp10 > 22) return false;
    const double d = exp10 < 0 ? (double)m / kPow10[-exp10] : (double)m * kPow10[exp10];
    out = neg ? -d : d;
    p = q;
    return true;
}

// The client's own message form, "<phase>,<type>:<x>,<y>,<z>,t:<ns>..." with plain decimals (msg = the
// text after '#', up to mend): parsed in place, with the server's semantics (see parse_general) for the
// cases it takes; false for anything else.
bool parse_fast(const char *msg, const char *mend, Message &o) {
    o.ph = msg[0];
    const char *s = msg + 2, *colon = s;
    while (colon < mend && *colon != ':') {
        if (*colon == '\0') return false;
        ++colon;
    }
    if (colon >= mend) return false;
    o.ty = colon > s ? s[0] : '\0';
    const char *p = colon + 1;
    for (int k = 0; k < 3; ++k) {
        if (!fast_decimal(p, mend, o.v[k])) return false;
        ++p;  // past the ','
    }
    if (mend - p < 3 || p[0] != 't' || p[1] != ':') return false;
    const char *q = p + 2;
    const bool neg = *q == '-';
    if (neg) ++q;
    long long t = 0;
    int nd = 0;
    for (; q < mend && (unsigned)(*q - '0') < 10u; ++q) {
        if (++nd > 18) return false;
        t = t * 10 + (*q - '0');
    }
    if (!nd) return false;
    o.t = neg ? -t : t;
    return true;
}

// Any message, as the server reads it: Type = the first character before the first ':'
// (FindValues(str, ":")[0]), each value std::stod of the text before the next ',' (strtod: leading
// blanks, a sign, hex, inf / nan, trailing text ignored; ERANGE throws), the time std::stoll of the text
// after the first "t:" that follows.  false where the server's stod / stoll would throw.
bool parse_general(std::string &msg, const char *text, int64_t len, Message &o) {
    msg.assign(text, (size_t)len);
    o.ph = msg[0];
    const char *s = msg.c_str() + 2;  // str.substr(2): past "<phase>,"
    const char *colon = std::strchr(s, ':');
    o.ty = (colon && colon > s) ? s[0] : '\0';  // FindValues(str, ":")[0]
    bool ok = colon != nullptr;
    const char *p = ok ? colon + 1 : s;
    for (int k = 0; ok && k < 3; ++k) {  // std::stod of the text before each ','
        const char *comma = std::strchr(p, ',');
        char *e = nullptr;
        errno = 0;
        o.v[k] = pekf::strtod_c(p, &e);
        ok = comma && e != p && errno != ERANGE;
        p = comma ? comma + 1 : p;
    }
    const char *tp = ok ? std::strstr(p, "t:") : nullptr;  // std::stoll of the text after "t:"
    if (!tp) return false;
    char *e = nullptr;
    errno = 0;
    o.t = std::strtoll(tp + 2, &e, 10);
    return e != tp + 2 && errno != ERANGE;
}

// The double std::stod makes of Float.toString(f): the printed decimal read back by the exact fast path
// where it applies, else by strtod.
double wire_value(float f) {
    if (!std::isfinite(f) || f == 0.0f) return (double)f;  // "NaN", "Infinity", "0.0", "-0.0": exact
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf) - 1, f, std::chars_format::scientific);
    int digits = 0;
    for (const char *p = buf; p < r.ptr && *p != 'e'; ++p) digits += (*p >= '0' && *p <= '9');
    if (digits == 1) r = std::to_chars(buf, buf + sizeof(buf) - 1, f, std::chars_format::scientific, 1);
    *r.ptr = '\0';
    const char *p = buf;
    double v;
    if (fast_decimal(p, r.ptr, v, '\0')) return v;
    return pekf::strtod_c(buf, nullptr);
}

}  // namespace

extern "C" {

int pekf_f32_wire_values(int64_t n, const float *in, double *out) {
    if (n < 0) return pekf::set_error(PEKF_ERR_INVALID, "negative size");
    if (n > 0 && (!in || !out)) return pekf::set_error(PEKF_ERR_INVALID, "null pointer");
    for (int64_t i = 0; i < n; ++i) out[i] = wire_value(in[i]);
    return PEKF_OK;
}

int pekf_wire_parse(const char *text, int64_t len, int64_t max_events, uint8_t *phase, uint8_t *type, double *xyz,
                    int64_t *t_ns, int64_t *n_events) {
    if (!text || len < 0 || !n_events) return pekf::set_error(PEKF_ERR_INVALID, "null pointer or negative size");
    const bool fill = phase || type || xyz || t_ns;
    if (fill && !(phase && type && xyz && t_ns)) return pekf::set_error(PEKF_ERR_INVALID, "need all four outputs");
    int64_t n = 0, line = 0;
    std::string msg;
    for (int64_t i = 0; i < len;) {
        // one message: up to and including its newline (the server's 100-byte frame holds the newline)
        const char *nl = static_cast<const char *>(std::memchr(text + i, '\n', (size_t)(len - i)));
        const int64_t end = nl ? (nl - text) + 1 : len;
        ++line;
        // Parser::run: only messages starting with '#', without it; ProcessString: longer than 30
        if (text[i] == '#' && end - i - 1 > 30) {
            Message m;
            if (!parse_fast(text + i + 1, text + end, m) && !parse_general(msg, text + i + 1, end - i - 1, m))
                return pekf::set_error(PEKF_ERR_INVALID, "wire message %lld: not '#<phase>,<type>:<x>,<y>,<z>,t:<ns>'",
                                       (long long)line);  // the server's std::stod / std::stoll would throw here
            if (fill) {
                if (n >= max_events)
                    return pekf::set_error(PEKF_ERR_INVALID, "more than max_events = %lld messages",
                                           (long long)max_events);
                phase[n] = (uint8_t)(m.ph - '0');
                type[n] = (uint8_t)(m.ty - '0');
                xyz[3 * n] = m.v[0];
                xyz[3 * n + 1] = m.v[1];
                xyz[3 * n + 2] = m.v[2];
                t_ns[n] = (int64_t)m.t;
            }
            ++n;
        }
        i = end;
    }
    *n_events = n;
    return PEKF_OK;
}

}  // extern "C"
