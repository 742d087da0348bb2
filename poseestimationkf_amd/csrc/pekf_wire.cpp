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

// The double std::stod makes of Float.toString(f).
double wire_value(float f) {
    if (!std::isfinite(f) || f == 0.0f) return (double)f;  // "NaN", "Infinity", "0.0", "-0.0": exact
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf) - 1, f, std::chars_format::scientific);
    int digits = 0;
    for (const char *p = buf; p < r.ptr && *p != 'e'; ++p) digits += (*p >= '0' && *p <= '9');
    if (digits == 1) r = std::to_chars(buf, buf + sizeof(buf) - 1, f, std::chars_format::scientific, 1);
    *r.ptr = '\0';
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
        int64_t j = i;
        while (j < len && text[j] != '\n') ++j;
        const int64_t end = j < len ? j + 1 : j;
        ++line;
        // Parser::run: only messages starting with '#', without it; ProcessString: longer than 30
        if (text[i] == '#' && end - i - 1 > 30) {
            msg.assign(text + i + 1, (size_t)(end - i - 1));
            const char ph = msg[0];
            const char *s = msg.c_str() + 2;  // str.substr(2): past "<phase>,"
            const char *colon = std::strchr(s, ':');
            const char ty = (colon && colon > s) ? s[0] : '\0';  // FindValues(str, ":")[0]
            double v[3] = {0, 0, 0};
            bool ok = colon != nullptr;
            const char *p = ok ? colon + 1 : s;
            for (int k = 0; ok && k < 3; ++k) {  // std::stod of the text before each ','
                const char *comma = std::strchr(p, ',');
                char *e = nullptr;
                errno = 0;
                v[k] = pekf::strtod_c(p, &e);
                ok = comma && e != p && errno != ERANGE;
                p = comma ? comma + 1 : p;
            }
            const char *tp = ok ? std::strstr(p, "t:") : nullptr;  // std::stoll of the text after "t:"
            long long t = 0;
            if (tp) {
                char *e = nullptr;
                errno = 0;
                t = std::strtoll(tp + 2, &e, 10);
                ok = e != tp + 2 && errno != ERANGE;
            } else {
                ok = false;
            }
            if (!ok)  // the server's std::stod / std::stoll would throw here
                return pekf::set_error(PEKF_ERR_INVALID, "wire message %lld: not '#<phase>,<type>:<x>,<y>,<z>,t:<ns>'",
                                       (long long)line);
            if (fill) {
                if (n >= max_events)
                    return pekf::set_error(PEKF_ERR_INVALID, "more than max_events = %lld messages",
                                           (long long)max_events);
                phase[n] = (uint8_t)(ph - '0');
                type[n] = (uint8_t)(ty - '0');
                xyz[3 * n] = v[0];
                xyz[3 * n + 1] = v[1];
                xyz[3 * n + 2] = v[2];
                t_ns[n] = (int64_t)t;
            }
            ++n;
        }
        i = end;
    }
    *n_events = n;
    return PEKF_OK;
}

}  // extern "C"
