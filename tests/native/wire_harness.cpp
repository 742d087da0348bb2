// Host-only harness for the wire parser (csrc/pekf_wire.cpp) under AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_log_sanitizers.py builds and runs it; no GPU, no HIP).  Each
// argument is a text file: count its messages, parse them into exactly-sized outputs, and parse with one
// slot too few; then pekf_f32_wire_values over every class of float.  pekf::set_error (pekf_capi.hip in
// the library) is replaced by a printing stub.
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "pekf.h"

namespace pekf {
int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char msg[512];
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    fprintf(stderr, "error %d: %s\n", code, msg);
    return code;
}
}  // namespace pekf

int main(int argc, char **argv) {
    for (int i = 1; i < argc; ++i) {
        std::string text;
        if (std::FILE *f = std::fopen(argv[i], "rb")) {
            char buf[4096];
            size_t n;
            while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
            std::fclose(f);
        }
        // an exactly-sized heap copy, so reading past the end is a sanitizer report
        std::vector<char> exact(text.begin(), text.end());
        const char *p = exact.empty() ? "" : exact.data();
        int64_t n = -1, m = -1;
        const int scan = pekf_wire_parse(p, (int64_t)exact.size(), 0, nullptr, nullptr, nullptr, nullptr, &n);
        printf("%s scan=%d messages=%lld", argv[i], scan, (long long)n);
        if (scan == 0 && n > 0) {
            std::vector<uint8_t> ph(n), ty(n);
            std::vector<double> xyz(3 * n);
            std::vector<int64_t> t(n);
            const int full = pekf_wire_parse(p, (int64_t)exact.size(), n, ph.data(), ty.data(), xyz.data(), t.data(), &m);
            const int under = pekf_wire_parse(p, (int64_t)exact.size(), n - 1, ph.data(), ty.data(), xyz.data(),
                                              t.data(), &m);
            double sum = 0;
            for (double v : xyz) sum += std::isfinite(v) ? v : 0.0;
            printf(" full=%d under=%d first_t=%lld sum=%.6g", full, under, (long long)t[0], sum);
        }
        printf("\n");
    }
    // every class of float: zeros, subnormals, normals, powers of ten, extremes, inf, NaN
    std::vector<float> f = {0.0f, -0.0f, 1e-45f, -1.4e-45f, 1.17549435e-38f, 0.1f, 9.81f, 1e7f, 3.4028235e38f,
                            std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                            std::numeric_limits<float>::quiet_NaN()};
    for (uint32_t b = 1; b < 4000000000u; b += 99991u) {
        float x;
        std::memcpy(&x, &b, 4);
        f.push_back(x);
    }
    std::vector<double> out(f.size());
    const int st = pekf_f32_wire_values((int64_t)f.size(), f.data(), out.data());
    int64_t back = 0;
    for (size_t k = 0; k < f.size(); ++k)
        back += (std::isnan(f[k]) && std::isnan(out[k])) || (float)out[k] == f[k];
    printf("f32_wire_values=%d n=%zu roundtrip=%lld\n", st, f.size(), (long long)back);
    return 0;
}
