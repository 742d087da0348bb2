// Host-only harness for the native log reader (csrc/pekf_log.cpp) under AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_log_sanitizers.py builds and runs it; no GPU, no HIP).
// Each argument is a log path: scan it, then read it with and without the dt side plane, as float64
// records, and with one record too many; then write the float64 records back (pekf_log_write) and scan
// the result.  pekf::set_error (pekf_capi.hip in the library) is replaced by a printing stub.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
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
        int64_t n = -1;
        int st = pekf_log_scan(argv[i], &n);
        printf("%s scan=%d records=%lld", argv[i], st, (long long)n);
        if (st == 0 && n > 0) {
            std::vector<float> g(3 * n), a(3 * n), m(3 * n);
            std::vector<uint32_t> dtw(n);
            std::vector<double> dtx(n);
            double acc0[3], mag0[3], t0 = 0;
            int64_t esc = -1;
            const int ext = pekf_log_read_ext(argv[i], n, g.data(), a.data(), m.data(), dtw.data(), dtx.data(), &esc,
                                              acc0, mag0, &t0);
            const int plain = pekf_log_read(argv[i], n, g.data(), a.data(), m.data(), dtw.data(), acc0, mag0, &t0);
            const int over = pekf_log_read_ext(argv[i], n + 1, g.data(), a.data(), m.data(), dtw.data(), dtx.data(),
                                               &esc, acc0, mag0, &t0);
            std::vector<double> g64(3 * n), a64(3 * n), m64(3 * n), dt64(n);
            const int r64 = pekf_log_read64(argv[i], n, g64.data(), a64.data(), m64.data(), dt64.data(), acc0, mag0, &t0);
            const int over64 =
                pekf_log_read64(argv[i], n + 1, g64.data(), a64.data(), m64.data(), dt64.data(), acc0, mag0, &t0);
            printf(" ext=%d escaped=%lld plain=%d over=%d r64=%d over64=%d", ext, (long long)esc, plain, over, r64,
                   over64);
            if (r64 == 0) {  // the emit side: the float64 records written back, then scanned again
                std::vector<int64_t> t(n + 1);
                t[0] = (int64_t)t0;
                for (int64_t k = 0; k < n; ++k) t[k + 1] = t[k] + (int64_t)dt64[k];
                std::vector<double> xk(4 * n, 0.5);  // a side channel (the others absent: zeros)
                const std::string out = std::string(argv[i]) + ".out";
                const int w = pekf_log_write(out.c_str(), n, t.data(), g64.data(), a64.data(), m64.data(), acc0, mag0,
                                             nullptr, xk.data(), nullptr);
                int64_t n2 = -1;
                const int s2 = pekf_log_scan(out.c_str(), &n2);
                printf(" write=%d rescan=%d records=%lld", w, s2, (long long)n2);
            }
        }
        printf("\n");
    }
    return 0;
}
