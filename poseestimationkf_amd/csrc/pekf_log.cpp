// pekf_log.cpp -- native ingest of the live server's text log into the 40 B record stream
// (SURVEY.md §8f-1), and its emit (pekf_log_write: the lines the server's KalmanFilter writes).  Host
// code (no device work): it feeds pekf_run_dev with recorded phone traces.
//
// Line tags and precedence follow the offline reader (Python Kalman Filter/ReadFile.py:27-45):
// mag_0, acc_0, Acc_1, Mag_1, q_gyro, gyro, any line containing 'T', Wahba_quart, X_k; values are
// the comma-separated numbers after the first ':' (strtod in the "C" locale == Python float() for these
// tokens, pekf_cnum.hpp).
// Records follow main_file.py:19-47: one per Acc_1 line, record i uses gyro[i], Mag_1[i],
// Acc_1[i] and dt_i = T[i+1] - T[i] (float64, as ExtendedKalmanFilter.py:62 computes
// T - previousT with previousT starting at the first timestamp).
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pekf.h"
#include "pekf_cnum.hpp"

namespace pekf {
int set_error(int code, const char *fmt, ...);  // pekf_capi.hip
}

namespace {

struct LogColumns {
    std::vector<double> mag0, acc0, T;
    std::vector<double> acc1, mag1, gyro;  // flattened triples
};

bool values(const char *line, std::vector<double> &dst, int want) {
    const char *p = std::strchr(line, ':');
    if (!p) return false;
    ++p;
    int got = 0;
    while (*p) {
        char *end = nullptr;
        errno = 0;
        const double v = pekf::strtod_c(p, &end);
        if (end == p) return false;
        dst.push_back(v);
        ++got;
        p = end;
        while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') ++p;
        if (*p == ',') {
            ++p;
        } else {
            break;
        }
    }
    return want < 0 || got == want;
}

int parse(const char *path, LogColumns &c) {
    FILE *f = std::fopen(path, "r");
    if (!f) return pekf::set_error(PEKF_ERR_INVALID, "cannot open log '%s': %s", path, std::strerror(errno));
    char *buf = nullptr;  // whole lines of any length, as Python's line iteration gives them
    size_t cap = 0;
    int64_t lineno = 0;
    int status = PEKF_OK;
    while (getline(&buf, &cap, f) != -1) {
        ++lineno;
        const char *l = buf;
        bool ok = true;
        if (std::strstr(l, "mag_0")) {
            c.mag0.clear();
            ok = values(l, c.mag0, 3);
        } else if (std::strstr(l, "acc_0")) {
            c.acc0.clear();
            ok = values(l, c.acc0, 3);
        } else if (std::strstr(l, "Acc_1")) {
            ok = values(l, c.acc1, 3);
        } else if (std::strstr(l, "Mag_1")) {
            ok = values(l, c.mag1, 3);
        } else if (std::strstr(l, "q_gyro")) {
            std::vector<double> tmp;  // side channel, not a filter input
            ok = values(l, tmp, -1);
        } else if (std::strstr(l, "gyro")) {
            ok = values(l, c.gyro, 3);
        } else if (std::strchr(l, 'T')) {
            std::vector<double> tmp;
            ok = values(l, tmp, -1) && !tmp.empty();
            if (ok) c.T.push_back(tmp[0]);
        }  // Wahba_quart / X_k: logged side channels, not inputs
        if (!ok) {
            status = pekf::set_error(PEKF_ERR_INVALID, "%s:%lld: cannot parse '%.60s'", path, (long long)lineno, l);
            break;
        }
    }
    std::free(buf);
    std::fclose(f);
    return status;
}

int validate(const char *path, const LogColumns &c, int64_t *n) {
    const int64_t nrec = (int64_t)c.acc1.size() / 3;
    if (c.acc0.size() != 3 || c.mag0.size() != 3)
        return pekf::set_error(PEKF_ERR_INVALID, "%s: missing acc_0 / mag_0 line", path);
    if ((int64_t)c.gyro.size() / 3 < nrec || (int64_t)c.mag1.size() / 3 < nrec || (int64_t)c.T.size() < nrec + 1)
        return pekf::set_error(PEKF_ERR_INVALID, "%s: %lld Acc_1 records but %zu gyro, %zu Mag_1, %zu T lines",
                               path, (long long)nrec, c.gyro.size() / 3, c.mag1.size() / 3, c.T.size());
    *n = nrec;
    return PEKF_OK;
}

}  // namespace

extern "C" {

int pekf_log_scan(const char *path, int64_t *n_records) {
    if (!path || !n_records) return pekf::set_error(PEKF_ERR_INVALID, "null pointer");
    LogColumns c;
    if (int st = parse(path, c)) return st;
    return validate(path, c, n_records);
}

int pekf_log_read_ext(const char *path, int64_t n_records, float *gyro, float *acc, float *mag, uint32_t *dtw,
                      double *dt_ext, int64_t *n_escaped, double *acc0, double *mag0, double *t0) {
    if (!path || !gyro || !acc || !mag || !dtw || !acc0 || !mag0)
        return pekf::set_error(PEKF_ERR_INVALID, "null pointer");
    LogColumns c;
    if (int st = parse(path, c)) return st;
    int64_t n = 0;
    if (int st = validate(path, c, &n)) return st;
    if (n_records > n)
        return pekf::set_error(PEKF_ERR_INVALID, "%s has %lld records, %lld requested", path, (long long)n,
                               (long long)n_records);
    for (int k = 0; k < 3; ++k) {
        acc0[k] = c.acc0[k];
        mag0[k] = c.mag0[k];
    }
    if (t0) *t0 = c.T[0];
    int64_t escaped = 0;
    for (int64_t i = 0; i < n_records; ++i) {
        for (int k = 0; k < 3; ++k) {
            gyro[3 * i + k] = (float)c.gyro[3 * i + k];
            acc[3 * i + k] = (float)c.acc1[3 * i + k];
            mag[3 * i + k] = (float)c.mag1[3 * i + k];
        }
        // T - previousT exactly as the reference forms it (ExtendedKalmanFilter.py:62): float64 difference
        const double dt = c.T[i + 1] - c.T[i];
        const bool fits = dt >= 0.0 && dt < (double)PEKF_DT_ESCAPE && dt == std::floor(dt);
        if (dt_ext) dt_ext[i] = fits ? 0.0 : dt;
        if (fits) {
            dtw[i] = (uint32_t)dt;
        } else if (dt_ext) {
            dtw[i] = PEKF_DT_ESCAPE;  // the record's dt is dt_ext[i]
            ++escaped;
        } else {
            return pekf::set_error(PEKF_ERR_INVALID,
                                   "%s: record %lld has dt = %.17g ns, not an integer in [0, 2^31 - 1) "
                                   "(use pekf_log_read_ext: the dt side plane takes any gap)",
                                   path, (long long)i, dt);
        }
    }
    if (n_escaped) *n_escaped = escaped;
    return PEKF_OK;
}

int pekf_log_read64(const char *path, int64_t n_records, double *gyro, double *acc, double *mag, double *dt_ns,
                    double *acc0, double *mag0, double *t0) {
    if (!path || !gyro || !acc || !mag || !dt_ns || !acc0 || !mag0)
        return pekf::set_error(PEKF_ERR_INVALID, "null pointer");
    LogColumns c;
    if (int st = parse(path, c)) return st;
    int64_t n = 0;
    if (int st = validate(path, c, &n)) return st;
    if (n_records > n)
        return pekf::set_error(PEKF_ERR_INVALID, "%s has %lld records, %lld requested", path, (long long)n,
                               (long long)n_records);
    for (int k = 0; k < 3; ++k) {
        acc0[k] = c.acc0[k];
        mag0[k] = c.mag0[k];
    }
    if (t0) *t0 = c.T[0];
    for (int64_t i = 0; i < n_records; ++i) {
        for (int k = 0; k < 3; ++k) {
            gyro[3 * i + k] = c.gyro[3 * i + k];
            acc[3 * i + k] = c.acc1[3 * i + k];
            mag[3 * i + k] = c.mag1[3 * i + k];
        }
        dt_ns[i] = c.T[i + 1] - c.T[i];  // T - previousT as the reference forms it (ExtendedKalmanFilter.py:62)
    }
    return PEKF_OK;
}

int pekf_log_read(const char *path, int64_t n_records, float *gyro, float *acc, float *mag, uint32_t *dtw,
                  double *acc0, double *mag0, double *t0) {
    return pekf_log_read_ext(path, n_records, gyro, acc, mag, dtw, nullptr, nullptr, acc0, mag0, t0);
}

int pekf_log_write(const char *path, int64_t n_records, const int64_t *t_ns, const double *gyro, const double *acc,
                   const double *mag, const double *acc0, const double *mag0, const double *q_gyro, const double *x_k,
                   const double *wahba) {
    if (n_records < 0) return pekf::set_error(PEKF_ERR_INVALID, "negative size");
    if (!path || !t_ns || !acc0 || !mag0 || (n_records > 0 && (!gyro || !acc || !mag)))
        return pekf::set_error(PEKF_ERR_INVALID, "null pointer");
    FILE *f = std::fopen(path, "w");
    if (!f) return pekf::set_error(PEKF_ERR_INVALID, "cannot open log '%s': %s", path, std::strerror(errno));
    // std::to_string is "%f" / "%lld" in the server's "C" locale, whatever this process has set
    const locale_t prev = uselocale(pekf::c_locale());
    static const double kZero4[4] = {0.0, 0.0, 0.0, 0.0};  // an absent side channel is written as zeros
    auto vec = [&](const char *tag, const double *v, int n) {
        std::fprintf(f, "%s : ", tag);
        for (int k = 0; k < n; ++k) std::fprintf(f, k ? ",%f" : "%f", v[k]);
        std::fputc('\n', f);
    };
    vec("mag_0", mag0, 3);                                           // set_mag_0 (:26-29)
    vec("acc_0", acc0, 3);                                           // set_acc_0 (:30-33)
    std::fputs("q_gyro : 1.0, 0.0, 0.0, 0.0\nX_k : 1.0, 0.0, 0.0, 0.0\nWahba_quart : 1.0, 0.0, 0.0, 0.0\n",
               f);                                                   // compute_initial_params (:55-67)
    for (int64_t i = 0; i < n_records; ++i) {
        vec("gyro", gyro + 3 * i, 3);                                // SetAngularVelocity (:265-277)
        if (i == 0) std::fprintf(f, "T : %lld\n", (long long)t_ns[0]);  // Prediction's first call (:136-141)
        std::fprintf(f, "T : %lld\n", (long long)t_ns[i + 1]);          // (:150-151)
        vec("q_gyro", q_gyro ? q_gyro + 4 * i : kZero4, 4);          // (:152-153)
        vec("Mag_1", mag + 3 * i, 3);                                // SetMagnetometerMeasurements (:279-290)
        vec("Acc_1", acc + 3 * i, 3);                                // SetAccelerometerMeasurements (:292-303)
        vec("X_k", x_k ? x_k + 4 * i : kZero4, 4);                   // Correction (:180-183)
        vec("Wahba_quart", wahba ? wahba + 4 * i : kZero4, 4);
    }
    uselocale(prev);
    const bool bad = std::ferror(f) != 0;
    if (std::fclose(f) != 0 || bad) return pekf::set_error(PEKF_ERR_INVALID, "cannot write log '%s'", path);
    return PEKF_OK;
}

}  // extern "C"
