// wire_client.cpp -- the live server's per-client pipeline from the phone's wire text, in C++ over the
// C ABI (include/pekf.h), no Python involved: for K phones at once, each phone's text (the Android
// client's "#<phase>,<type>:<x>,<y>,<z>,t:<ns>" messages, ASC/MessageSender.java:217-233) is parsed
// as the server parses it (pekf_wire_parse: std::stod / std::stoll, KFS/Parser.cpp:12-26), packed into
// FP64 event planes (PEKF_EV_F64_EVENTS: the server's own doubles and times), and run through phase 2
// (pekf_frontend_init_ext_dev: the means of the first 100 samples, the time phase 3 starts from,
// Parser.cpp:36-58,84-140) and phase 3 fused with the filter (pekf_live_ext_dev: Parser.cpp:148-267,
// then Prediction + Correction per record).  Phase-1 messages (magnetometer calibration, a no-op in the
// reference) are skipped.
//
// usage: wire_client [--device] <out.txt> <phone0.txt> [phone1.txt ...]
//        writes one line per phone: records applied, then the final quaternion (%.17g).  --device: the
//        texts are cut into the server's 100-byte frames and parsed on the GPU (pekf_wire_events_dev)
//        into the same planes instead of by pekf_wire_parse on the host.
// tests/test_c_client.py runs the library form (pekf_wire_example_run_mode, both parses) on the GPU and
// compares with engine.run_session(..., events="f64") on wire.events_from_wire of the same texts, bit for
// bit.
//
// build: g++ -O2 -std=c++17 examples/wire_client.cpp -Iinclude -Lposeestimationkf_amd -lpekf
//        -Wl,-rpath,$PWD/poseestimationkf_amd -o build/wire_client
//        (add -shared -fPIC -DPEKF_EXAMPLE_LIBRARY for the library form)
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pekf.h"

#define CHECK(call)                                                                    \
    do {                                                                               \
        int st_ = (call);                                                              \
        if (st_) {                                                                     \
            std::fprintf(stderr, "%s failed: %d %s\n", #call, st_, pekf_last_error()); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

namespace {

struct Messages {
    std::vector<uint8_t> phase, type;
    std::vector<double> xyz;
    std::vector<int64_t> t;
};

bool read_text(const char *path, std::string &out) {
    std::FILE *f = std::fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
    std::fclose(f);
    return true;
}

int parse(const std::string &text, Messages &m) {
    int64_t n = 0;
    CHECK(pekf_wire_parse(text.data(), (int64_t)text.size(), 0, nullptr, nullptr, nullptr, nullptr, &n));
    m.phase.resize(n);
    m.type.resize(n);
    m.xyz.resize(3 * n);
    m.t.resize(n);
    CHECK(pekf_wire_parse(text.data(), (int64_t)text.size(), n, m.phase.data(), m.type.data(), m.xyz.data(),
                          m.t.data(), &n));
    return 0;
}

// One FP64 event {x, y, z, bits(t) | type} (PEKF_EV_F64_EVENTS); xyz = NULL: no message at all, w = the
// bits of -0.0 with type 3, which pads short streams.
void put_event(double *e, const double *xyz, int64_t t, unsigned type) {
    e[0] = xyz ? xyz[0] : 0.0;
    e[1] = xyz ? xyz[1] : 0.0;
    e[2] = xyz ? xyz[2] : 0.0;
    const double td = (double)t;
    uint64_t bits;
    std::memcpy(&bits, &td, 8);
    bits = xyz ? bits | type : 0x8000000000000003ull;
    std::memcpy(&e[3], &bits, 8);
}

// The phase-p messages of every phone as an [E][K] double4 plane on the device; E = the longest stream.
int planes(const std::vector<Messages> &ms, uint8_t p, void **dev, int64_t *E, std::vector<int64_t> *first_t) {
    const int64_t K = (int64_t)ms.size();
    std::vector<std::vector<int64_t>> idx(K);
    *E = 0;
    for (int64_t k = 0; k < K; ++k) {
        for (size_t i = 0; i < ms[k].phase.size(); ++i)
            if (ms[k].phase[i] == p) idx[k].push_back((int64_t)i);
        if ((int64_t)idx[k].size() > *E) *E = (int64_t)idx[k].size();
    }
    std::vector<double> ev(4 * (size_t)(*E > 0 ? *E : 1) * K);
    if (first_t) first_t->assign(K, 0);
    for (int64_t k = 0; k < K; ++k) {
        if (first_t && !idx[k].empty()) (*first_t)[k] = ms[k].t[idx[k][0]];
        for (int64_t e = 0; e < *E; ++e) {
            double *dst = &ev[4 * (e * K + k)];
            if (e < (int64_t)idx[k].size()) {
                const int64_t i = idx[k][e];
                // a sensor type other than 0 / 1 / 2 matches no sensor in the server's state machine
                // (KFS/Parser.cpp:148-219) but is a message (in phase 2 it moves the time, :36-62): type 3
                const unsigned ty = ms[k].type[i] <= 2 ? ms[k].type[i] : 3u;
                put_event(dst, &ms[k].xyz[3 * i], ms[k].t[i], ty);
            } else {
                put_event(dst, nullptr, 0, 3u);
            }
        }
    }
    CHECK(pekf_malloc(dev, ev.size() * 8));
    CHECK(pekf_memcpy_h2d(*dev, ev.data(), ev.size() * 8, nullptr));
    return 0;
}

// The device form: each phone's text cut into the server's 100-byte recv frames ([F][K][100] bytes, short
// streams padded with blank frames), parsed on the GPU into the same FP64 event planes
// (pekf_wire_events_dev); phase 2 starts from each phone's first phase-2 time, as above.
int device_planes(const std::vector<const char *> &paths, void **ev2, int64_t *E2, void **ev3, int64_t *E3,
                  void **d_ts) {
    const int64_t K = (int64_t)paths.size();
    std::vector<std::string> texts(K);
    int64_t F = 0;
    for (int64_t k = 0; k < K; ++k) {
        if (!read_text(paths[k], texts[k]) || texts[k].size() % 100) return 2;
        if ((int64_t)texts[k].size() / 100 > F) F = (int64_t)texts[k].size() / 100;
    }
    std::vector<char> frames((size_t)(F > 0 ? F : 1) * K * 100, ' ');
    for (int64_t k = 0; k < K; ++k)
        for (int64_t f = 0; f < (int64_t)texts[k].size() / 100; ++f)
            std::memcpy(&frames[(size_t)(f * K + k) * 100], texts[k].data() + f * 100, 100);
    void *d_frames, *d_n2, *d_n3, *d_err;
    CHECK(pekf_malloc(&d_frames, frames.size()));
    CHECK(pekf_memcpy_h2d(d_frames, frames.data(), frames.size(), nullptr));
    const int64_t rows = F > 0 ? F : 1;
    CHECK(pekf_malloc(ev2, 32 * rows * K));
    CHECK(pekf_malloc(ev3, 32 * rows * K));
    CHECK(pekf_malloc(d_ts, 8 * K));
    CHECK(pekf_malloc(&d_n2, 4 * K));
    CHECK(pekf_malloc(&d_n3, 4 * K));
    CHECK(pekf_malloc(&d_err, 4));
    const int zero = 0;
    CHECK(pekf_memcpy_h2d(d_err, &zero, 4, nullptr));
    CHECK(pekf_wire_events_dev(K, F, d_frames, F, F, *ev2, *ev3, (int64_t *)*d_ts, (int32_t *)d_n2, (int32_t *)d_n3,
                               nullptr, (int *)d_err, nullptr));
    std::vector<int32_t> n2(K), n3(K);
    int err = 0;
    CHECK(pekf_memcpy_d2h(n2.data(), d_n2, 4 * K, nullptr));
    CHECK(pekf_memcpy_d2h(n3.data(), d_n3, 4 * K, nullptr));
    CHECK(pekf_memcpy_d2h(&err, d_err, 4, nullptr));
    for (void *q : {d_frames, d_n2, d_n3, d_err}) CHECK(pekf_free(q));
    if (err) return 3;  // a frame the device parser does not take: use the host form
    *E2 = *E3 = 0;
    for (int64_t k = 0; k < K; ++k) {
        if (n2[k] > *E2) *E2 = n2[k];
        if (n3[k] > *E3) *E3 = n3[k];
    }
    return 0;
}

int run(const std::vector<const char *> &paths, std::FILE *o, bool device = false) {
    const int64_t K = (int64_t)paths.size();
    void *ev2 = nullptr, *ev3 = nullptr, *d_ts = nullptr;
    int64_t E2 = 0, E3 = 0;
    if (device) {
        if (int st = device_planes(paths, &ev2, &E2, &ev3, &E3, &d_ts)) return st;
    } else {
        std::vector<Messages> ms(K);
        for (int64_t k = 0; k < K; ++k) {
            std::string text;
            if (!read_text(paths[k], text)) return 2;
            if (int st = parse(text, ms[k])) return st;
        }
        std::vector<int64_t> t_start;
        if (int st = planes(ms, 2, &ev2, &E2, &t_start)) return st;
        if (int st = planes(ms, 3, &ev3, &E3, nullptr)) return st;
        CHECK(pekf_malloc(&d_ts, 8 * K));
        CHECK(pekf_memcpy_h2d(d_ts, t_start.data(), 8 * K, nullptr));
    }
    void *d_init, *d_tinit, *d_ready, *d_X, *d_P, *d_counts, *d_refs;
    CHECK(pekf_malloc(&d_init, 48 * K));
    CHECK(pekf_malloc(&d_tinit, 8 * K));
    CHECK(pekf_malloc(&d_ready, 4 * K));
    CHECK(pekf_malloc(&d_X, 32 * K));
    CHECK(pekf_malloc(&d_P, 128 * K));
    CHECK(pekf_malloc(&d_counts, 4 * K));
    CHECK(pekf_malloc(&d_refs, 48 * K));
    // phase 2: the means of each sensor's first 100 samples and the time phase 3 continues from
    CHECK(pekf_frontend_init_ext_dev(K, E2, ev2, (const int64_t *)d_ts, 100, (double *)d_init, (int64_t *)d_tinit,
                                     nullptr, (int32_t *)d_ready, PEKF_EV_F64_EVENTS, nullptr));
    // phase 3 fused with the filter, from X = [1,0,0,0], P = I (main_file.py:23,26), Q = I, R = 0.1 I
    CHECK(pekf_reset_state_dev(K, (double *)d_X, (double *)d_P, nullptr));
    CHECK(pekf_live_ext_dev(K, E3, ev3, (const double *)d_init, (const int64_t *)d_tinit, 0.1, (double *)d_X,
                            (double *)d_P, 1.0, 0.1, (int32_t *)d_counts, (double *)d_refs, PEKF_EV_F64_EVENTS, nullptr,
                            nullptr));
    CHECK(pekf_device_sync());
    std::vector<double> X(4 * K);
    std::vector<int32_t> counts(K);
    CHECK(pekf_memcpy_d2h(X.data(), d_X, 32 * K, nullptr));
    CHECK(pekf_memcpy_d2h(counts.data(), d_counts, 4 * K, nullptr));
    for (int64_t k = 0; k < K; ++k)
        std::fprintf(o, "%d %.17g %.17g %.17g %.17g\n", counts[k], X[4 * k], X[4 * k + 1], X[4 * k + 2], X[4 * k + 3]);
    for (void *p : {ev2, ev3, d_ts, d_init, d_tinit, d_ready, d_X, d_P, d_counts, d_refs}) CHECK(pekf_free(p));
    return 0;
}

}  // namespace

#ifdef PEKF_EXAMPLE_LIBRARY
// paths: phone text files separated by '\n'; device: parse on the GPU (pekf_wire_events_dev)
extern "C" int pekf_wire_example_run_mode(const char *paths, const char *outputs, int device) {
    std::vector<std::string> names;
    for (const char *p = paths; *p;) {
        const char *e = std::strchr(p, '\n');
        names.emplace_back(p, e ? (size_t)(e - p) : std::strlen(p));
        p = e ? e + 1 : p + std::strlen(p);
    }
    std::vector<const char *> v;
    for (const auto &n : names)
        if (!n.empty()) v.push_back(n.c_str());
    std::FILE *o = std::fopen(outputs, "w");
    if (!o) return 2;
    const int st = run(v, o, device != 0);
    std::fclose(o);
    return st;
}
extern "C" int pekf_wire_example_run(const char *paths, const char *outputs) {
    return pekf_wire_example_run_mode(paths, outputs, 0);
}
#else
int main(int argc, char **argv) {
    const bool device = argc > 1 && std::strcmp(argv[1], "--device") == 0;
    if (argc < 3 + device) return 2;
    std::FILE *o = std::fopen(argv[1 + device], "w");
    if (!o) return 2;
    const int st = run(std::vector<const char *>(argv + 2 + device, argv + argc), o, device);
    std::fclose(o);
    return st;
}
#endif
