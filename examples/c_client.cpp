// c_client.cpp -- a C++ caller of the filter handle (include/pekf.h), no Python involved: B
// filters created from their reference vectors, fed one record each per pekf_filter_update
// (main_file.py:42-45 for every filter), then a resident-window launch through pekf_filter_run.
//
// usage: c_client <inputs.bin> [outputs.txt]   (int64 B, N, W; f64 acc0[B*3], mag0[B*3]; per update
//        i < N: f64 gyro[B*3], acc[B*3], mag[B*3], int64 t_ns[B]; f32 planes gd[W*B*4], am[W*B*4],
//        my[W*B*2]).  Writes the quaternions after the N updates and after the window, one filter
//        per line (stdout by default).
// tests/test_c_client.py writes the inputs, runs this on the GPU and compares with the same
// sequence through the Python engine, bit for bit.  It loads the client as a shared library
// (pekf_example_run) rather than starting a process from the GPU-initialised test process.
//
// build: g++ -O2 -std=c++17 examples/c_client.cpp -Iinclude -Lposeestimationkf_amd -lpekf
//        -Wl,-rpath,$PWD/poseestimationkf_amd -o build/c_client
//        (add -shared -fPIC -DPEKF_EXAMPLE_LIBRARY for the library form)
#include <cstdint>
#include <cstdio>
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

template <class T>
static bool get(std::FILE *f, std::vector<T> &v, size_t n) {
    v.resize(n);
    return std::fread(v.data(), sizeof(T), n, f) == n;
}

static void print(std::FILE *o, const std::vector<double> &X, int64_t B) {
    for (int64_t b = 0; b < B; ++b)
        std::fprintf(o, "%.17g %.17g %.17g %.17g\n", X[4 * b], X[4 * b + 1], X[4 * b + 2], X[4 * b + 3]);
}

static int run(const char *inputs, std::FILE *o) {
    std::FILE *in = std::fopen(inputs, "rb");
    if (!in) return 2;
    int64_t hdr[3];
    if (std::fread(hdr, 8, 3, in) != 3) return 2;
    const int64_t B = hdr[0], N = hdr[1], W = hdr[2];
    std::vector<double> acc0, mag0;
    if (!get(in, acc0, 3 * B) || !get(in, mag0, 3 * B)) return 2;

    pekf_filter *f = nullptr;
    CHECK(pekf_filter_create(B, acc0.data(), mag0.data(), 1.0, 0.1, nullptr, PEKF_RUN_STATE_SOA, &f));
    std::vector<double> gyro, acc, mag, X(4 * B);
    std::vector<int64_t> t;
    for (int64_t i = 0; i < N; ++i) {
        if (!get(in, gyro, 3 * B) || !get(in, acc, 3 * B) || !get(in, mag, 3 * B) || !get(in, t, B)) return 2;
        CHECK(pekf_filter_update(f, gyro.data(), t.data(), acc.data(), mag.data(), nullptr, X.data()));
    }
    print(o, X, B);

    std::vector<float> gd, am, my;
    if (!get(in, gd, 4 * W * B) || !get(in, am, 4 * W * B) || !get(in, my, 2 * W * B)) return 2;
    std::fclose(in);
    void *dgd, *dam, *dmy;
    CHECK(pekf_malloc(&dgd, gd.size() * 4));
    CHECK(pekf_malloc(&dam, am.size() * 4));
    CHECK(pekf_malloc(&dmy, my.size() * 4));
    CHECK(pekf_memcpy_h2d(dgd, gd.data(), gd.size() * 4, nullptr));
    CHECK(pekf_memcpy_h2d(dam, am.data(), am.size() * 4, nullptr));
    CHECK(pekf_memcpy_h2d(dmy, my.data(), my.size() * 4, nullptr));
    CHECK(pekf_filter_run(f, W, W, 0, dgd, dam, dmy, nullptr, nullptr, nullptr));
    CHECK(pekf_device_sync());
    std::vector<double> P(16 * B);
    CHECK(pekf_filter_get_state(f, X.data(), P.data()));
    print(o, X, B);
    CHECK(pekf_free(dgd));
    CHECK(pekf_free(dam));
    CHECK(pekf_free(dmy));
    CHECK(pekf_filter_destroy(f));
    return 0;
}

#ifdef PEKF_EXAMPLE_LIBRARY
extern "C" int pekf_example_run(const char *inputs, const char *outputs) {
    std::FILE *o = std::fopen(outputs, "w");
    if (!o) return 2;
    const int st = run(inputs, o);
    std::fclose(o);
    return st;
}
#else
int main(int argc, char **argv) {
    if (argc < 2) return 2;
    std::FILE *o = argc > 2 ? std::fopen(argv[2], "w") : stdout;
    if (!o) return 2;
    const int st = run(argv[1], o);
    if (o != stdout) std::fclose(o);
    return st;
}
#endif
