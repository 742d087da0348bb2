// percall_latency.cpp -- diagnostic: latency of the n = 1 host-pointer entry points (what the
// drop-in modules pay per main_file.py call) measured from C++, without Python / ctypes.
// build: g++ -O2 -std=c++17 scripts/percall_latency.cpp -Iinclude -Lposeestimationkf_amd \
//        -lpekf -Wl,-rpath,$PWD/poseestimationkf_amd -o build/percall_latency
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "pekf.h"

int main() {
    double gyro[3] = {0.1, -0.2, 0.3}, dt = 1e7, X[4] = {1, 0, 0, 0}, P[16] = {}, Q[9] = {}, R[16] = {};
    for (int i = 0; i < 4; ++i) { P[5 * i] = 1; R[5 * i] = 0.1; }
    for (int i = 0; i < 3; ++i) Q[4 * i] = 1;
    double z[4], Pm[16], K[16], Xo[4], Po[16];
    double acc[3] = {0, 0.1, 0.99}, mag[3] = {0.5, 0.01, -0.86}, a0[3] = {0, 0, 1}, m0[3] = {0.5, 0, -0.86};
    auto bench = [&](const char *name, auto fn) {
        for (int i = 0; i < 50; ++i) fn();
        std::vector<double> us;
        for (int i = 0; i < 500; ++i) {
            auto t0 = std::chrono::steady_clock::now();
            fn();
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(us.begin(), us.end());
        std::printf("%-16s median %.1f us  p10 %.1f  p90 %.1f\n", name, us[250], us[50], us[450]);
    };
    bench("pekf_predict", [&] { pekf_predict(1, gyro, &dt, X, P, Q, R, z, Pm, K); });
    bench("pekf_correct", [&] { pekf_correct(1, mag, acc, z, Pm, K, a0, m0, Xo, Po); });
    bench("pekf_rk4", [&] { pekf_rk4(1, X, &dt, gyro, z); });
    bench("pekf_device_sync", [&] { pekf_device_sync(); });
    return 0;
}
