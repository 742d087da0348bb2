// sync_probe.hip -- diagnostic: host-side round-trip latency of one tiny kernel launch that reads
// and writes coherent mapped pinned memory (the shape of a drop-in n = 1 call), under different
// ways of waiting for it.
// build: hipcc --offload-arch=gfx950 -O2 scripts/sync_probe.hip -o build/sync_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) (void)(x)

__global__ void k_tiny(const double *in, double *out) {
    if (threadIdx.x < 4) out[threadIdx.x] = in[threadIdx.x] * 2.0;
}

__global__ void k_tiny_flag(const double *in, double *out, volatile unsigned *flag, unsigned seq) {
    if (threadIdx.x < 4) out[threadIdx.x] = in[threadIdx.x] * 2.0;
    __threadfence_system();
    if (threadIdx.x == 0) *flag = seq;
}

template <class F>
void bench(const char *name, F fn) {
    for (int i = 0; i < 100; ++i) fn();
    std::vector<double> us;
    for (int i = 0; i < 1000; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        fn();
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(us.begin(), us.end());
    std::printf("%-44s median %6.1f us  p10 %6.1f  p90 %6.1f\n", name, us[500], us[100], us[900]);
}

int main(int argc, char **argv) {
    const bool spin = argc > 1;
    if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    char *host, *hdev;
    CK(hipHostMalloc(&host, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&hdev), host, 0));
    double *in = reinterpret_cast<double *>(hdev), *out = in + 8;
    volatile unsigned *hflag = reinterpret_cast<volatile unsigned *>(host + 1024);
    unsigned *dflag = reinterpret_cast<unsigned *>(hdev + 1024);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::printf("device flags: %s\n", spin ? "hipDeviceScheduleSpin" : "default");
    bench("launch + hipStreamSynchronize", [&] {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, in, out);
        CK(hipStreamSynchronize(s));
    });
    bench("launch + hipEventRecord + spin hipEventQuery", [&] {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, in, out);
        CK(hipEventRecord(ev, s));
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
    });
    unsigned seq = 0;
    bench("launch (kernel writes flag) + spin on flag", [&] {
        ++seq;
        hipLaunchKernelGGL(k_tiny_flag, dim3(1), dim3(64), 0, s, in, out, dflag, seq);
        while (*hflag != seq) {
        }
    });
    bench("launch only (no wait)", [&] { hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, in, out); });
    CK(hipStreamSynchronize(s));
    return 0;
}
