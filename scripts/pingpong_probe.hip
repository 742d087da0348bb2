// pingpong_probe.hip -- diagnostic: host <-> resident-kernel round trip through coherent mapped
// pinned memory (the host posts a request word, one resident lane polls it, answers with a
// response word), against the launch-per-call round trip of sync_probe.hip.
// The resident kernel always ends: it exits after `n` requests or after an idle period measured
// on the constant-rate wall clock.
// build: hipcc --offload-arch=gfx950 -O2 scripts/pingpong_probe.hip -o build/pingpong_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                           \
        }                                                                       \
    } while (0)

__global__ void k_resident(unsigned *req, unsigned *resp, const double *in, double *out, unsigned n,
                           unsigned long long idle_ticks, int sleep) {
    if (threadIdx.x != 0) return;
    unsigned last = 0;
    unsigned long long t0 = wall_clock64();
    while (last < n) {
        const unsigned r = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (r != last) {
            double v[4];
            for (int k = 0; k < 4; ++k) v[k] = __hip_atomic_load(in + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (int k = 0; k < 4; ++k) __hip_atomic_store(out + k, v[k] * 2.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(resp, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            last = r;
            t0 = wall_clock64();
        } else {
            if (wall_clock64() - t0 > idle_ticks) break;
            if (sleep) __builtin_amdgcn_s_sleep(1);
        }
    }
}

// The same responder with K polls in flight: a new load of the request word is issued every
// `gap` s_sleep units while the K - 1 older ones are still travelling, so a posted request is seen
// by the next poll to return rather than by one issued after it lands.
template <int K>
__global__ void k_resident_pipelined(unsigned *req, unsigned *resp, const double *in, double *out, unsigned n,
                                     unsigned long long idle_ticks) {
    if (threadIdx.x != 0) return;
    unsigned last = 0;
    unsigned long long t0 = wall_clock64();
    unsigned r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        r[k] = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(4);
    }
    while (last < n) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned v = r[k];  // the oldest poll in flight
            r[k] = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v != last && last < n) {
                __atomic_thread_fence(__ATOMIC_ACQUIRE);
                double w[4];
                for (int j = 0; j < 4; ++j) w[j] = __hip_atomic_load(in + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                for (int j = 0; j < 4; ++j) __hip_atomic_store(out + j, w[j] * 2.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(resp, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                last = v;
                t0 = wall_clock64();
            }
            __builtin_amdgcn_s_sleep(4);
        }
        if (wall_clock64() - t0 > idle_ticks) break;
    }
}

template <int K>
int run_pipelined(unsigned *dreq, unsigned *dresp, volatile unsigned *hreq, volatile unsigned *hresp, double *din,
                  double *dout, hipStream_t s, unsigned long long idle) {
    const unsigned N = 3000;
    *hreq = 0;
    *hresp = 0;
    hipLaunchKernelGGL(k_resident_pipelined<K>, dim3(1), dim3(64), 0, s, dreq, dresp, din, dout, N, idle);
    CK(hipGetLastError());
    std::vector<double> us;
    bool lost = false;
    for (unsigned i = 1; i <= N && !lost; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(hreq, i, __ATOMIC_RELEASE);
        while (__atomic_load_n(hresp, __ATOMIC_ACQUIRE) != i) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.1) {
                lost = true;
                break;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(s));
    if (lost) {
        std::printf("pipelined K=%d: no response within 100 ms\n", K);
        return 0;
    }
    std::vector<double> tail(us.begin() + 500, us.end());
    std::sort(tail.begin(), tail.end());
    std::printf("resident round trip, %d polls in flight: median %.2f us  p10 %.2f  p90 %.2f  p99 %.2f\n", K,
                tail[tail.size() / 2], tail[tail.size() / 10], tail[tail.size() * 9 / 10], tail[tail.size() * 99 / 100]);
    return 0;
}

// NW polling waves, staggered: wave k starts k * gap sleep units late, so a posted request is first
// seen by whichever wave's poll lands next; the wave that sees it claims it with an atomic CAS on a
// device-memory word (the others skip it) and answers.
__global__ void k_resident_multi(unsigned *req, unsigned *resp, unsigned *claim, const double *in, double *out,
                                 unsigned n, unsigned long long idle_ticks, int gap) {
    if (threadIdx.x % 64 != 0) return;
    const int wave = threadIdx.x / 64;
    for (int k = 0; k < wave * gap; ++k) __builtin_amdgcn_s_sleep(1);
    unsigned long long t0 = wall_clock64();
    for (;;) {
        const unsigned r = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned c = __hip_atomic_load(claim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c >= n) break;
        if (r != c) {
            unsigned expect = c;
            if (__hip_atomic_compare_exchange_strong(claim, &expect, r, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                double w[4];
                for (int j = 0; j < 4; ++j) w[j] = __hip_atomic_load(in + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                for (int j = 0; j < 4; ++j) __hip_atomic_store(out + j, w[j] * 2.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(resp, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            t0 = wall_clock64();
        } else if (wall_clock64() - t0 > idle_ticks) {
            break;
        }
    }
}

int run_multi(int nw, int gap, unsigned *dreq, unsigned *dresp, volatile unsigned *hreq, volatile unsigned *hresp,
              double *din, double *dout, hipStream_t s, unsigned long long idle) {
    const unsigned N = 3000;
    unsigned *claim;
    CK(hipMalloc(&claim, 4));
    CK(hipMemset(claim, 0, 4));
    *hreq = 0;
    *hresp = 0;
    hipLaunchKernelGGL(k_resident_multi, dim3(1), dim3(64 * nw), 0, s, dreq, dresp, claim, din, dout, N, idle, gap);
    CK(hipGetLastError());
    std::vector<double> us;
    bool lost = false;
    for (unsigned i = 1; i <= N && !lost; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(hreq, i, __ATOMIC_RELEASE);
        while (__atomic_load_n(hresp, __ATOMIC_ACQUIRE) != i) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.1) {
                lost = true;
                break;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CK(hipStreamSynchronize(s));
    CK(hipFree(claim));
    if (lost) {
        std::printf("%d waves gap %d: no response within 100 ms\n", nw, gap);
        return 0;
    }
    std::vector<double> tail(us.begin() + 500, us.end());
    std::sort(tail.begin(), tail.end());
    std::printf("resident round trip, %d staggered polling waves (gap %d): median %.2f us  p10 %.2f  p90 %.2f  p99 %.2f\n",
                nw, gap, tail[tail.size() / 2], tail[tail.size() / 10], tail[tail.size() * 9 / 10],
                tail[tail.size() * 99 / 100]);
    return 0;
}

int main() {
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    std::printf("wall clock rate: %d kHz\n", rate_khz);
    char *host, *hdev;
    CK(hipHostMalloc(&host, 8192, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&hdev), host, 0));
    volatile unsigned *hreq = reinterpret_cast<volatile unsigned *>(host);
    volatile unsigned *hresp = reinterpret_cast<volatile unsigned *>(host + 4096);
    unsigned *dreq = reinterpret_cast<unsigned *>(hdev), *dresp = reinterpret_cast<unsigned *>(hdev + 4096);
    double *din = reinterpret_cast<double *>(hdev + 256), *dout = reinterpret_cast<double *>(hdev + 4096 + 256);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned long long idle = (unsigned long long)rate_khz * 200;  // 200 ms
    for (int sleep = 0; sleep < 2; ++sleep) {
        const unsigned N = 3000;
        *hreq = 0;
        *hresp = 0;
        hipLaunchKernelGGL(k_resident, dim3(1), dim3(64), 0, s, dreq, dresp, din, dout, N, idle, sleep);
        CK(hipGetLastError());
        std::vector<double> us;
        bool lost = false;
        for (unsigned i = 1; i <= N && !lost; ++i) {
            auto t0 = std::chrono::steady_clock::now();
            __atomic_store_n(hreq, i, __ATOMIC_RELEASE);
            while (__atomic_load_n(hresp, __ATOMIC_ACQUIRE) != i) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.1) {
                    lost = true;
                    break;
                }
            }
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        CK(hipStreamSynchronize(s));
        if (lost) {
            std::printf("sleep=%d: no response within 100 ms\n", sleep);
            continue;
        }
        std::vector<double> tail(us.begin() + 500, us.end());
        std::sort(tail.begin(), tail.end());
        std::printf("resident round trip (s_sleep %d): median %.2f us  p10 %.2f  p90 %.2f  p99 %.2f\n", sleep,
                    tail[tail.size() / 2], tail[tail.size() / 10], tail[tail.size() * 9 / 10],
                    tail[tail.size() * 99 / 100]);
    }
    run_multi(1, 0, dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_multi(2, 8, dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_multi(4, 4, dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_multi(8, 2, dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_multi(16, 1, dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_pipelined<2>(dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_pipelined<4>(dreq, dresp, hreq, hresp, din, dout, s, idle);
    run_pipelined<8>(dreq, dresp, hreq, hresp, din, dout, s, idle);
    // Variant: the request word in fine-grained device memory written by the CPU through the
    // BAR mapping (if the platform maps it), the response in pinned host memory.
    unsigned *vreq = nullptr;
    if (hipExtMallocWithFlags(reinterpret_cast<void **>(&vreq), 4096, hipDeviceMallocFinegrained) != hipSuccess) {
        std::printf("fine-grained device memory: allocation failed\n");
        return 0;
    }
    hipPointerAttribute_t attr;
    CK(hipPointerGetAttributes(&attr, vreq));
    std::printf("fine-grained device memory: device ptr %p host ptr %p\n", attr.devicePointer, attr.hostPointer);
    if (!attr.hostPointer) return 0;
    volatile unsigned *hv = reinterpret_cast<volatile unsigned *>(attr.hostPointer);
    for (int sleep = 0; sleep < 2; ++sleep) {
        const unsigned N = 3000;
        *hv = 0;
        *hresp = 0;
        hipLaunchKernelGGL(k_resident, dim3(1), dim3(64), 0, s, vreq, dresp, din, dout, N, idle, sleep);
        CK(hipGetLastError());
        std::vector<double> us;
        bool lost = false;
        for (unsigned i = 1; i <= N && !lost; ++i) {
            auto t0 = std::chrono::steady_clock::now();
            __atomic_store_n(hv, i, __ATOMIC_RELEASE);
            while (__atomic_load_n(hresp, __ATOMIC_ACQUIRE) != i) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 0.1) {
                    lost = true;
                    break;
                }
            }
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        CK(hipStreamSynchronize(s));
        if (lost) {
            std::printf("VRAM request, sleep=%d: no response within 100 ms\n", sleep);
            continue;
        }
        std::vector<double> tail(us.begin() + 500, us.end());
        std::sort(tail.begin(), tail.end());
        std::printf("VRAM request round trip (s_sleep %d): median %.2f us  p10 %.2f  p90 %.2f  p99 %.2f\n", sleep,
                    tail[tail.size() / 2], tail[tail.size() / 10], tail[tail.size() * 9 / 10],
                    tail[tail.size() * 99 / 100]);
    }
    return 0;
}
