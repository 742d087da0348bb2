// pekf_internal.hpp -- shared host-side plumbing of libpekf.so (error state, HIP checks,
// the pinned/device staging workspace used by the host-pointer entry points).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <initializer_list>

#include "../../include/pekf.h"

namespace pekf {

int set_error(int code, const char *fmt, ...);
int hip_fail(hipError_t e, const char *what);
int require_device();

#define PEKF_HIP(call)                                                   \
    do {                                                                 \
        hipError_t e_ = (call);                                          \
        if (e_ != hipSuccess) return ::pekf::hip_fail(e_, #call);        \
    } while (0)

#define PEKF_CHECK_ARG(cond, msg)                                        \
    do {                                                                 \
        if (!(cond)) return ::pekf::set_error(PEKF_ERR_INVALID, "%s", msg); \
    } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned grid_for(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

// One record of the stream as it sits in the three planes (include/pekf.h, pekf_run_dev)
struct Rec {
    float4 gd;  // gx, gy, gz, bits(dt word)
    float4 am;  // ax, ay, az, mx
    float2 my;  // my, mz
};
// The FP64 record (pekf_run_rec64_dev's planes; pekf_frontend_ext_dev's output with FP64 events)
struct Rec64 {
    double4 gd;  // gx, gy, gz, dt_ns
    double4 am;  // ax, ay, az, mx
    double2 my;  // my, mz
};

// Host-pointer calls: inputs are packed into one coherent, mapped pinned buffer.  Small calls
// (<= kZeroCopyMaxBytes of inputs + outputs, e.g. the n = 1 calls of main_file.py) run
// zero-copy: the kernel reads and writes that buffer over PCIe, so a call is one launch and one
// synchronisation.  Larger calls copy it to device memory once each way.
constexpr size_t kZeroCopyMaxBytes = (size_t)1 << 16;
struct HostArg {
    const void *ptr;
    size_t bytes;
};
struct HostOut {
    void *ptr;
    size_t bytes;
};

// Completion signal of a one-block per-call launch (the zero-copy calls): every thread makes its
// writes visible system-wide, then one thread stores `seq` into a host-visible flag that the
// host polls instead of calling hipStreamSynchronize (measured on MI355X: 7.8 vs 12.4 us per
// round trip, scripts/sync_probe.hip).  flag == nullptr: no signal (device-pointer calls).
struct Done {
    unsigned *flag;
    unsigned seq;
    __device__ __forceinline__ void signal() const {
        if (!flag) return;  // uniform: a kernel argument
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
};
constexpr Done kNoSignal = {nullptr, 0u};

class Staging {
  public:
    // Packs `ins` into device memory; returns device addresses for ins and outs.
    // The caller enqueues its kernel on stream() between stage_in() and stage_out(), passing
    // done(grid blocks) to it so that a zero-copy one-block launch signals its completion.
    int stage_in(std::initializer_list<HostArg> ins, std::initializer_list<size_t> out_bytes,
                 void **dev_in, void **dev_out);
    int stage_out(std::initializer_list<HostOut> outs, void *const *dev_out);
    Done done(unsigned blocks);
    hipStream_t stream() const { return stream_; }
    ~Staging();

    static Staging &get();  // per calling thread, per current device
  private:
    int reserve(size_t bytes);
    int wait();
    hipStream_t stream_ = nullptr;
    char *dev_ = nullptr;
    char *host_ = nullptr;
    char *host_dev_ = nullptr;  // device address of host_
    unsigned *flag_ = nullptr;      // coherent pinned completion flag (host address)
    unsigned *flag_dev_ = nullptr;  // its device address
    unsigned seq_ = 0;
    bool signalled_ = false;        // the launch since stage_in() signals through flag_
    size_t cap_ = 0;
    size_t in_bytes_ = 0;
    bool zero_copy_ = false;
    int device_ = -1;
};

// Stops the resident per-call service kernel (pekf_percall.hip) of every device, e.g. before a
// device-wide synchronisation, which would otherwise wait for its idle limit.
void service_quiesce_all();

// Filter-handle update kernel launcher (pekf_run.hip): one FP64 record per filter.
int launch_update(int64_t batch, const double *gyro, const int64_t *t_ns, const double *acc, const double *mag,
                  const uint8_t *missing, const double *refs, int64_t *prev_t, double *X, double *P, double q,
                  double r, double *x_out, uint32_t flags, hipStream_t stream);

// Multi-record fused launches (pekf_run_multi.hip, compiled with the max-ILP scheduler): every
// k_run<TRAJ, MIXED, SOA, COUNTS, ONE = false> variant; arguments checked by pekf_run_dev.
int launch_run_multi(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const float4 *gd,
                     const float4 *am, const float2 *my, const double *dtx, const double *refs, double *X,
                     double *P, double q, double r, double *traj, const int32_t *counts, bool mixed, bool soa,
                     hipStream_t stream);

}  // namespace pekf
