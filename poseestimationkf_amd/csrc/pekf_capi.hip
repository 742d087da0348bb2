// pekf_capi.hip -- host plumbing of the C ABI: error reporting, device / memory / stream /
// event helpers (so the Python host needs no PyTorch), and the per-thread staging
// workspace used by the host-pointer per-call entry points.
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "pekf_internal.hpp"

namespace pekf {

static thread_local char g_err[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_fail(hipError_t e, const char *what) {
    return set_error(e == hipErrorNoDevice ? PEKF_ERR_NODEVICE : PEKF_ERR_HIP, "%s: %s (%d)", what,
                     hipGetErrorString(e), (int)e);
}

int require_device() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return set_error(PEKF_ERR_NODEVICE,
                         "no HIP device visible (libpekf has no CPU path; run on an MI355X)");
    return PEKF_OK;
}

// ---------------------------------------------------------------------------------------------
Staging &Staging::get() {
    static thread_local Staging per_device[16];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
    Staging &s = per_device[dev];
    s.device_ = dev;
    return s;
}

Staging::~Staging() {
    // Runtime teardown order at process exit is not ours to control: leave the
    // (process-lifetime) buffers to the driver rather than calling into HIP here.
}

int Staging::reserve(size_t bytes) {
    if (!stream_) PEKF_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    if (!flag_) {
        PEKF_HIP(hipHostMalloc(reinterpret_cast<void **>(&flag_), 256, hipHostMallocMapped | hipHostMallocCoherent));
        PEKF_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&flag_dev_), flag_, 0));
        __atomic_store_n(flag_, seq_, __ATOMIC_RELAXED);
    }
    if (bytes <= cap_) return PEKF_OK;
    size_t cap = cap_ ? cap_ : (size_t)1 << 16;
    while (cap < bytes) cap *= 2;
    if (dev_) (void)hipFree(dev_);
    if (host_) (void)hipHostFree(host_);
    dev_ = nullptr;
    host_ = nullptr;
    host_dev_ = nullptr;
    cap_ = 0;
    PEKF_HIP(hipMalloc(&dev_, cap));
    // coherent, mapped pinned memory: small calls run zero-copy (the kernel reads its inputs and
    // writes its outputs over PCIe), so a call costs one launch and one synchronisation
    PEKF_HIP(hipHostMalloc(&host_, cap, hipHostMallocMapped | hipHostMallocCoherent));
    PEKF_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&host_dev_), host_, 0));
    cap_ = cap;
    return PEKF_OK;
}

static inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

int Staging::stage_in(std::initializer_list<HostArg> ins, std::initializer_list<size_t> out_bytes,
                      void **dev_in, void **dev_out) {
    size_t total = 0;
    for (const HostArg &a : ins) total += align_up(a.bytes);
    size_t in_total = total;
    for (size_t b : out_bytes) total += align_up(b);
    if (int st = reserve(total)) return st;
    zero_copy_ = total <= kZeroCopyMaxBytes;
    char *base = zero_copy_ ? host_dev_ : dev_;
    size_t off = 0;
    int i = 0;
    for (const HostArg &a : ins) {
        if (a.bytes) std::memcpy(host_ + off, a.ptr, a.bytes);
        dev_in[i++] = base + off;
        off += align_up(a.bytes);
    }
    i = 0;
    for (size_t b : out_bytes) {
        dev_out[i++] = base + off;
        off += align_up(b);
    }
    in_bytes_ = in_total;
    signalled_ = false;
    if (!zero_copy_ && in_total) PEKF_HIP(hipMemcpyAsync(dev_, host_, in_total, hipMemcpyHostToDevice, stream_));
    return PEKF_OK;
}

Done Staging::done(unsigned blocks) {
    // only a zero-copy launch of ONE block can signal completion with one flag store
    if (!zero_copy_ || blocks != 1 || !flag_dev_) return kNoSignal;
    signalled_ = true;
    return Done{flag_dev_, ++seq_};
}

// Wait for the launch since stage_in(): spin on the completion flag when the kernel signals,
// falling back to hipStreamSynchronize (which also reports a faulted kernel) after 20 ms.
int Staging::wait() {
    if (signalled_) {
        const auto t0 = std::chrono::steady_clock::now();
        for (unsigned it = 0;; ++it) {
            if (__atomic_load_n(flag_, __ATOMIC_ACQUIRE) == seq_) return PEKF_OK;
            if ((it & 1023u) == 1023u &&
                std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20))
                break;
        }
    }
    PEKF_HIP(hipStreamSynchronize(stream_));
    return PEKF_OK;
}

int Staging::stage_out(std::initializer_list<HostOut> outs, void *const *dev_out) {
    // outputs were laid out contiguously right after the inputs: one D2H for all of them
    size_t total = 0;
    for (const HostOut &o : outs) total += align_up(o.bytes);
    if (total && !zero_copy_) {
        PEKF_HIP(hipMemcpyAsync(host_ + in_bytes_, dev_out[0], total, hipMemcpyDeviceToHost, stream_));
    }
    if (int st = wait()) return st;
    size_t off = in_bytes_;
    for (const HostOut &o : outs) {
        if (o.bytes) std::memcpy(o.ptr, host_ + off, o.bytes);
        off += align_up(o.bytes);
    }
    return PEKF_OK;
}

}  // namespace pekf

using namespace pekf;

extern "C" {

int pekf_abi_version(void) { return PEKF_ABI_VERSION; }
const char *pekf_last_error(void) { return g_err; }

int pekf_device_count(int *count) {
    PEKF_CHECK_ARG(count, "count is NULL");
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e == hipErrorNoDevice) {
        *count = 0;
        return PEKF_OK;
    }
    PEKF_HIP(e);
    return PEKF_OK;
}

int pekf_set_device(int device) {
    if (int st = require_device()) return st;
    PEKF_HIP(hipSetDevice(device));
    return PEKF_OK;
}

int pekf_get_device(int *device) {
    PEKF_CHECK_ARG(device, "device is NULL");
    if (int st = require_device()) return st;
    PEKF_HIP(hipGetDevice(device));
    return PEKF_OK;
}

int pekf_device_name(int device, char *buf, int buflen) {
    PEKF_CHECK_ARG(buf && buflen > 0, "bad buffer");
    if (int st = require_device()) return st;
    hipDeviceProp_t p;
    PEKF_HIP(hipGetDeviceProperties(&p, device));
    snprintf(buf, (size_t)buflen, "%s", p.gcnArchName);
    return PEKF_OK;
}

int pekf_malloc(void **dptr, size_t bytes) {
    PEKF_CHECK_ARG(dptr, "dptr is NULL");
    if (int st = require_device()) return st;
    PEKF_HIP(hipMalloc(dptr, bytes ? bytes : 1));
    return PEKF_OK;
}

int pekf_free(void *dptr) {
    if (dptr) PEKF_HIP(hipFree(dptr));
    return PEKF_OK;
}

int pekf_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    PEKF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, as_stream(stream)));
    PEKF_HIP(hipStreamSynchronize(as_stream(stream)));
    return PEKF_OK;
}

int pekf_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    PEKF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, as_stream(stream)));
    PEKF_HIP(hipStreamSynchronize(as_stream(stream)));
    return PEKF_OK;
}

int pekf_memcpy_d2d(void *dst, const void *src, size_t bytes, void *stream) {
    PEKF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, as_stream(stream)));
    return PEKF_OK;
}

int pekf_memset(void *dst, int value, size_t bytes, void *stream) {
    PEKF_HIP(hipMemsetAsync(dst, value, bytes, as_stream(stream)));
    return PEKF_OK;
}

int pekf_stream_create(void **stream) {
    PEKF_CHECK_ARG(stream, "stream is NULL");
    if (int st = require_device()) return st;
    hipStream_t s;
    PEKF_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return PEKF_OK;
}

int pekf_stream_destroy(void *stream) {
    if (stream) PEKF_HIP(hipStreamDestroy(as_stream(stream)));
    return PEKF_OK;
}

int pekf_stream_sync(void *stream) {
    PEKF_HIP(hipStreamSynchronize(as_stream(stream)));
    return PEKF_OK;
}

int pekf_device_sync(void) {
    service_quiesce_all();
    PEKF_HIP(hipDeviceSynchronize());
    return PEKF_OK;
}

int pekf_event_create(void **event) {
    PEKF_CHECK_ARG(event, "event is NULL");
    if (int st = require_device()) return st;
    hipEvent_t e;
    PEKF_HIP(hipEventCreate(&e));
    *event = e;
    return PEKF_OK;
}

int pekf_event_destroy(void *event) {
    if (event) PEKF_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)));
    return PEKF_OK;
}

int pekf_event_record(void *event, void *stream) {
    PEKF_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(event), as_stream(stream)));
    return PEKF_OK;
}

int pekf_event_sync(void *event) {
    PEKF_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(event)));
    return PEKF_OK;
}

int pekf_event_elapsed_ms(float *ms, void *start, void *stop) {
    PEKF_CHECK_ARG(ms, "ms is NULL");
    PEKF_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start),
                                 reinterpret_cast<hipEvent_t>(stop)));
    return PEKF_OK;
}

}  // extern "C"
