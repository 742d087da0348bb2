// pekf_filter.hip -- the filter handle (include/pekf.h): B KalmanFilter objects
// (ExtendedKalmanFilter.py:6-15) with their state kept in device memory between calls.
//
// Host code only; the per-record kernel is k_update in pekf_run.hip (same ekf_record_step as the
// stream kernel) and the stream path is pekf_run_dev.
#include <cstring>
#include <vector>

#include "pekf_internal.hpp"

struct pekf_filter {
    int64_t batch = 0;
    double q = 1.0, r = 1.0;
    uint32_t flags = 0;
    int device = -1;
    double *X = nullptr;      // [batch][4] or SoA [4][batch]
    double *P = nullptr;      // [batch][16] or SoA [10][batch]
    double *refs = nullptr;   // [batch][6] = {acc0, mag0}
    int64_t *prev_t = nullptr;
    char *upd = nullptr;      // device staging of one host update (records in, X out)
    char *upd_host = nullptr; // pinned mirror of upd
    hipStream_t stream = nullptr;
};

namespace {

using namespace pekf;

constexpr uint32_t kFilterFlags = PEKF_RUN_MIXED_PRECISION | PEKF_RUN_STATE_SOA;

size_t p_bytes(const pekf_filter *f) { return (size_t)f->batch * ((f->flags & PEKF_RUN_STATE_SOA) ? 80 : 128); }

// Per-filter record bytes of one host update: gyro, acc, mag (3 f64 each), t (i64), missing (u8),
// X out (4 f64), each array 16 B aligned.
size_t align16(size_t n) { return (n + 15) & ~(size_t)15; }

struct UpdLayout {
    size_t gyro, t, acc, mag, miss, xout, total;
    explicit UpdLayout(int64_t B) {
        const size_t b = (size_t)B;
        gyro = 0;
        t = gyro + align16(24 * b);
        acc = t + align16(8 * b);
        mag = acc + align16(24 * b);
        miss = mag + align16(24 * b);
        xout = miss + align16(b);
        total = xout + align16(32 * b);
    }
};

int check_handle(const pekf_filter *f) {
    PEKF_CHECK_ARG(f != nullptr, "null filter handle");
    int dev = -1;
    PEKF_HIP(hipGetDevice(&dev));
    if (dev != f->device)
        return set_error(PEKF_ERR_INVALID, "filter handle belongs to device %d, current device is %d", f->device, dev);
    return PEKF_OK;
}

// AoS host state -> device state in the handle's layout (via a temporary AoS device copy for SoA).
int upload_state(pekf_filter *f, const double *X, const double *P) {
    const size_t B = (size_t)f->batch;
    if (!(f->flags & PEKF_RUN_STATE_SOA)) {
        if (X) PEKF_HIP(hipMemcpyAsync(f->X, X, 32 * B, hipMemcpyHostToDevice, f->stream));
        if (P) PEKF_HIP(hipMemcpyAsync(f->P, P, 128 * B, hipMemcpyHostToDevice, f->stream));
        PEKF_HIP(hipStreamSynchronize(f->stream));
        return PEKF_OK;
    }
    double *Xa = nullptr, *Pa = nullptr;
    PEKF_HIP(hipMalloc(&Xa, 32 * B));
    if (hipMalloc(&Pa, 128 * B) != hipSuccess) {
        (void)hipFree(Xa);
        return set_error(PEKF_ERR_HIP, "hipMalloc of %zu B failed", 128 * B);
    }
    int st = PEKF_OK;
    // keep the parts the caller does not replace: start from the current state
    if ((st = pekf_state_layout_dev(f->batch, Xa, Pa, f->X, f->P, 0, f->stream)) == PEKF_OK) {
        hipError_t e = hipSuccess;
        if (X) e = hipMemcpyAsync(Xa, X, 32 * B, hipMemcpyHostToDevice, f->stream);
        if (e == hipSuccess && P) e = hipMemcpyAsync(Pa, P, 128 * B, hipMemcpyHostToDevice, f->stream);
        if (e != hipSuccess) st = hip_fail(e, "hipMemcpyAsync");
    }
    if (st == PEKF_OK) st = pekf_state_layout_dev(f->batch, Xa, Pa, f->X, f->P, 1, f->stream);
    hipError_t e = hipStreamSynchronize(f->stream);
    if (st == PEKF_OK && e != hipSuccess) st = hip_fail(e, "hipStreamSynchronize");
    (void)hipFree(Xa);
    (void)hipFree(Pa);
    return st;
}

void release(pekf_filter *f) {
    if (!f) return;
    (void)hipFree(f->X);
    (void)hipFree(f->P);
    (void)hipFree(f->refs);
    (void)hipFree(f->prev_t);
    (void)hipFree(f->upd);
    if (f->upd_host) (void)hipHostFree(f->upd_host);
    if (f->stream) (void)hipStreamDestroy(f->stream);
    delete f;
}

}  // namespace

extern "C" {

int pekf_filter_create(int64_t batch, const double *acc0, const double *mag0, double q, double r,
                       const int64_t *t0_ns, uint32_t flags, pekf_filter **out) {
    PEKF_CHECK_ARG(out != nullptr, "null output handle");
    *out = nullptr;
    PEKF_CHECK_ARG(batch > 0 && batch < ((int64_t)1 << 28), "batch must be in [1, 2^28)");
    PEKF_CHECK_ARG(acc0 && mag0, "null pointer");
    PEKF_CHECK_ARG(r > 0.0, "r must be > 0 (S = P- + rI must be SPD)");
    PEKF_CHECK_ARG((flags & ~kFilterFlags) == 0, "unknown flags");
    if (int st = require_device()) return st;
    pekf_filter *f = new pekf_filter();
    f->batch = batch;
    f->q = q;
    f->r = r;
    f->flags = flags;
    const size_t B = (size_t)batch;
    hipError_t e = hipGetDevice(&f->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&f->X, 32 * B);
    if (e == hipSuccess) e = hipMalloc(&f->P, p_bytes(f));
    if (e == hipSuccess) e = hipMalloc(&f->refs, 48 * B);
    if (e == hipSuccess) e = hipMalloc(&f->prev_t, 8 * B);
    if (e != hipSuccess) {
        release(f);
        return hip_fail(e, "pekf_filter_create allocation");
    }
    // refs = {acc0, mag0} per filter (Wahba(acc_0, mag_0), ExtendedKalmanFilter.py:8; Wahba.py:4-6)
    std::vector<double> refs(6 * B);
    for (size_t b = 0; b < B; ++b) {
        std::memcpy(&refs[6 * b], acc0 + 3 * b, 24);
        std::memcpy(&refs[6 * b + 3], mag0 + 3 * b, 24);
    }
    std::vector<int64_t> t0(B, 0);
    if (t0_ns) std::memcpy(t0.data(), t0_ns, 8 * B);
    e = hipMemcpyAsync(f->refs, refs.data(), 48 * B, hipMemcpyHostToDevice, f->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(f->prev_t, t0.data(), 8 * B, hipMemcpyHostToDevice, f->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
    if (e != hipSuccess) {
        release(f);
        return hip_fail(e, "pekf_filter_create upload");
    }
    int st;
    if (flags & PEKF_RUN_STATE_SOA) {
        double *Xa = nullptr, *Pa = nullptr;
        st = hipMalloc(&Xa, 32 * B) == hipSuccess && hipMalloc(&Pa, 128 * B) == hipSuccess
                 ? PEKF_OK : set_error(PEKF_ERR_HIP, "hipMalloc failed");
        if (st == PEKF_OK) st = pekf_reset_state_dev(batch, Xa, Pa, f->stream);
        if (st == PEKF_OK) st = pekf_state_layout_dev(batch, Xa, Pa, f->X, f->P, 1, f->stream);
        if (st == PEKF_OK && hipStreamSynchronize(f->stream) != hipSuccess)
            st = set_error(PEKF_ERR_HIP, "hipStreamSynchronize failed");
        (void)hipFree(Xa);
        (void)hipFree(Pa);
    } else {
        st = pekf_reset_state_dev(batch, f->X, f->P, f->stream);
        if (st == PEKF_OK && hipStreamSynchronize(f->stream) != hipSuccess)
            st = set_error(PEKF_ERR_HIP, "hipStreamSynchronize failed");
    }
    if (st != PEKF_OK) {
        release(f);
        return st;
    }
    *out = f;
    return PEKF_OK;
}

int pekf_filter_destroy(pekf_filter *f) {
    if (!f) return PEKF_OK;
    (void)hipStreamSynchronize(f->stream);
    release(f);
    return PEKF_OK;
}

int pekf_filter_set_state(pekf_filter *f, const double *X, const double *P) {
    if (int st = check_handle(f)) return st;
    PEKF_CHECK_ARG(X || P, "null pointer");
    return upload_state(f, X, P);
}

int pekf_filter_get_state(pekf_filter *f, double *X, double *P) {
    if (int st = check_handle(f)) return st;
    PEKF_CHECK_ARG(X || P, "null pointer");
    const size_t B = (size_t)f->batch;
    const double *Xs = f->X, *Ps = f->P;
    double *Xa = nullptr, *Pa = nullptr;
    int st = PEKF_OK;
    if (f->flags & PEKF_RUN_STATE_SOA) {
        PEKF_HIP(hipMalloc(&Xa, 32 * B));
        if (hipMalloc(&Pa, 128 * B) != hipSuccess) {
            (void)hipFree(Xa);
            return set_error(PEKF_ERR_HIP, "hipMalloc of %zu B failed", 128 * B);
        }
        st = pekf_state_layout_dev(f->batch, Xa, Pa, f->X, f->P, 0, f->stream);
        Xs = Xa;
        Ps = Pa;
    }
    hipError_t e = hipSuccess;
    if (st == PEKF_OK && X) e = hipMemcpyAsync(X, Xs, 32 * B, hipMemcpyDeviceToHost, f->stream);
    if (st == PEKF_OK && e == hipSuccess && P) e = hipMemcpyAsync(P, Ps, 128 * B, hipMemcpyDeviceToHost, f->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(f->stream);
    if (st == PEKF_OK && e != hipSuccess) st = hip_fail(e, "pekf_filter_get_state copy");
    (void)hipFree(Xa);
    (void)hipFree(Pa);
    return st;
}

int pekf_filter_set_time(pekf_filter *f, const int64_t *t_ns) {
    if (int st = check_handle(f)) return st;
    PEKF_CHECK_ARG(t_ns != nullptr, "null pointer");
    PEKF_HIP(hipMemcpyAsync(f->prev_t, t_ns, 8 * (size_t)f->batch, hipMemcpyHostToDevice, f->stream));
    PEKF_HIP(hipStreamSynchronize(f->stream));
    return PEKF_OK;
}

int pekf_filter_get_time(pekf_filter *f, int64_t *t_ns) {
    if (int st = check_handle(f)) return st;
    PEKF_CHECK_ARG(t_ns != nullptr, "null pointer");
    PEKF_HIP(hipMemcpyAsync(t_ns, f->prev_t, 8 * (size_t)f->batch, hipMemcpyDeviceToHost, f->stream));
    PEKF_HIP(hipStreamSynchronize(f->stream));
    return PEKF_OK;
}

int pekf_filter_device_state(pekf_filter *f, double **X, double **P, double **refs) {
    if (int st = check_handle(f)) return st;
    if (X) *X = f->X;
    if (P) *P = f->P;
    if (refs) *refs = f->refs;
    return PEKF_OK;
}

int pekf_filter_update_dev(pekf_filter *f, const double *gyro, const int64_t *t_ns, const double *acc,
                           const double *mag, const uint8_t *mag_missing, double *X_out, void *stream) {
    if (int st = check_handle(f)) return st;
    PEKF_CHECK_ARG(gyro && t_ns && acc && mag, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)X_out % 16 == 0, "misaligned X_out");
    return launch_update(f->batch, gyro, t_ns, acc, mag, mag_missing, f->refs, f->prev_t, f->X, f->P, f->q, f->r,
                         X_out, f->flags, as_stream(stream));
}

int pekf_filter_update(pekf_filter *f, const double *gyro, const int64_t *t_ns, const double *acc,
                       const double *mag, const uint8_t *mag_missing, double *X_out) {
    if (int st = check_handle(f)) return st;
    PEKF_CHECK_ARG(gyro && t_ns && acc && mag, "null pointer");
    const size_t B = (size_t)f->batch;
    const UpdLayout L(f->batch);
    if (!f->upd) {
        PEKF_HIP(hipMalloc(&f->upd, L.total));
        PEKF_HIP(hipHostMalloc(&f->upd_host, L.total, hipHostMallocDefault));
    }
    char *h = f->upd_host;
    std::memcpy(h + L.gyro, gyro, 24 * B);
    std::memcpy(h + L.t, t_ns, 8 * B);
    std::memcpy(h + L.acc, acc, 24 * B);
    std::memcpy(h + L.mag, mag, 24 * B);
    if (mag_missing) std::memcpy(h + L.miss, mag_missing, B);
    PEKF_HIP(hipMemcpyAsync(f->upd, h, L.xout, hipMemcpyHostToDevice, f->stream));
    char *d = f->upd;
    if (int st = launch_update(f->batch, reinterpret_cast<const double *>(d + L.gyro),
                               reinterpret_cast<const int64_t *>(d + L.t), reinterpret_cast<const double *>(d + L.acc),
                               reinterpret_cast<const double *>(d + L.mag),
                               mag_missing ? reinterpret_cast<const uint8_t *>(d + L.miss) : nullptr, f->refs,
                               f->prev_t, f->X, f->P, f->q, f->r, X_out ? reinterpret_cast<double *>(d + L.xout) : nullptr,
                               f->flags, f->stream))
        return st;
    if (X_out) PEKF_HIP(hipMemcpyAsync(h + L.xout, d + L.xout, 32 * B, hipMemcpyDeviceToHost, f->stream));
    PEKF_HIP(hipStreamSynchronize(f->stream));
    if (X_out) std::memcpy(X_out, h + L.xout, 32 * B);
    return PEKF_OK;
}

int pekf_filter_run(pekf_filter *f, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                    const void *plane_am, const void *plane_my, double *traj, const int32_t *counts,
                    void *stream) {
    return pekf_filter_run_ext(f, n_steps, window, step0, plane_gd, plane_am, plane_my, nullptr, traj, counts,
                               stream);
}

int pekf_filter_run_ext(pekf_filter *f, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                        const void *plane_am, const void *plane_my, const double *dt_ext, double *traj,
                        const int32_t *counts, void *stream) {
    if (int st = check_handle(f)) return st;
    return pekf_run_ext_dev(f->batch, n_steps, window, step0, plane_gd, plane_am, plane_my, dt_ext, f->refs, f->X,
                            f->P, f->q, f->r, traj, counts, f->flags, stream);
}

}  // extern "C"
