// pekf_side.hip -- side outputs beside the fused filter: what main_file.py
// plots next to the filter quaternion.
//   k_gyro_chain   pure-gyro attitude: the RK4 chain of the gyro record alone, same dt as the
//                  filter (KFS/KalmanFilter.cpp:149 RungeKuttaEval(Quarternion_Gyro_pure, ...),
//                  logged as "q_gyro"; the step is ExtendedKalmanFilter.py:25-41)
//   k_wahba_stream pure-Wahba attitude per record with fixed weights (main_file.py:40,
//                  Wahba.getQuarternion(acc, mag, 0.5, 0.5), Wahba.py:49-50)
//   k_rpy          UtilityFunctions.Quart2RPY (UtilityFunctions.py:3-14), degrees
// Each reads the same resident planes as pekf_run_dev (one lane per filter, coalesced).
#include "pekf_internal.hpp"
#include "pekf_math.hpp"

namespace pekf {

// The gyro chain's record loads carry the non-temporal hint (each record is read once): 28.9 -> 26.7 ms
// at 1M x 10,000 records; the Wahba stream's do not (+1 % with it) (profiles/r4/ntload/).
__device__ __forceinline__ float4 ld_nt(const float4 *p) {
    typedef float v4 __attribute__((ext_vector_type(4)));
    const v4 v = __builtin_nontemporal_load((const v4 *)p);
    return make_float4(v.x, v.y, v.z, v.w);
}

constexpr int kSideBlock = 256;

// Both stream kernels are HBM-bound (a few dozen FP64 ops per 16-24 B record), so each lane keeps
// kDepth records in flight: a register ring filled kDepth rows ahead, the time loop unrolled by
// kDepth so every ring index is static.  The prefetch row wraps inside the resident window, so
// the loads past the last step read valid (unused) records and need no predicate.
constexpr int kDepth = 8;

// 32-bit row and step counters (window, n_steps < 2^31: checked on the host), so the wave-uniform
// tests are scalar compares; the time loop runs whole blocks of kDepth records with no exit inside the
// unrolled body (an exit per record made the compiler copy the ring on the back edge, behind a wait
// for the loads just issued), then the last n_steps % kDepth records.
__device__ __forceinline__ int32_t next_row(int32_t r, int32_t window) { return r + 1 == window ? 0 : r + 1; }

// LONGDT: the window has a dt side plane dtx[window][batch] (float64 ns); a record whose dt word is
// PEKF_DT_ESCAPE takes its dt from there, exactly as the filter does (k_run<..., LONGDT>).
template <bool LONGDT>
__global__ __launch_bounds__(kSideBlock) void k_gyro_chain(int64_t batch, int64_t n_steps, int64_t window,
                                                           int64_t step0, const float4 *__restrict__ gd,
                                                           const double *__restrict__ dtx,
                                                           double *__restrict__ q, double *__restrict__ traj) {
    const int64_t b = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    if (b >= batch) return;
    const uint32_t lane = (uint32_t)b;
    const int32_t n = (int32_t)n_steps, W = (int32_t)window;
    double x[4] = {q[4 * b], q[4 * b + 1], q[4 * b + 2], q[4 * b + 3]};
    float4 ring[kDepth];
    int32_t pf = (int32_t)(step0 % window);  // next row to prefetch
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
        ring[k] = ld_nt(gd + (int64_t)pf * batch + lane);
        pf = next_row(pf, W);
    }
    auto one = [&](int k, int32_t t) {
        const float4 r = ring[k];
        ring[k] = ld_nt(gd + (int64_t)pf * batch + lane);
        pf = next_row(pf, W);
        const double hw[3] = {0.5 * (double)r.x, 0.5 * (double)r.y, 0.5 * (double)r.z};
        const uint32_t word = __float_as_uint(r.w) & PEKF_DT_MASK;
        double dt_ns = (double)word;
        if constexpr (LONGDT) {  // off the fast path: the escaped record's row, (step0 + t) % window
            if (word == PEKF_DT_ESCAPE) dt_ns = dtx[((step0 + t) % window) * batch + b];
        }
        double z[4];
        rk4_closed(x, x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3], dt_ns, hw, z);
        x[0] = z[0]; x[1] = z[1]; x[2] = z[2]; x[3] = z[3];
        if (traj) {
            double2 *o = reinterpret_cast<double2 *>(traj + (int64_t)t * batch * 4) + 2 * (int64_t)lane;
            o[0] = make_double2(x[0], x[1]);
            o[1] = make_double2(x[2], x[3]);
        }
    };
    const int32_t n_full = n - n % kDepth;
    int32_t t0 = 0;
    for (; t0 < n_full; t0 += kDepth) {
#pragma unroll
        for (int k = 0; k < kDepth; ++k) one(k, t0 + k);
    }
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
        if (t0 + k >= n) break;  // uniform
        one(k, t0 + k);
    }
    q[4 * b] = x[0]; q[4 * b + 1] = x[1]; q[4 * b + 2] = x[2]; q[4 * b + 3] = x[3];
}

__global__ __launch_bounds__(kSideBlock) void k_wahba_stream(int64_t batch, int64_t n_steps, int64_t window,
                                                             int64_t step0, const float4 *__restrict__ am,
                                                             const float2 *__restrict__ my,
                                                             const double *__restrict__ refs, double ka,
                                                             double km, double *__restrict__ out) {
    const int64_t b = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    if (b >= batch) return;
    const uint32_t lane = (uint32_t)b;
    const int32_t n = (int32_t)n_steps, W = (int32_t)window;
    Frame Wf;
    {
        const double a0[3] = {refs[6 * b + 0], refs[6 * b + 1], refs[6 * b + 2]};
        const double m0[3] = {refs[6 * b + 3], refs[6 * b + 4], refs[6 * b + 5]};
        make_frame<true>(a0, m0, Wf);
    }
    const double sg = wahba_sign(ka, km);
    float4 ra[kDepth];
    float2 rm[kDepth];
    int32_t pf = (int32_t)(step0 % window);
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
        ra[k] = (am + (int64_t)pf * batch)[lane];
        rm[k] = (my + (int64_t)pf * batch)[lane];
        pf = next_row(pf, W);
    }
    auto one = [&](int k, int32_t t) {
        const float4 a = ra[k];
        const float2 m = rm[k];
        ra[k] = (am + (int64_t)pf * batch)[lane];
        rm[k] = (my + (int64_t)pf * batch)[lane];
        pf = next_row(pf, W);
        const double acc[3] = {a.x, a.y, a.z}, mag[3] = {a.w, m.x, m.y};
        Frame Vf;
        make_frame<true>(acc, mag, Vf, sg);
        double R[9], y[4];
        wahba_rotation<true>(Wf, Vf, ka, km, R);
        if (frame_degenerate(Vf)) {  // a zero sample or acc parallel to mag: B has rank 1 (pekf_math.hpp)
            const double sa[3] = {a.x, a.y, a.z}, sm[3] = {a.w, m.x, m.y};  // from the f32 record again
            double a0[3], m0[3];
            frame_pair(Wf, a0, m0);
            wahba_current_rank1<1>(a0, m0, sa, sm, ka, km, R);
        }
        rotm_to_quat_fast(R, y);  // keeps the reference's branch / sign convention
        double2 *o = reinterpret_cast<double2 *>(out + (int64_t)t * batch * 4) + 2 * (int64_t)lane;
        o[0] = make_double2(y[0], y[1]);
        o[1] = make_double2(y[2], y[3]);
    };
    const int32_t n_full = n - n % kDepth;
    int32_t t0 = 0;
    for (; t0 < n_full; t0 += kDepth) {
#pragma unroll
        for (int k = 0; k < kDepth; ++k) one(k, t0 + k);
    }
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
        if (t0 + k >= n) break;  // uniform
        one(k, t0 + k);
    }
}

// The same two side outputs over FP64 records (pekf_run_rec64_dev's planes: gd double4 {gyro xyz, dt_ns},
// am double4 {acc xyz, mag x}, my double2 {mag yz}), so a log replayed in FP64 gets its q_gyro / Wahba
// attitudes from the values as parsed.  The arithmetic is the 40 B-record kernels' line for line (on
// f32-representable values the results are bit-identical); dt is the float64 itself.  Shallower rings:
// a record is 32-48 B of registers here.
constexpr int kDepth64 = 4;

__global__ __launch_bounds__(kSideBlock) void k_gyro_chain64(int64_t batch, int64_t n_steps, int64_t window,
                                                             int64_t step0, const double4 *__restrict__ gd,
                                                             double *__restrict__ q, double *__restrict__ traj) {
    const int64_t b = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    if (b >= batch) return;
    const int32_t n = (int32_t)n_steps, W = (int32_t)window;
    double x[4] = {q[4 * b], q[4 * b + 1], q[4 * b + 2], q[4 * b + 3]};
    double4 ring[kDepth64];
    int32_t pf = (int32_t)(step0 % window);
#pragma unroll
    for (int k = 0; k < kDepth64; ++k) {
        ring[k] = gd[(int64_t)pf * batch + b];
        pf = next_row(pf, W);
    }
    auto one = [&](int k, int32_t t) {
        const double4 r = ring[k];
        ring[k] = gd[(int64_t)pf * batch + b];
        pf = next_row(pf, W);
        const double hw[3] = {0.5 * r.x, 0.5 * r.y, 0.5 * r.z};
        double z[4];
        rk4_closed(x, x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3], r.w, hw, z);
        x[0] = z[0]; x[1] = z[1]; x[2] = z[2]; x[3] = z[3];
        if (traj) {
            double2 *o = reinterpret_cast<double2 *>(traj + (int64_t)t * batch * 4) + 2 * b;
            o[0] = make_double2(x[0], x[1]);
            o[1] = make_double2(x[2], x[3]);
        }
    };
    const int32_t n_full = n - n % kDepth64;
    int32_t t0 = 0;
    for (; t0 < n_full; t0 += kDepth64) {
#pragma unroll
        for (int k = 0; k < kDepth64; ++k) one(k, t0 + k);
    }
#pragma unroll
    for (int k = 0; k < kDepth64; ++k) {
        if (t0 + k >= n) break;  // uniform
        one(k, t0 + k);
    }
    q[4 * b] = x[0]; q[4 * b + 1] = x[1]; q[4 * b + 2] = x[2]; q[4 * b + 3] = x[3];
}

__global__ __launch_bounds__(kSideBlock) void k_wahba_stream64(int64_t batch, int64_t n_steps, int64_t window,
                                                               int64_t step0, const double4 *__restrict__ am,
                                                               const double2 *__restrict__ my,
                                                               const double *__restrict__ refs, double ka,
                                                               double km, double *__restrict__ out) {
    const int64_t b = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    if (b >= batch) return;
    const int32_t n = (int32_t)n_steps, W = (int32_t)window;
    Frame Wf;
    {
        const double a0[3] = {refs[6 * b + 0], refs[6 * b + 1], refs[6 * b + 2]};
        const double m0[3] = {refs[6 * b + 3], refs[6 * b + 4], refs[6 * b + 5]};
        make_frame<true>(a0, m0, Wf);
    }
    const double sg = wahba_sign(ka, km);
    double4 ra[kDepth64];
    double2 rm[kDepth64];
    int32_t pf = (int32_t)(step0 % window);
#pragma unroll
    for (int k = 0; k < kDepth64; ++k) {
        ra[k] = am[(int64_t)pf * batch + b];
        rm[k] = my[(int64_t)pf * batch + b];
        pf = next_row(pf, W);
    }
    auto one = [&](int k, int32_t t) {
        const double4 a = ra[k];
        const double2 m = rm[k];
        ra[k] = am[(int64_t)pf * batch + b];
        rm[k] = my[(int64_t)pf * batch + b];
        pf = next_row(pf, W);
        const double acc[3] = {a.x, a.y, a.z}, mag[3] = {a.w, m.x, m.y};
        Frame Vf;
        make_frame<true>(acc, mag, Vf, sg);
        double R[9], y[4];
        wahba_rotation<true>(Wf, Vf, ka, km, R);
        if (frame_degenerate(Vf)) {  // a zero sample or acc parallel to mag: B has rank 1 (pekf_math.hpp)
            double a0[3], m0[3];
            frame_pair(Wf, a0, m0);
            wahba_current_rank1<1>(a0, m0, acc, mag, ka, km, R);
        }
        rotm_to_quat_fast(R, y);  // keeps the reference's branch / sign convention
        double2 *o = reinterpret_cast<double2 *>(out + (int64_t)t * batch * 4) + 2 * b;
        o[0] = make_double2(y[0], y[1]);
        o[1] = make_double2(y[2], y[3]);
    };
    const int32_t n_full = n - n % kDepth64;
    int32_t t0 = 0;
    for (; t0 < n_full; t0 += kDepth64) {
#pragma unroll
        for (int k = 0; k < kDepth64; ++k) one(k, t0 + k);
    }
#pragma unroll
    for (int k = 0; k < kDepth64; ++k) {
        if (t0 + k >= n) break;  // uniform
        one(k, t0 + k);
    }
}

// UtilityFunctions.Quart2RPY: roll = atan2(2(q0q1+q2q3), 1-2(q1^2+q2^2)), pitch = asin(2(q0q2-q3q1)),
// yaw = atan2(2(q0q3+q1q2), 1-2(q2^2+q3^2)), times 180/pi
__device__ __forceinline__ void d_rpy(int64_t i, const double *__restrict__ q, double *__restrict__ rpy) {
#pragma clang fp contract(off)  // round like NumPy: at gimbal lock sinp may round past 1 -> NaN there too
    const double *p = q + 4 * i;
    const double sinr = 2 * (p[0] * p[1] + p[2] * p[3]);
    const double cosr = 1 - 2 * (p[1] * p[1] + p[2] * p[2]);
    const double sinp = 2 * (p[0] * p[2] - p[3] * p[1]);
    const double siny = 2 * (p[0] * p[3] + p[1] * p[2]);
    const double cosy = 1 - 2 * (p[2] * p[2] + p[3] * p[3]);
    const double k = 180.0 / 3.141592653589793;
    rpy[3 * i + 0] = atan2(sinr, cosr) * k;
    rpy[3 * i + 1] = asin(sinp) * k;
    rpy[3 * i + 2] = atan2(siny, cosy) * k;
}

__global__ __launch_bounds__(kSideBlock) void k_rpy(int64_t n, const double *__restrict__ q,
                                                    double *__restrict__ rpy, Done done) {
    const int64_t i = (int64_t)blockIdx.x * kSideBlock + threadIdx.x;
    if (i < n) d_rpy(i, q, rpy);
    done.signal();
}

static int launched(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, what);
    return PEKF_OK;
}

}  // namespace pekf

using namespace pekf;

extern "C" {

int pekf_gyro_chain_ext_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                            const double *dt_ext, double *q_gyro, double *traj, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_steps >= 0, "negative size");
    if (batch == 0 || n_steps == 0) return PEKF_OK;
    PEKF_CHECK_ARG(window > 0 && step0 >= 0, "window must be > 0 and step0 >= 0");
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(plane_gd && q_gyro, "null pointer");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31) && window < ((int64_t)1 << 31), "n_steps and window must be < 2^31");
    const dim3 grid(grid_for(batch, kSideBlock)), block(kSideBlock);
    const float4 *gd = static_cast<const float4 *>(plane_gd);
    if (dt_ext)
        hipLaunchKernelGGL(k_gyro_chain<true>, grid, block, 0, as_stream(stream), batch, n_steps, window, step0, gd,
                           dt_ext, q_gyro, traj);
    else
        hipLaunchKernelGGL(k_gyro_chain<false>, grid, block, 0, as_stream(stream), batch, n_steps, window, step0, gd,
                           nullptr, q_gyro, traj);
    return launched("k_gyro_chain");
}

int pekf_gyro_chain_rec64_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                              double *q_gyro, double *traj, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_steps >= 0, "negative size");
    if (batch == 0 || n_steps == 0) return PEKF_OK;
    PEKF_CHECK_ARG(window > 0 && step0 >= 0, "window must be > 0 and step0 >= 0");
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(plane_gd && q_gyro, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)plane_gd % 32 == 0 && (uintptr_t)traj % 16 == 0, "misaligned plane / traj pointer");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31) && window < ((int64_t)1 << 31), "n_steps and window must be < 2^31");
    const dim3 grid(grid_for(batch, kSideBlock)), block(kSideBlock);
    hipLaunchKernelGGL(k_gyro_chain64, grid, block, 0, as_stream(stream), batch, n_steps, window, step0,
                       static_cast<const double4 *>(plane_gd), q_gyro, traj);
    return launched("k_gyro_chain64");
}

int pekf_wahba_stream_rec64_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_am,
                                const void *plane_my, const double *refs, double k_acc, double k_mag, double *out,
                                void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_steps >= 0, "negative size");
    if (batch == 0 || n_steps == 0) return PEKF_OK;
    PEKF_CHECK_ARG(window > 0 && step0 >= 0, "window must be > 0 and step0 >= 0");
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(plane_am && plane_my && refs && out, "null pointer");
    PEKF_CHECK_ARG((uintptr_t)plane_am % 32 == 0 && (uintptr_t)plane_my % 16 == 0 && (uintptr_t)out % 16 == 0,
                   "misaligned plane / out pointer");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31) && window < ((int64_t)1 << 31), "n_steps and window must be < 2^31");
    const dim3 grid(grid_for(batch, kSideBlock)), block(kSideBlock);
    hipLaunchKernelGGL(k_wahba_stream64, grid, block, 0, as_stream(stream), batch, n_steps, window, step0,
                       static_cast<const double4 *>(plane_am), static_cast<const double2 *>(plane_my), refs, k_acc,
                       k_mag, out);
    return launched("k_wahba_stream64");
}

int pekf_gyro_chain_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                        const void *plane_gd, double *q_gyro, double *traj, void *stream) {
    return pekf_gyro_chain_ext_dev(batch, n_steps, window, step0, plane_gd, nullptr, q_gyro, traj, stream);
}

int pekf_wahba_stream_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                          const void *plane_am, const void *plane_my, const double *refs, double k_acc,
                          double k_mag, double *out, void *stream) {
    PEKF_CHECK_ARG(batch >= 0 && n_steps >= 0, "negative size");
    if (batch == 0 || n_steps == 0) return PEKF_OK;
    PEKF_CHECK_ARG(window > 0 && step0 >= 0, "window must be > 0 and step0 >= 0");
    PEKF_CHECK_ARG(batch < ((int64_t)1 << 28), "batch must be < 2^28 filters per launch");
    PEKF_CHECK_ARG(plane_am && plane_my && refs && out, "null pointer");
    PEKF_CHECK_ARG(n_steps < ((int64_t)1 << 31) && window < ((int64_t)1 << 31), "n_steps and window must be < 2^31");
    hipLaunchKernelGGL(k_wahba_stream, dim3(grid_for(batch, kSideBlock)), dim3(kSideBlock), 0,
                       as_stream(stream), batch, n_steps, window, step0,
                       static_cast<const float4 *>(plane_am), static_cast<const float2 *>(plane_my),
                       refs, k_acc, k_mag, out);
    return launched("k_wahba_stream");
}

int pekf_quat_to_rpy_dev(int64_t n, const double *q, double *rpy, void *stream) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(q && rpy, "null pointer");
    hipLaunchKernelGGL(k_rpy, dim3(grid_for(n, kSideBlock)), dim3(kSideBlock), 0, as_stream(stream), n,
                       q, rpy, kNoSignal);
    return launched("k_rpy");
}

int pekf_quat_to_rpy(int64_t n, const double *q, double *rpy) {
    PEKF_CHECK_ARG(n >= 0, "n < 0");
    if (n == 0) return PEKF_OK;
    PEKF_CHECK_ARG(q && rpy, "null pointer");
    if (int st = require_device()) return st;
    Staging &s = Staging::get();
    const size_t b = (size_t)n * sizeof(double);
    void *in[1], *out[1];
    if (int st = s.stage_in({{q, 4 * b}}, {3 * b}, in, out)) return st;
    hipLaunchKernelGGL(k_rpy, dim3(grid_for(n, kSideBlock)), dim3(kSideBlock), 0, s.stream(), n,
                       static_cast<const double *>(in[0]), static_cast<double *>(out[0]),
                       s.done(grid_for(n, kSideBlock)));
    if (int st = launched("k_rpy")) return st;
    return s.stage_out({{rpy, 3 * b}}, out);
}

}  // extern "C"
