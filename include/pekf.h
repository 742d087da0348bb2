/*
 * pekf.h -- C ABI of libpekf.so, the MI355X (gfx950) batched quaternion-EKF engine.
 *
 * The reference exposes this path as a pure-Python module API with no FFI
 * (SURVEY.md §8b).  Each entry point below replaces one reference interface; the
 * Python drop-in modules (poseestimationkf_amd/dropin/) bind them with ctypes, exactly
 * as a maintainer would bind them from the reference side.
 * Paths are relative to "/root/reference/Python Kalman Filter/".
 *
 * Conventions
 *   - Plain C types only: int64_t counts, double/float/uint32_t arrays, void* streams.
 *   - Quaternions are [w, x, y, z]; 4x4 / 3x3 / 4x3 matrices are row-major.
 *   - "_dev" entry points take DEVICE pointers and a hipStream_t (as void*, NULL =
 *     the null stream) and only enqueue work.  The other batched entry points take
 *     HOST pointers, stage through a pinned buffer, and return when results are on
 *     the host.  All pointers are caller-owned and contiguous.
 *   - Every entry returns a status (PEKF_OK = 0).  pekf_last_error() gives the
 *     calling thread's message for the last failure.  No exceptions cross the ABI.
 *   - There is no CPU fallback: without a usable gfx950 device every compute entry
 *     returns PEKF_ERR_NODEVICE.
 */
#ifndef PEKF_H
#define PEKF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PEKF_ABI_VERSION 1

#define PEKF_OK 0
#define PEKF_ERR_INVALID 1  /* bad argument (null pointer, negative size, ...)          */
#define PEKF_ERR_HIP 2      /* HIP runtime error (message has hipGetErrorString)        */
#define PEKF_ERR_SINGULAR 3 /* S = P + R singular in predict: np.linalg.LinAlgError      */
#define PEKF_ERR_NODEVICE 4 /* no HIP device visible                                     */
#define PEKF_ERR_SVD 5      /* non-finite Wahba matrix B: np.linalg.svd raises LinAlgError  */
                            /* "SVD did not converge" (Wahba.py:14)                         */
#define PEKF_ERR_COMM 6     /* collective library (RCCL) unavailable or failed              */
#define PEKF_ERR_TIMEOUT 7  /* a collective step passed its deadline; the communicator was aborted */

/* Bit 31 of a stream record's dt word: magnetometer sample missing ("Wahba-skip"). */
#define PEKF_MISSING_MAG_BIT 0x80000000u
/* Bits 0-30 of the dt word: the record's dt = T - previousT in ns (ExtendedKalmanFilter.py:62), an
 * integer in [0, 2^31 - 1).  All ones (PEKF_DT_ESCAPE) = the dt is not in the word: it is the float64
 * dt_ext[row][filter] of the window's dt side plane -- any value the reference's float64 T - previousT
 * can take: a pause of 2^31 ns (2.1 s) or more, a negative or a fractional difference. */
#define PEKF_DT_MASK 0x7FFFFFFFu
#define PEKF_DT_ESCAPE 0x7FFFFFFFu

/* pekf_run_dev flags.  Default (0): every operation in FP64, as the reference.
 * PEKF_RUN_MIXED_PRECISION: opt-in; the covariance recursion (P-, S^-1, K, P) in FP32, the
 * quaternion path (RK4, Wahba, R->q, X update) in FP64.  Quaternions stay within ~1e-8 of FP64. */
#define PEKF_RUN_MIXED_PRECISION 0x1u
/* PEKF_RUN_STATE_SOA: X and P are in the coalesced SoA layout of pekf_state_layout_dev (for launches
 * that cover few records, where the state read/write dominates: online serving). */
#define PEKF_RUN_STATE_SOA 0x2u

int pekf_abi_version(void);
const char *pekf_last_error(void);

/* ---------------- device, memory, streams, events (host plumbing, no PyTorch) ---------------- */
int pekf_device_count(int *count);
int pekf_set_device(int device);
int pekf_get_device(int *device);
int pekf_device_name(int device, char *buf, int buflen); /* gcnArchName, e.g. "gfx950:sramecc+:xnack-" */
int pekf_malloc(void **dptr, size_t bytes);
int pekf_free(void *dptr);
int pekf_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int pekf_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int pekf_memcpy_d2d(void *dst, const void *src, size_t bytes, void *stream);
int pekf_memset(void *dst, int value, size_t bytes, void *stream);
int pekf_stream_create(void **stream);
int pekf_stream_destroy(void *stream);
int pekf_stream_sync(void *stream);
int pekf_device_sync(void);
int pekf_event_create(void **event);
int pekf_event_destroy(void *event);
int pekf_event_record(void *event, void *stream);
int pekf_event_sync(void *event);
int pekf_event_elapsed_ms(float *ms, void *start, void *stop);

/* ---------------- per-call operators (batched over n independent items) ----------------
 * One GPU thread per item.  These are the drop-in replacements for the reference's
 * per-timestep methods; at n = 1 they serve main_file.py through the Python shims. */

/* How n = 1 calls of pekf_predict / pekf_correct / pekf_wahba_quaternion (one record of
 * main_file.py:38-45 at a time) reach the GPU:
 *   PEKF_PERCALL_SERVICE (default): a resident one-wave kernel answers requests posted in
 *     coherent pinned host memory (~4 us round trip instead of a launch); it ends by itself
 *     after 5 ms without requests and before pekf_device_sync, and is restarted on demand.
 *   PEKF_PERCALL_LAUNCH: one kernel launch per call (also selected by PEKF_PERCALL=launch).
 * Both run the same device code, so results are identical. */
#define PEKF_PERCALL_SERVICE 0
#define PEKF_PERCALL_LAUNCH 1
int pekf_set_percall_mode(int mode);
int pekf_get_percall_mode(int *mode);

/* KalmanFilter.RungeKutta4(q_0, T, w), ExtendedKalmanFilter.py:25-41.
 * q0[n*4], dt_ns[n] (nanoseconds; dt = dt_ns * 1e-9 as at :32), w[n*3] -> q_out[n*4]. */
int pekf_rk4(int64_t n, const double *q0, const double *dt_ns, const double *w, double *q_out);
int pekf_rk4_dev(int64_t n, const double *q0, const double *dt_ns, const double *w, double *q_out,
                 void *stream);

/* UtilityFunctions.norm(a), UtilityFunctions.py:16-21: sqrt of the sequential sum of squares
 * of each of n vectors of length len: a[n*len] -> out[n]. */
int pekf_norm(int64_t n, int64_t len, const double *a, double *out);

/* KalmanFilter.GetJacobian_A(w) -> 0.5*Omega(w) [n*16], ExtendedKalmanFilter.py:43-48 */
int pekf_jacobian_a(int64_t n, const double *w, double *A);
/* KalmanFilter.GetJacobian_B(q) -> 0.5*Xi(q) [n*12], ExtendedKalmanFilter.py:51-56 */
int pekf_jacobian_b(int64_t n, const double *q, double *Jb);
/* KalmanFilter.Comparator(q1, q2) -> conj(q1) (x) q2 [n*4], ExtendedKalmanFilter.py:16-23 */
int pekf_comparator(int64_t n, const double *q1, const double *q2, double *out);

/* KalmanFilter.Prediction(Gyro, T, X_k, P_k), ExtendedKalmanFilter.py:58-68, minus the
 * previousT bookkeeping (:62,:67), which stays with the caller: dt_ns = T - previousT.
 * gyro[n*3], dt_ns[n], X[n*4], P[n*16], Q[n*9], R[n*16] -> z[n*4], Pm[n*16], K[n*16].
 * Returns PEKF_ERR_SINGULAR if any S = Pm + R is singular (the reference raises
 * np.linalg.LinAlgError from np.linalg.inv, :65). */
int pekf_predict(int64_t n, const double *gyro, const double *dt_ns, const double *X,
                 const double *P, const double *Q, const double *R, double *z, double *Pm,
                 double *K);
int pekf_predict_dev(int64_t n, const double *gyro, const double *dt_ns, const double *X,
                     const double *P, const double *Q, const double *R, double *z, double *Pm,
                     double *K, int32_t *status /* device int32[n]: 1 = S singular; may be NULL */,
                     void *stream);

/* KalmanFilter.Correction(Mag, Acc, z_k, P_k, K_k), ExtendedKalmanFilter.py:70-80, with the
 * filter's Wahba reference vectors acc0/mag0 (Wahba.__init__, Wahba.py:4-6).
 * mag[n*3], acc[n*3], z[n*4], P[n*16], K[n*16], acc0[n*3], mag0[n*3] -> X[n*4], P_out[n*16].
 * Returns PEKF_ERR_SVD if any item's B is non-finite (outputs of that item are NaN). */
int pekf_correct(int64_t n, const double *mag, const double *acc, const double *z,
                 const double *P, const double *K, const double *acc0, const double *mag0,
                 double *X, double *P_out);
int pekf_correct_dev(int64_t n, const double *mag, const double *acc, const double *z,
                     const double *P, const double *K, const double *acc0, const double *mag0,
                     double *X, double *P_out, void *stream);

/* Wahba.getRotation(acc, mag, k_acc, k_mag), Wahba.py:8-17 -> R[n*9] (closed form).
 * Returns PEKF_ERR_SVD if any item's B is non-finite, as np.linalg.svd raises there. */
int pekf_wahba_rotation(int64_t n, const double *acc0, const double *mag0, const double *acc,
                        const double *mag, const double *k_acc, const double *k_mag, double *R);
/* Wahba.getQuarternion(acc, mag, k_acc, k_mag), Wahba.py:49-50 -> q[n*4] */
int pekf_wahba_quaternion(int64_t n, const double *acc0, const double *mag0, const double *acc,
                          const double *mag, const double *k_acc, const double *k_mag, double *q);
/* Wahba.RotationMatrix2Quart(M), Wahba.py:19-47 -> q[n*4] (3-branch, strict '>', no trace branch) */
int pekf_rotmat_to_quat(int64_t n, const double *M, double *q);

/* ---------------- fused hot path: the whole main_file.py:38-47 loop on the device ----------------
 * One lane per filter; each lane runs n_steps of Prediction + Correction with X and P in
 * registers.  Step t of the launch reads stream row (step0 + t) % window:
 *   plane_gd : float4 [window][batch] {gyro x, y, z, bits(dt word)}   dt word = dt_ns | flags
 *   plane_am : float4 [window][batch] {acc x, y, z, mag x}
 *   plane_my : float2 [window][batch] {mag y, z}
 * refs[batch*6] = {acc0 xyz, mag0 xyz} (float64; KalmanFilter(T0, mag_0, acc_0), :6-11).
 * X[batch*4], P[batch*16] (row-major, symmetric; the kernel reads the upper triangle) are
 * read at launch start and written at the end.  q, r: setQ/setR scales (:12-15).
 * A record whose dt word has PEKF_MISSING_MAG_BIT set runs Prediction only (X = z, P = P-).
 * A non-finite sample cannot raise per filter inside a batch: that filter's X and P become NaN
 * (the reference raises LinAlgError from np.linalg.svd at that record).
 * traj (optional, NULL to skip): X after every step, [n_steps][batch][4].
 * counts (optional, NULL = all n_steps): filter b applies only its first min(counts[b], n_steps)
 *   records of this launch (ragged logs / front-end output sharing one launch); its traj rows after
 *   that repeat its final X.
 * flags: PEKF_RUN_MIXED_PRECISION and/or PEKF_RUN_STATE_SOA (X[4][batch], P[10][batch]). */
int pekf_run_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                 const void *plane_gd, const void *plane_am, const void *plane_my,
                 const double *refs, double *X, double *P, double q, double r, double *traj,
                 const int32_t *counts, uint32_t flags, void *stream);
/* pekf_run_dev for a window with escaped dt words: dt_ext = the window's dt side plane, float64
 * [window][batch] (read only at rows whose dt word is PEKF_DT_ESCAPE; NULL = no escapes, exactly
 * pekf_run_dev). */
int pekf_run_ext_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                     const void *plane_gd, const void *plane_am, const void *plane_my, const double *dt_ext,
                     const double *refs, double *X, double *P, double q, double r, double *traj,
                     const int32_t *counts, uint32_t flags, void *stream);
/* The same launch over FP64 records, for inputs that are float64 to begin with (recorded logs, which the
 * reference parses into float64, ReadFile.py:14-21): 80 B per filter-record in three
 * filter-minor planes,
 *   plane_gd : double4 [window][batch] {gyro x, y, z, dt_ns} -- dt the float64 T - previousT itself
 *              (ExtendedKalmanFilter.py:62): any pause, clock step or fraction
 *   plane_am : double4 [window][batch] {acc x, y, z, mag x}
 *   plane_my : double2 [window][batch] {mag y, z}
 * Every record is a full record (no missing-magnetometer flag).  refs, X, P, q, r, traj, counts as
 * pekf_run_dev (AoS FP64 state); always the multi-record arithmetic, so a window of f32-representable
 * values gives pekf_run_dev's state (n_steps >= 2) bit for bit.  batch < 2^27 (32-bit lane offsets of
 * the 32 B planes); planes 32 B aligned (my: 16 B). */
int pekf_run_rec64_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                       const void *plane_am, const void *plane_my, const double *refs, double *X, double *P,
                       double q, double r, double *traj, const int32_t *counts, void *stream);
/* AoS state (X[batch][4], P[batch][4][4]) <-> SoA state (X[4][batch], P[10][batch] holding
 * P00 P01 P02 P03 P11 P12 P13 P22 P23 P33).  to_soa != 0: AoS -> SoA, else SoA -> AoS. */
int pekf_state_layout_dev(int64_t batch, double *X_aos, double *P_aos, double *X_soa, double *P_soa,
                          int to_soa, void *stream);

/* ---------------- side outputs: what main_file.py plots beside X ----------------
 * Pure-gyro attitude: the RK4 chain of the gyro records alone, same dt as the filter (KFS/KalmanFilter.cpp:149,
 * logged as "q_gyro"; step = ExtendedKalmanFilter.py:25-41).  q_gyro[batch*4] in/out; traj optional. */
int pekf_gyro_chain_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                        const void *plane_gd, double *q_gyro, double *traj, void *stream);
/* pekf_gyro_chain_dev for a window with escaped dt words: dt_ext = the window's dt side plane, float64
 * [window][batch], read at rows whose dt word is PEKF_DT_ESCAPE (NULL = exactly pekf_gyro_chain_dev). */
int pekf_gyro_chain_ext_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                            const double *dt_ext, double *q_gyro, double *traj, void *stream);
/* Pure-Wahba attitude of every record with fixed weights (main_file.py:40: getQuarternion(acc, mag,
 * 0.5, 0.5)), out[n_steps][batch][4], same branch/sign convention as Wahba.RotationMatrix2Quart. */
int pekf_wahba_stream_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0,
                          const void *plane_am, const void *plane_my, const double *refs, double k_acc,
                          double k_mag, double *out, void *stream);
/* The pure-gyro chain and the pure-Wahba stream over FP64 records (pekf_run_rec64_dev's planes: the gd
 * plane double4 {gyro xyz, dt_ns}, am double4 {acc xyz, mag x}, my double2 {mag yz}); the same arithmetic as
 * the two above, dt the float64 itself. */
int pekf_gyro_chain_rec64_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                              double *q_gyro, double *traj, void *stream);
int pekf_wahba_stream_rec64_dev(int64_t batch, int64_t n_steps, int64_t window, int64_t step0, const void *plane_am,
                                const void *plane_my, const double *refs, double k_acc, double k_mag, double *out,
                                void *stream);
/* UtilityFunctions.Quart2RPY(q), UtilityFunctions.py:3-14: q[n*4] -> rpy[n*3] in degrees. */
int pekf_quat_to_rpy(int64_t n, const double *q, double *rpy);
int pekf_quat_to_rpy_dev(int64_t n, const double *q, double *rpy, void *stream);

/* ---------------- recorded traces: the server's text log -> 40 B records ----------------
 * Host-side ingest (no device work).  Tags / precedence of ReadFile.py:27-45; one record per Acc_1 line
 * (main_file.py:38), dt_ns = T[i+1] - T[i] in float64 (ExtendedKalmanFilter.py:62).
 * pekf_log_scan gives the record count; pekf_log_read fills gyro/acc/mag[n*3] (float), dtw[n],
 * acc0/mag0[3] (double) and t0 (first timestamp; may be NULL); it refuses a log with a dt that is not an
 * integer in [0, 2^31 - 1).  pekf_log_read_ext takes any dt: such a record gets the escape word and its
 * float64 dt in dt_ext[n] (the window's dt side plane; other entries are set to 0); *n_escaped (may be
 * NULL) receives how many records were escaped. */
int pekf_log_scan(const char *path, int64_t *n_records);
int pekf_log_read(const char *path, int64_t n_records, float *gyro, float *acc, float *mag, uint32_t *dtw,
                  double *acc0, double *mag0, double *t0);
int pekf_log_read_ext(const char *path, int64_t n_records, float *gyro, float *acc, float *mag, uint32_t *dtw,
                      double *dt_ext, int64_t *n_escaped, double *acc0, double *mag0, double *t0);
/* The log's records as parsed, float64 (the records of pekf_run_rec64_dev): gyro/acc/mag[n*3], dt_ns[n] =
 * T[i+1] - T[i] (any value), acc0/mag0[3], t0 (may be NULL). */
int pekf_log_read64(const char *path, int64_t n_records, double *gyro, double *acc, double *mag, double *dt_ns,
                    double *acc0, double *mag0, double *t0);
/* The emit side: writes (truncates) path with the lines the server's KalmanFilter writes for one client
 * (KFS/KalmanFilter.cpp WriteTextFile, :335-340): mag_0 / acc_0 (:26-33), the initial q_gyro / X_k /
 * Wahba_quart (:55-67), then per record gyro (:265-277), T (the first record: previousT before it,
 * :136-141), q_gyro (:150-153), Mag_1 / Acc_1 (:279-303), X_k / Wahba_quart (:180-183).  Numbers as
 * std::to_string prints them in the "C" locale ("%f", the integer ns times).  t_ns[n_records + 1] = T0
 * then one time per record; gyro/acc/mag[n*3]; acc0/mag0[3]; q_gyro / x_k / wahba[n*4] may be NULL
 * (written as zeros).  Replaces the server's logging for traces made elsewhere (a batch run's inputs and
 * outputs, synthetic streams); pekf_log_read* and ReadFile.getData read it back. */
int pekf_log_write(const char *path, int64_t n_records, const int64_t *t_ns, const double *gyro, const double *acc,
                   const double *mag, const double *acc0, const double *mag0, const double *q_gyro, const double *x_k,
                   const double *wahba);

/* ---------------- server front-end: raw phone events -> records ----------------
 * Device kernel.  Per filter, the phase-3 state machine of Parser::WriteKalmanFilterMeasurement
 * (KFS/Parser.cpp:148-219), linear interpolation of acc / mag to the gyro time (:259-267),
 * normalisation (:221-228) and the alpha low-pass from a zero state (KFS/KalmanFilter.cpp:16-18,
 * 21-24,279-303) -> records written to plane_gd / plane_am / plane_my rows 0..counts[b]-1
 * ([r_max][batch], the layout pekf_run_dev reads), dt = gyro time - previous record's (initially
 * t_init[b]).  Events: ev_planes float4 [n_events][batch] {x, y, z, bits(word)}, 16 B each, with
 * word = (ns since the filter's previous event, first: since t_init[b]) << 2 | type (0 acc, 1 gyro,
 * 2 mag, 3 a message no sensor takes: skipped in phase 3, a message like any other in phase 2), so gaps
 * must be < 2^30 ns (and a type-3 message's > 0: word 3 is the time event below).  init[batch*6] = raw phase-2 means {acc xyz, mag xyz}
 * (Parser.cpp:44-53); refs[batch*6] receives their normalised values (the filter's acc0 / mag0).
 * A filter whose init is not finite (pekf_frontend_init_dev's "not ready") produces no record (counts 0).
 * *dev_error |= 1 if a record dt does not fit 31 bits, 2 if a filter had more than r_max records. */
int pekf_frontend_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                      const int64_t *t_init, double alpha, int64_t r_max,
                      void *plane_gd, void *plane_am, void *plane_my, int32_t *counts, double *refs,
                      int *dev_error, void *stream);
/* Time events (type 3, PEKF_EV_TIME): an event whose word is exactly 3 carries no sample; its x and y
 * floats are the two halves (low, high) of a float64 time step in ns added to the filter's clock --
 * any gap the 30-bit field cannot hold (a pause of 2^30 ns or more, or a clock that steps back).  The
 * event after it then has its own gap from the new time (usually 0).  A time event with step 0 is a
 * no-op, which pads shorter event streams to the plane's length.  Phase 2 (pekf_frontend_init_dev)
 * always honours them; the phase-3 kernels do with PEKF_EV_TIME_EVENTS in flags (without it a word-3
 * event is skipped and the clock does not move, at no cost to the event loop). */
#define PEKF_EV_TIME 3u
#define PEKF_EV_TIME_EVENTS 0x1u
#define PEKF_EV_F32_RECORDS 0x2u /* pekf_live_ext_dev: records rounded to the f32 stream record format */
/* FP64 events (pekf_live_ext_dev, pekf_frontend_ext_dev, pekf_frontend_init_ext_dev): ev_planes is double4
 * [n_events][batch], 32 B per event, {x, y, z, w} where x, y, z are the sample as the server parses it
 * (std::stod of the phone's text, KFS/Parser.cpp:23-25 -- in general not the f32 the phone measured) and
 * w's bits are those of the event's absolute time in ns as a float64 (an integer, |t| < 2^51) with the
 * type (0 acc, 1 gyro, 2 mag, 3 a message no sensor takes) in its two lowest bits; w = the bits of -0.0
 * with type 3 (0x8000000000000003, which no time packs to) is no message at all, for padding.  t_init /
 * t_start are times on the same clock.  Any gap or clock step is just the next event's time (no time events); records are FP64
 * throughout, their dt any float64.  Host packing: pekf_wire_parse (wire text) or pekf_f32_wire_values
 * (f32 samples -> the doubles the server would parse). */
#define PEKF_EV_F64_EVENTS 0x4u
/* pekf_frontend_dev with time events (flags) and escaped records: a record whose dt does not fit the
 * dt word gets PEKF_DT_ESCAPE and its float64 dt in dt_ext[r_max][batch] (the window's dt side plane for
 * pekf_run_ext_dev; only escaped entries are written), and *dev_error |= 4 says some record was escaped.
 * dt_ext = NULL: such a record sets *dev_error bit 1, as pekf_frontend_dev. */
int pekf_frontend_ext_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                          const int64_t *t_init, double alpha, int64_t r_max, void *plane_gd, void *plane_am,
                          void *plane_my, double *dt_ext, int32_t *counts, double *refs, uint32_t flags,
                          int *dev_error, void *stream);

/* The server's phase 3 with the filter fused in: pekf_frontend_dev's records are not
 * written anywhere -- each is applied to the filter's state on the same lane (Prediction + Correction,
 * main_file.py:42-45) as soon as the wave runs its next filter step.  Same events, init, t_init, alpha
 * and refs as pekf_frontend_dev; X[batch*4], P[batch*16] (AoS, FP64) are the filters' state, read at
 * the start and written at the end (left untouched for a filter with no record, as for one whose init
 * is not finite: phase 2 never got ready); q, r as pekf_run_dev.
 * counts[b] receives the number of records filter b applied.  A record's acc / mag reach the filter as
 * the FP64 low-pass outputs, as the server hands them to its filter (KFS/KalmanFilter.cpp:279-303); with
 * PEKF_EV_F32_RECORDS (pekf_live_ext_dev) they are rounded to f32 first, as in the 40 B stream record,
 * and the final state then equals pekf_frontend_dev followed by pekf_run_dev with those counts, bit for
 * bit.  A record whose dt does not fit the dt word
 * keeps its float64 dt beside it on the lane (as pekf_frontend_ext_dev + pekf_run_ext_dev would), so any
 * gap is applied; dev_error is kept for the ABI and never set by this kernel (no r_max either: there is
 * no record window). */
int pekf_live_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                  const int64_t *t_init, double alpha, double *X, double *P, double q, double r,
                  int32_t *counts, double *refs, int *dev_error, void *stream);
/* pekf_live_dev with flags (PEKF_EV_TIME_EVENTS: the planes hold time events; PEKF_EV_F32_RECORDS: f32
 * records, the split pipeline's; PEKF_EV_F64_EVENTS alone: FP64 events, every record field FP64 -- the
 * server's own input values end to end). */
int pekf_live_ext_dev(int64_t batch, int64_t n_events, const void *ev_planes, const double *init,
                      const int64_t *t_init, double alpha, double *X, double *P, double q, double r,
                      int32_t *counts, double *refs, uint32_t flags, int *dev_error, void *stream);

/* Phase 2 of the server's Parser (KFS/Parser.cpp:36-58,84-140; KFS/InitialValues.cpp) on the device: per
 * filter, the mean and sample variance of the first n_avg (the server: 100) samples of each sensor type,
 * and the time phase 3 continues from.  Events as for pekf_frontend_dev (ev_planes [n_events][batch], word
 * = gap << 2 | type, the first gap from t_start[b]).  A filter is ready once every sensor has had a sample
 * after its first n_avg and one more message of any type (3 included) has arrived (the KalmanFilter
 * construction, :41-55); later messages move t_init to their time (:57-62).  Time events and FP64
 * no-message events are not messages.  Outputs (device): init[batch*6] = raw means {acc xyz, mag
 * xyz} and t_init[batch] -- pekf_frontend_dev's init / t_init --, ready[batch] (0: not enough phase-2
 * events; init is then NaN), stats[batch*12] (optional) = {gyro mean, acc / mag / gyro variance};
 * with stats NULL the second pass over the events (the variances) is skipped. */
int pekf_frontend_init_dev(int64_t batch, int64_t n_events, const void *ev_planes, const int64_t *t_start,
                           int n_avg, double *init, int64_t *t_init, double *stats, int32_t *ready, void *stream);
/* pekf_frontend_init_dev with flags: PEKF_EV_F64_EVENTS (FP64 events: the means and variances of the
 * server's own stod values, Parser.cpp:23-25,84-140; times absolute).  PEKF_EV_TIME_EVENTS is accepted
 * and changes nothing (phase 2 always honours time events). */
int pekf_frontend_init_ext_dev(int64_t batch, int64_t n_events, const void *ev_planes, const int64_t *t_start,
                               int n_avg, double *init, int64_t *t_init, double *stats, int32_t *ready,
                               uint32_t flags, void *stream);

/* The wire on the device: the clients' 100-byte frames (as MessageSender.java:217-233 sends and Server.cpp:35,84
 * receives them: "#<phase>,<type>:<x>,<y>,<z>,t:<ns>", spaces to 99 characters, '\n') -> FP64 event planes.
 * frames: [n_frames][batch][100] bytes (device; 4-byte aligned), phone b's frames in order along the first
 * axis (a frame not starting with '#' is no message, e.g. padding; a frame is one message whatever it holds,
 * as the server takes each recv -- a newline inside it does not split it).  Each phase-2 / phase-3 message of phone b
 * becomes the next row of ev2 / ev3 ([e2_max][batch] / [e3_max][batch] double4, PEKF_EV_F64_EVENTS' form;
 * type 3 for a Type no sensor takes); rows after its last message get the no-message event.  n2 / n3[batch]:
 * messages per phase (more than e_max: *dev_error |= 2, the extra ones dropped); first_t2[batch]: the time of
 * the first phase-2 message (t_start of pekf_frontend_init_ext_dev; 0 if none).  Values and times equal
 * pekf_wire_parse's (std::stod / std::stoll) bit for bit for the forms the client prints -- decimals (any
 * of at most 19 significant digits within 1e-80 .. 1e80 of the exponent; an exact big-integer path where
 * one IEEE operation is not exact), "NaN", "Infinity", "-Infinity"; a phone's first frame in another form,
 * or with a time of 2^51 ns or more, stops that phone: bad_frame[b] (may be NULL) = its index (-1: none),
 * *dev_error |= 1 (parse such a stream with pekf_wire_parse).  Phase-1 and other phases are skipped. */
int pekf_wire_events_dev(int64_t batch, int64_t n_frames, const void *frames, int64_t e2_max, int64_t e3_max,
                         void *ev2, void *ev3, int64_t *first_t2, int32_t *n2, int32_t *n3, int32_t *bad_frame,
                         int *dev_error, void *stream);
/* pekf_wire_events_dev with flags.  PEKF_WIRE_FRAME_ROWS: the planes get a row per frame index instead of
 * a row per message -- row f of ev2 / ev3 holds frame f's message if it is one of that phase, else the
 * no-message event, which phase 2 (pekf_frontend_init_ext_dev) and phase 3 (pekf_live_ext_dev) skip, so
 * they give the same results on n_frames rows as on the compacted planes.  Every lane of a wave then
 * stores the same row: for phones whose rows would drift apart (phase-1 / phase-2 parts of different
 * lengths), at 32 B more written per frame.  Needs e2_max, e3_max >= n_frames; n2 / n3 still count the
 * messages.  A phone's rows from its refused frame on are no-message events.  Where the grid leaves the
 * GPU's SIMDs short of 4 waves, the frames are split into chunks parsed by separate waves (a stream-ordered
 * allocation of 24 B per phone and chunk holds their counts until a second kernel combines them;
 * PEKF_WIRE_CHUNKS=n in the environment forces n chunks).  row_bounds (device, 2 int32, may be NULL; with
 * PEKF_WIRE_FRAME_ROWS only): [0] = 1 + the last row holding a phase-2 message of any phone, [1] = n_frames
 * - the first row holding a phase-3 message of any phone (0: none) -- the rows outside them are no-message
 * rows in every column, which a consumer may leave out (ev2's first [0] rows, ev3 from row n_frames - [1]). */
#define PEKF_WIRE_FRAME_ROWS 0x1u
int pekf_wire_events_ext_dev(int64_t batch, int64_t n_frames, const void *frames, int64_t e2_max, int64_t e3_max,
                             void *ev2, void *ev3, int64_t *first_t2, int32_t *n2, int32_t *n3, int32_t *bad_frame,
                             int *dev_error, int32_t *row_bounds, uint32_t flags, void *stream);

/* ---------------- the phone -> server wire: host code ----------------
 * The Android client sends each sample as text, Float.toString of each value
 * (ASC/MessageSender.java:217-233: "#<phase>,<type>:<x>,<y>,<z>,t:<ns>" padded to 99 characters), and
 * the server parses the values with std::stod (KFS/Parser.cpp:12-26): doubles, in general not the
 * floats the phone measured.  These two functions give the FP64 event planes those doubles.
 * pekf_wire_parse: the server's parse of such text, one message per line (Parser::run keeps messages
 * starting with '#'; ProcessString skips one of 30 characters or fewer after the '#', newline
 * included).  phase / type: the digits' values; xyz[3n] as strtod (= std::stod) gives them; t_ns as
 * strtoll (= std::stoll).  All four outputs NULL: count only (*n_events).  A message the server's stod /
 * stoll would throw on returns PEKF_ERR_INVALID naming its line. */
int pekf_wire_parse(const char *text, int64_t len, int64_t max_events, uint8_t *phase, uint8_t *type, double *xyz,
                    int64_t *t_ns, int64_t *n_events);
/* out[i] = the double std::stod makes of Float.toString(in[i]): the shortest decimal that rounds to the
 * float, the closest one among those (JDK 19+ Float.toString; one that needs a single digit prints the
 * closest of one or two digits), read back correctly rounded. */
int pekf_f32_wire_values(int64_t n, const float *in, double *out);

/* X = [1,0,0,0], P = I for every filter (main_file.py:23,26). */
int pekf_reset_state_dev(int64_t batch, double *X, double *P, void *stream);

/* ---------------- filter handle: the batched core of SURVEY.md §8b ----------------
 * One handle = `batch` KalmanFilter objects (ExtendedKalmanFilter.py:6-15): it owns, on the
 * current device, each filter's Wahba reference (acc0, mag0), Q = q I, R = r I, previousT and
 * the state X = [1,0,0,0], P = I (main_file.py:23,26), which stays device-resident between calls.
 * flags: PEKF_RUN_MIXED_PRECISION and/or PEKF_RUN_STATE_SOA (device layout of the state).
 * acc0 / mag0: host [batch*3]; t0_ns: host [batch] initial previousT (NULL = 0). */
typedef struct pekf_filter pekf_filter;
int pekf_filter_create(int64_t batch, const double *acc0, const double *mag0, double q, double r,
                       const int64_t *t0_ns, uint32_t flags, pekf_filter **out);
int pekf_filter_destroy(pekf_filter *f);
/* Host copies of the state in the reference layout: X[batch*4], P[batch*16] (P may be NULL). */
int pekf_filter_set_state(pekf_filter *f, const double *X, const double *P);
int pekf_filter_get_state(pekf_filter *f, double *X, double *P);
/* previousT of every filter (host [batch]); the stream path (pekf_filter_run) uses dt records and
 * leaves it untouched, so set it before switching back to pekf_filter_update. */
int pekf_filter_set_time(pekf_filter *f, const int64_t *t_ns);
/* previousT of every filter (host [batch]; KalmanFilter.previousT, ExtendedKalmanFilter.py:8,67), as the
 * last pekf_filter_update left it (work enqueued by pekf_filter_update_dev on another stream must be
 * synchronised by the caller first, as for pekf_filter_get_state). */
int pekf_filter_get_time(pekf_filter *f, int64_t *t_ns);
/* Device addresses of the state (layout per flags) and refs[batch*6], e.g. for a collective. */
int pekf_filter_device_state(pekf_filter *f, double **X, double **P, double **refs);
/* One record per filter, FP64: Prediction(gyro, t_ns) then Correction(mag, acc) (main_file.py:42-45),
 * dt = t_ns - previousT.  gyro/acc/mag [batch*3], t_ns [batch], mag_missing [batch] (NULL = none
 * missing; nonzero = Wahba-skip), X_out [batch*4] (NULL to skip).  Host pointers, synchronous. */
int pekf_filter_update(pekf_filter *f, const double *gyro, const int64_t *t_ns, const double *acc,
                       const double *mag, const uint8_t *mag_missing, double *X_out);
/* Same with device pointers, enqueued on `stream`. */
int pekf_filter_update_dev(pekf_filter *f, const double *gyro, const int64_t *t_ns, const double *acc,
                           const double *mag, const uint8_t *mag_missing, double *X_out, void *stream);
/* pekf_run_dev on the handle's state and references (stream planes, traj, counts as there). */
int pekf_filter_run(pekf_filter *f, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                    const void *plane_am, const void *plane_my, double *traj, const int32_t *counts,
                    void *stream);
/* pekf_run_ext_dev on the handle (dt_ext: the window's dt side plane, NULL = none). */
int pekf_filter_run_ext(pekf_filter *f, int64_t n_steps, int64_t window, int64_t step0, const void *plane_gd,
                        const void *plane_am, const void *plane_my, const double *dt_ext, double *traj,
                        const int32_t *counts, void *stream);

/* ---------------- synthetic IMU streams (device mirror of poseestimationkf_amd/synth.py) --------
 * Filters first_filter .. first_filter+batch-1, window steps, bit-identical to the host
 * generator.  scales[5] = sqrt(3)*sigma for {ref, w, gyro, acc, mag}; ar_w = AR(1) factor.
 * Writes the three planes ([window][batch]) and refs[batch*6]. */
int pekf_synth_dev(int64_t batch, int64_t window, int64_t first_filter, uint32_t seed,
                   int missing_mag, const double *scales, double ar_w, void *plane_gd,
                   void *plane_am, void *plane_my, double *refs, void *stream);

/* ---------------- sharding over GPUs: the one collective of the path ----------------
 * Filters are independent (ExtendedKalmanFilter.py:6-80 shares nothing between KalmanFilter objects),
 * so each GPU runs its own contiguous shard of the batch with no per-record exchange; the final
 * quaternions are gathered to the root by ONE RCCL gather over xGMI (ncclGather, rccl.h:745).
 * RCCL is loaded on first use (librccl.so.1; the copy already in the process if there is one).
 * Every collective call below must be made by all ranks of the communicator; PEKF_ERR_COMM reports
 * an RCCL failure or a missing librccl.
 *
 * One process per GPU: rank 0 makes an id, every rank receives it out of band (any channel:
 * a file, a TCP store, MPI) and calls pekf_comm_init on its current device.
 * One process for several GPUs: pekf_comm_init_all (ncclCommInitAll, rccl.h:236) gives one
 * communicator per device, driven from one host thread with pekf_gather_multi_dev. */
#define PEKF_COMM_ID_BYTES 128
typedef struct pekf_comm pekf_comm;
int pekf_comm_version(int *version); /* RCCL's version code, e.g. 22707 */
int pekf_comm_unique_id(void *id /* PEKF_COMM_ID_BYTES */);
/* Communicator creation has a deadline: ncclCommInitRank (rccl.h) runs on a helper thread and the call
 * waits for it at most PEKF_COMM_TIMEOUT_S seconds (environment; default 300).  If the other ranks do not
 * all join by then it returns PEKF_ERR_TIMEOUT, so a rank that died before joining fails the job instead
 * of hanging it.  The abandoned helper stays blocked inside RCCL until the process exits: after an init
 * timeout the PROCESS MUST EXIT (without its exit handlers, e.g. _exit); until then every later
 * pekf_comm_init* call fails at once with PEKF_ERR_COMM rather than reuse RCCL's bootstrap state.
 * (RCCL 2.27's non-blocking ncclCommInitRankConfig still blocks the caller while a rank is missing.) */
int pekf_comm_init(const void *id, int nranks, int rank, pekf_comm **out);
/* The same with an explicit deadline in seconds (<= 0: wait forever, the blocking behaviour). */
int pekf_comm_init_timeout(const void *id, int nranks, int rank, double timeout_s, pekf_comm **out);
/* devices: ndev device indices (NULL = 0 .. ndev-1); out: ndev communicators, rank i on devices[i].
 * ncclCommInitAll (rccl.h:236) under the same PEKF_COMM_TIMEOUT_S deadline and rules as pekf_comm_init. */
int pekf_comm_init_all(int ndev, const int *devices, pekf_comm **out);
/* The same with an explicit deadline in seconds (<= 0: none). */
int pekf_comm_init_all_timeout(int ndev, const int *devices, double timeout_s, pekf_comm **out);
int pekf_comm_destroy(pekf_comm *c);
/* Abort a communicator (ncclCommAbort: its kernels in flight give up) and free it; for error paths. */
int pekf_comm_abort(pekf_comm *c);
/* Wait until `stream` has drained everything enqueued on it, collectives of c included, watching c for
 * asynchronous RCCL errors meanwhile.  The deadline timeout_s (<= 0: none) applies to each collective of c
 * enqueued on `stream` (pekf_gather_dev, pekf_gather_multi_dev, pekf_allreduce_max_dev) and starts when the
 * stream reaches it -- the work queued before it has finished -- so compute ahead of a collective, however
 * long, is never charged to it.  On expiry or error c is aborted (it must then only be destroyed) and
 * PEKF_ERR_TIMEOUT / PEKF_ERR_COMM returned: a peer that died turns into an error here instead of a host
 * thread stuck in hipStreamSynchronize.
 * The clock starts when THIS rank's inputs are ready, so it also runs while slower peers finish the compute
 * queued ahead of the collective on their side: the deadline must exceed the ranks' skew at the
 * collective (bench.py's final gather follows the whole timed run; size PEKF_COMM_TIMEOUT_S to the run).
 * Every collective is tracked: at most 1,024 incomplete ones per communicator, one more is refused with
 * PEKF_ERR_COMM and not enqueued.  If a collective could not be tracked after it was enqueued (its
 * completion event could not be recorded), the drain of that stream is bounded by timeout_s from the
 * wait call instead, compute included. */
int pekf_comm_wait(pekf_comm *c, void *stream, double timeout_s);
int pekf_comm_rank(const pekf_comm *c, int *rank, int *nranks, int *device); /* outputs may be NULL */
/* recv[nranks * count] on the root (rows in rank order) <- every rank's send[count]; device
 * pointers, enqueued on stream.  recv is ignored (may be NULL) on the other ranks. */
int pekf_gather_dev(pekf_comm *c, const double *send, int64_t count, double *recv, int root, void *stream);
/* The same gather for the ndev communicators of pekf_comm_init_all, as one RCCL group:
 * send[i] / streams[i] belong to comms[i]'s device; recv is on comms[root]'s device. */
int pekf_gather_multi_dev(int ndev, pekf_comm *const *comms, const double *const *send, int64_t count,
                          double *recv, int root, void *const *streams);
/* buf[count] <- elementwise max over the ranks (in place), e.g. the slowest rank's wall time. */
int pekf_allreduce_max_dev(pekf_comm *c, double *buf, int64_t count, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PEKF_H */
