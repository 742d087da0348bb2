/*
 * ekf_oracle.c -- plain-C FP64 restatement of the reference EKF hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load this (as the checker / the timed CPU baseline).  The product
 * library (poseestimationkf_amd/libpekf.so) never links or calls it.
 *
 * It follows the reference operation by operation in dense form (compiled with
 * -ffp-contract=off, so no fused multiply-adds):
 *   oracle_jacobian_a   ExtendedKalmanFilter.py:43-48      0.5*Omega(w)
 *   oracle_jacobian_b   ExtendedKalmanFilter.py:51-56      0.5*Xi(q)
 *   oracle_rk4          ExtendedKalmanFilter.py:25-41      classical 4-stage RK4, dt = dt_ns*1e-9
 *   oracle_norm4        UtilityFunctions.py:16-21          sequential sum of squares
 *   oracle_predict      ExtendedKalmanFilter.py:58-68      P = A P A' + Jb Q Jb'; z = RK4; K = P inv(P+R)
 *   oracle_correct      ExtendedKalmanFilter.py:70-80      Wahba, hemisphere flip, X = z + K(Y-z), P -= K P
 *   oracle_wahba_rotation Wahba.py:8-17                    R = U diag(1,1,det U det V') V' of B
 *   oracle_rotm_to_quat Wahba.py:19-47                     3-branch, strict '>' ties
 *   oracle_run          main_file.py:19-47 loop over the packed record stream (+ Wahba-skip rule)
 * Paths are relative to "/root/reference/Python Kalman Filter/".
 *
 * np.linalg.svd is LAPACK (gesdd); here the SVD is a one-sided (Hestenes) Jacobi
 * iteration.  For the rank-2 B of Wahba.py:11-13 the rotation is unique, so any
 * accurate SVD gives the same R to rounding (pinned against the reference's own
 * outputs in tests/test_oracle_golden.py).  np.linalg.inv is LAPACK getrf/getri;
 * here Gauss-Jordan with partial pivoting.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define NS_TO_S 1e-09 /* ExtendedKalmanFilter.py:32, 10**-9 */

static void mat_mul(const double *a, const double *b, double *c, int n, int k, int m)
{
    /* c[n x m] = a[n x k] * b[k x m], row-major, sequential k summation */
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) {
            double s = 0.0;
            for (int t = 0; t < k; ++t) s += a[i * k + t] * b[t * m + j];
            c[i * m + j] = s;
        }
}

static void mat_transpose(const double *a, double *at, int n, int m)
{
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) at[j * n + i] = a[i * m + j];
}

void oracle_jacobian_a(const double w[3], double A[16])
{
    const double m[16] = {0.0, -w[0], -w[1], -w[2],
                          w[0], 0.0, w[2], -w[1],
                          w[1], -w[2], 0.0, w[0],
                          w[2], w[1], -w[0], 0.0};
    for (int i = 0; i < 16; ++i) A[i] = 0.5 * m[i];
}

void oracle_jacobian_b(const double q[4], double J[12])
{
    const double m[12] = {-q[1], -q[2], -q[3],
                          q[0], q[3], -q[2],
                          -q[3], q[0], q[1],
                          q[2], -q[1], q[0]};
    for (int i = 0; i < 12; ++i) J[i] = 0.5 * m[i];
}

double oracle_norm4(const double a[4])
{
    double s = 0.0;
    for (int i = 0; i < 4; ++i) s += a[i] * a[i];
    return sqrt(s);
}

void oracle_rk4(const double q0[4], double dt_ns, const double w[3], double out[4])
{
    double W[16], k1[4], k2[4], k3[4], k4[4], tmp[4];
    oracle_jacobian_a(w, W);
    const double h = dt_ns * NS_TO_S;
    mat_mul(W, q0, k1, 4, 4, 1);
    for (int i = 0; i < 4; ++i) tmp[i] = q0[i] + h / 2 * k1[i];
    mat_mul(W, tmp, k2, 4, 4, 1);
    for (int i = 0; i < 4; ++i) tmp[i] = q0[i] + h / 2 * k2[i];
    mat_mul(W, tmp, k3, 4, 4, 1);
    for (int i = 0; i < 4; ++i) tmp[i] = q0[i] + h * k3[i];
    mat_mul(W, tmp, k4, 4, 4, 1);
    const double c = 1.0 / 6.0 * h;
    for (int i = 0; i < 4; ++i) out[i] = q0[i] + c * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
    const double n = oracle_norm4(out);
    for (int i = 0; i < 4; ++i) out[i] = out[i] / n;
}

/* Gauss-Jordan inverse with partial pivoting; returns 0 on success, 1 if singular. */
int oracle_inv4(const double S[16], double inv[16])
{
    double a[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) a[i][j] = j < 4 ? S[i * 4 + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int p = c;
        for (int r = c + 1; r < 4; ++r)
            if (fabs(a[r][c]) > fabs(a[p][c])) p = r;
        if (a[p][c] == 0.0) return 1;
        if (p != c)
            for (int j = 0; j < 8; ++j) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
        const double d = a[c][c];
        for (int j = 0; j < 8; ++j) a[c][j] /= d;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            const double f = a[r][c];
            if (f == 0.0) continue;
            for (int j = 0; j < 8; ++j) a[r][j] -= f * a[c][j];
        }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) inv[i * 4 + j] = a[i][j + 4];
    return 0;
}

int oracle_predict(const double gyro[3], double dt_ns, const double X[4], const double P[16],
                   const double Q[9], const double R[16], double z[4], double Pm[16], double K[16])
{
    double A[16], At[16], Jb[12], Jbt[12], t16[16], a16[16], t12[12], b16[16], S[16], Si[16];
    oracle_jacobian_a(gyro, A);
    oracle_jacobian_b(X, Jb);
    mat_transpose(A, At, 4, 4);
    mat_transpose(Jb, Jbt, 4, 3);
    mat_mul(A, P, t16, 4, 4, 4);
    mat_mul(t16, At, a16, 4, 4, 4);
    mat_mul(Jb, Q, t12, 4, 3, 3);
    mat_mul(t12, Jbt, b16, 4, 3, 4);
    for (int i = 0; i < 16; ++i) Pm[i] = a16[i] + b16[i];
    oracle_rk4(X, dt_ns, gyro, z);
    for (int i = 0; i < 16; ++i) S[i] = Pm[i] + R[i];
    if (oracle_inv4(S, Si)) return 1;
    mat_mul(Pm, Si, K, 4, 4, 4);
    return 0;
}

/* ---- 3x3 SVD by one-sided Jacobi (Hestenes) ---------------------------------------- */
static double det3(const double m[9])
{
    return m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
           m[2] * (m[3] * m[7] - m[4] * m[6]);
}

static void svd3(const double B[9], double U[9], double s[3], double V[9])
{
    double a[9], v[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    memcpy(a, B, sizeof(a));
    for (int sweep = 0; sweep < 60; ++sweep) {
        int rotated = 0;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < 3; ++i) {
                    al += a[i * 3 + p] * a[i * 3 + p];
                    be += a[i * 3 + q] * a[i * 3 + q];
                    ga += a[i * 3 + p] * a[i * 3 + q];
                }
                if (ga == 0.0 || fabs(ga) <= 1e-17 * sqrt(al * be)) continue;
                rotated = 1;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                for (int i = 0; i < 3; ++i) {
                    const double x = a[i * 3 + p], y = a[i * 3 + q];
                    a[i * 3 + p] = c * x - sn * y;
                    a[i * 3 + q] = sn * x + c * y;
                    const double vx = v[i * 3 + p], vy = v[i * 3 + q];
                    v[i * 3 + p] = c * vx - sn * vy;
                    v[i * 3 + q] = sn * vx + c * vy;
                }
            }
        if (!rotated) break;
    }
    double n[3];
    int order[3] = {0, 1, 2};
    for (int j = 0; j < 3; ++j)
        n[j] = sqrt(a[j] * a[j] + a[3 + j] * a[3 + j] + a[6 + j] * a[6 + j]);
    for (int i = 0; i < 3; ++i) /* sort descending */
        for (int j = i + 1; j < 3; ++j)
            if (n[order[j]] > n[order[i]]) { int t = order[i]; order[i] = order[j]; order[j] = t; }
    for (int k = 0; k < 3; ++k) {
        const int j = order[k];
        s[k] = n[j];
        for (int i = 0; i < 3; ++i) {
            V[i * 3 + k] = v[i * 3 + j];
            U[i * 3 + k] = n[j] > 0 ? a[i * 3 + j] / n[j] : 0.0;
        }
    }
    /* B = sum of two outer products has rank <= 2: complete U by u3 = u1 x u2. */
    const double tol = 1e-14 * s[0];
    if (!(s[2] > tol)) {
        U[2] = U[3] * U[7] - U[6] * U[4];
        U[5] = U[6] * U[1] - U[0] * U[7];
        U[8] = U[0] * U[4] - U[3] * U[1];
    }
}

void oracle_wahba_rotation(const double acc0[3], const double mag0[3], const double acc[3],
                           const double mag[3], double k_acc, double k_mag, double Rout[9])
{
    double B[9], U[9], s[3], V[9], Vt[9], M[9] = {0}, t9[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            B[i * 3 + j] = k_acc * (acc0[i] * acc[j]) + k_mag * (mag0[i] * mag[j]);
    svd3(B, U, s, V);
    mat_transpose(V, Vt, 3, 3);
    M[0] = 1.0;
    M[4] = 1.0;
    M[8] = det3(U) * det3(Vt);
    mat_mul(U, M, t9, 3, 3, 3);
    mat_mul(t9, Vt, Rout, 3, 3, 3);
}

void oracle_rotm_to_quat(const double M[9], double q[4])
{
    const double t1 = 1.0 + M[0] - M[4] - M[8];
    const double t2 = 1.0 - M[0] + M[4] - M[8];
    const double t3 = 1.0 - M[0] - M[4] + M[8];
    if (t1 > t2 && t1 > t3) {
        const double S = sqrt(t1) * 2;
        q[0] = (M[7] - M[5]) / S; q[1] = 0.25 * S; q[2] = (M[1] + M[3]) / S; q[3] = (M[2] + M[6]) / S;
    } else if (t2 > t1 && t2 > t3) {
        const double S = sqrt(t2) * 2;
        q[0] = (M[2] - M[6]) / S; q[1] = (M[1] + M[3]) / S; q[2] = 0.25 * S; q[3] = (M[5] + M[7]) / S;
    } else {
        const double S = sqrt(t3) * 2;
        q[0] = (M[3] - M[1]) / S; q[1] = (M[2] + M[6]) / S; q[2] = (M[5] + M[7]) / S; q[3] = 0.25 * S;
    }
}

void oracle_wahba_quat(const double acc0[3], const double mag0[3], const double acc[3],
                       const double mag[3], double k_acc, double k_mag, double q[4])
{
    double R[9];
    oracle_wahba_rotation(acc0, mag0, acc, mag, k_acc, k_mag, R);
    oracle_rotm_to_quat(R, q);
}

void oracle_correct(const double mag[3], const double acc[3], const double z[4], const double P[16],
                    const double K[16], const double acc0[3], const double mag0[3], double X[4],
                    double Pout[16])
{
    double y[4], e[4], ke[4], kp[16];
    const double ka = fabs(acc[2]);
    oracle_wahba_quat(acc0, mag0, acc, mag, ka, 1 - ka, y);
    /* Comparator(y, z)[0] = conj(y) (x) z, scalar part (ExtendedKalmanFilter.py:16-23,73) */
    const double cmp = y[0] * z[0] + y[1] * z[1] + y[2] * z[2] + y[3] * z[3];
    if (cmp < 0.0)
        for (int i = 0; i < 4; ++i) y[i] = -y[i];
    for (int i = 0; i < 4; ++i) e[i] = y[i] - z[i];
    mat_mul(K, e, ke, 4, 4, 1);
    for (int i = 0; i < 4; ++i) X[i] = z[i] + ke[i];
    mat_mul(K, P, kp, 4, 4, 4);
    for (int i = 0; i < 16; ++i) Pout[i] = P[i] - kp[i];
    const double n = oracle_norm4(X);
    for (int i = 0; i < 4; ++i) X[i] = X[i] / n;
}

/*
 * Run filters over a packed per-filter record stream (the layout of synth.Records):
 *   rec[f][t] = {gx,gy,gz, ax,ay,az, mx,my,mz} as float, dtw[f][t] = dt_ns | (missing << 31)
 * A dt field of all ones (0x7FFFFFFF, the stream's escape) takes the record's dt from the float64
 * side plane dtx[f][t] (may be NULL when no record is escaped): any T - previousT, as at
 * ExtendedKalmanFilter.py:62.
 * Step t of the run reads record (step0 + t) % window.  X[f][4], P[f][16] in/out.
 * traj (optional, may be NULL): traj[f][t][4].
 */
int oracle_run(int64_t n_filters, int64_t n_steps, int64_t window, int64_t step0,
               const float *rec, const uint32_t *dtw, const double *dtx, const double *acc0, const double *mag0,
               double q, double r, double *X, double *P, double *traj)
{
    int status = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(| : status)
    for (int64_t f = 0; f < n_filters; ++f) {
        double Q[9] = {0}, R[16] = {0}, x[4], p[16], z[4], pm[16], k[16];
        for (int i = 0; i < 3; ++i) Q[i * 4] = q;
        for (int i = 0; i < 4; ++i) R[i * 5] = r;
        memcpy(x, X + f * 4, sizeof(x));
        memcpy(p, P + f * 16, sizeof(p));
        for (int64_t t = 0; t < n_steps; ++t) {
            const int64_t row = (step0 + t) % window;
            const float *rc = rec + (f * window + row) * 9;
            const uint32_t word = dtw[f * window + row];
            const double g[3] = {rc[0], rc[1], rc[2]};
            const double a[3] = {rc[3], rc[4], rc[5]};
            const double m[3] = {rc[6], rc[7], rc[8]};
            const double dt = ((word & 0x7FFFFFFFu) == 0x7FFFFFFFu && dtx) ? dtx[f * window + row]
                                                                            : (double)(word & 0x7FFFFFFFu);
            if (oracle_predict(g, dt, x, p, Q, R, z, pm, k)) { status |= 1; break; }
            if (word & 0x80000000u) {
                memcpy(x, z, sizeof(x));
                memcpy(p, pm, sizeof(p));
            } else {
                oracle_correct(m, a, z, pm, k, acc0 + f * 3, mag0 + f * 3, x, p);
            }
            if (traj) memcpy(traj + (f * n_steps + t) * 4, x, sizeof(x));
        }
        memcpy(X + f * 4, x, sizeof(x));
        memcpy(P + f * 16, p, sizeof(p));
    }
    return status;
}
