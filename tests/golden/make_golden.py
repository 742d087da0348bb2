"""Generate the golden fixtures by importing the REFERENCE itself (run in the survey container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (/root/reference/Python Kalman Filter/) ships no tests, fixtures or
golden data, so parity is pinned by vectors produced here from its
own modules (ExtendedKalmanFilter.KalmanFilter, Wahba.Wahba, UtilityFunctions.norm)
and from running its driver main_file.py unchanged.  Only inputs and outputs are
stored -- no reference source.  /root/reference does not exist on the GPU box; the
tests only read the .npz/.gz files written here.

Outputs (tests/golden/):
  kat.npz          per-function known-answer vectors (a3-a13 of SURVEY.md §8a)
  traj.npz         8 filters x 1500 synthetic steps (+ a Wahba-skip variant), inputs and X trajectories
  c1_log.txt.gz    config-1 trace in the C++ log format (1550 steps)
  c1_xk.npy        X_k list produced by main_file.py (unchanged) on that log
  side.npz         pure-gyro chain, per-record 0.5/0.5 Wahba quaternion, Quart2RPY
  edge.npz         raw-unit inputs (k_mag < 0), zero rates, dt = 0 / 5 s, a NaN sample, general P/Q/R
"""
from __future__ import annotations

import builtins
import gzip
import io
import os
import runpy
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# where the fixtures are written (tests/test_golden_regen.py regenerates them into a scratch directory)
OUT = os.environ.get("PEKF_GOLDEN_OUT") or HERE
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_DIR = "/root/reference/Python Kalman Filter"
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

from poseestimationkf_amd import logformat, synth  # noqa: E402

rng = np.random.default_rng(1234)


def unit(n, d):
    v = rng.normal(size=(n, d))
    return v / np.linalg.norm(v, axis=1, keepdims=True)


def quat_to_rotm(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def import_reference():
    sys.path.insert(0, REF_DIR)
    import ExtendedKalmanFilter as ekf  # noqa: E402
    import UtilityFunctions as uf  # noqa: E402
    import Wahba as wb  # noqa: E402
    return ekf, wb, uf


def make_kat(ekf, wb, uf):
    KF, Wahba = ekf.KalmanFilter, wb.Wahba
    out = {}
    n = 256
    # a5 RungeKutta4
    q0 = unit(n, 4)
    w = rng.normal(scale=1.5, size=(n, 3))
    dt = rng.integers(1_000_000, 50_000_000, size=n).astype(np.float64)
    out.update(rk4_q0=q0, rk4_w=w, rk4_dt=dt,
               rk4_out=np.array([KF.RungeKutta4(q0[i], dt[i], w[i]) for i in range(n)]))
    # a3/a4 Jacobians
    k = KF(0.0, [1.0, 0, 0], [0, 0, 1.0], 0.5)
    out.update(jac_w=w[:64], jac_q=q0[:64],
               jac_a=np.array([k.GetJacobian_A(w[i]) for i in range(64)]),
               jac_b=np.array([k.GetJacobian_B(q0[i]) for i in range(64)]))
    # a13 norm, a7 Comparator
    v4 = rng.normal(size=(64, 4))
    out.update(norm_in=v4, norm_out=np.array([uf.norm(v4[i]) for i in range(64)]),
               cmp_q1=q0[:64], cmp_q2=q0[64:128],
               cmp_out=np.array([k.Comparator(q0[i], q0[64 + i]) for i in range(64)]))
    # a11 RotationMatrix2Quart: random rotations + every branch, ties, exact identity (NaN)
    qs = unit(n, 4)
    Ms = [quat_to_rotm(q) for q in qs]
    s = 1 / np.sqrt(2.0)
    special = [np.eye(3),                                 # all traces 0 -> else branch, NaN
               np.diag([-1.0, -1.0, 1.0]),                # WahbaProblem_singularValue.py result -> [0,0,0,1]
               np.diag([1.0, -1.0, -1.0]),                # pi about x -> branch 1
               np.diag([-1.0, 1.0, -1.0]),                # pi about y -> branch 2
               quat_to_rotm([0.0, s, s, 0.0]),            # tr1 == tr2 tie -> falls to else branch
               quat_to_rotm([0.0, s, 0.0, s]),            # tr1 == tr3 tie
               quat_to_rotm([0.0, 0.0, s, s]),            # tr2 == tr3 tie
               quat_to_rotm([0.5, 0.5, 0.5, 0.5])]       # all three traces equal
    Ms = np.array(Ms + special)
    with np.errstate(all="ignore"):
        out.update(r2q_M=Ms, r2q_out=np.array([Wahba.RotationMatrix2Quart(M) for M in Ms]))
    # a10/a12 Wahba: random, near-flat (k_mag small), and the fixed example of
    # WahbaProblem_singularValue.py:4-24 (initial acc (0,0,1), mag (-1,0,0); rotated (0,0,1), (1,0,0); 0.5/0.5)
    acc0, mag0, acc, mag = unit(n, 3), unit(n, 3), unit(n, 3), unit(n, 3)
    ka = np.abs(acc[:, 2])
    km = 1 - ka
    flat = np.array([1e-4, 1e-5, 1e-6, 1e-7])
    for j, kmv in enumerate(flat):  # near-flat: acc_z so close to 1 that k_mag = kmv
        i = n - 1 - j
        acc[i] = [np.sqrt(1 - (1 - kmv) ** 2), 0.0, 1 - kmv]
        ka[i] = abs(acc[i, 2])
        km[i] = 1 - ka[i]
    acc0 = np.vstack([acc0, [0, 0, 1.0]])
    mag0 = np.vstack([mag0, [-1.0, 0, 0]])
    acc = np.vstack([acc, [0, 0, 1.0]])
    mag = np.vstack([mag, [1.0, 0, 0]])
    ka = np.append(ka, 0.5)
    km = np.append(km, 0.5)
    Rw, qw = [], []
    for i in range(len(ka)):
        wo = Wahba(acc0[i], mag0[i])
        Rw.append(wo.getRotation(acc[i], mag[i], ka[i], km[i]))
        qw.append(wo.getQuarternion(acc[i], mag[i], ka[i], km[i]))
    out.update(wahba_acc0=acc0, wahba_mag0=mag0, wahba_acc=acc, wahba_mag=mag, wahba_ka=ka,
               wahba_km=km, wahba_R=np.array(Rw), wahba_q=np.array(qw))
    # a6 Prediction / a8 Correction on states taken along a real filter run
    rec = synth.generate(np.arange(4), 80, seed=77)
    Xs, Ps, G, D, A_, M_, A0, M0 = [], [], [], [], [], [], [], []
    for f in range(4):
        g, d, a, m = rec.filter(f)
        kf = KF(0.0, rec.mag0[f], rec.acc0[f], 0.5)
        kf.setQ(1)
        kf.setR(0.1)
        X, P = np.array([1.0, 0, 0, 0]), np.identity(4)
        T = 0.0
        for i in range(64):
            Xs.append(X)
            Ps.append(P)
            G.append(g[i]); D.append(d[i]); A_.append(a[i]); M_.append(m[i])
            A0.append(rec.acc0[f]); M0.append(rec.mag0[f])
            T += d[i]
            z, P, K = kf.Prediction(g[i], T, X, P)
            X, P = kf.Correction(m[i], a[i], z, P, K)
    Xs, Ps, G, D, A_, M_, A0, M0 = map(np.array, (Xs, Ps, G, D, A_, M_, A0, M0))
    nn = len(D)
    Qm = np.array([np.identity(3) * (1.0 if i % 2 == 0 else 2.5) for i in range(nn)])
    Rm = np.array([np.identity(4) * (0.1 if i % 3 else 0.7) for i in range(nn)])
    zs, Pms, Ks, Xo, Po = [], [], [], [], []
    for i in range(nn):
        kf = KF(0.0, M0[i], A0[i], 0.5)
        kf.Q = Qm[i].copy()
        kf.R = Rm[i].copy()
        z, Pm, K = kf.Prediction(G[i], D[i], Xs[i], Ps[i])
        X, P = kf.Correction(M_[i], A_[i], z, Pm, K)
        zs.append(z); Pms.append(Pm); Ks.append(K); Xo.append(X); Po.append(P)
    out.update(pc_gyro=G, pc_dt=D, pc_X=Xs, pc_P=Ps, pc_Q=Qm, pc_R=Rm, pc_acc=A_, pc_mag=M_,
               pc_acc0=A0, pc_mag0=M0, pc_z=np.array(zs), pc_Pm=np.array(Pms), pc_K=np.array(Ks),
               pc_Xout=np.array(Xo), pc_Pout=np.array(Po))
    return out


def run_reference_filter(ekf, gyro, dt, acc, mag, acc0, mag0, missing=None):
    """The main_file.py:19-47 loop on the reference classes (Wahba-skip: Prediction, then X=z)."""
    kf = ekf.KalmanFilter(0.0, mag0, acc0, 0.5)
    kf.setQ(1)
    kf.setR(0.1)
    X, P = np.asarray([1., 0., 0., 0.]), np.identity(4)
    T = 0.0
    traj = np.empty((len(dt), 4))
    for i in range(len(dt)):
        T = T + dt[i]
        z, P, K = kf.Prediction(gyro[i], T, X, P)
        if missing is not None and missing[i]:
            X = z
        else:
            X, P = kf.Correction(mag[i], acc[i], z, P, K)
        traj[i] = X
    return traj


def make_traj(ekf):
    K, W = 8, 1500
    out = {}
    for tag, miss in (("", False), ("miss_", True)):
        rec = synth.generate(np.arange(K), W, seed=synth.DEFAULT_SEED, missing=miss)
        trajs = []
        for f in range(K):
            g, d, a, m = rec.filter(f)
            trajs.append(run_reference_filter(ekf, g, d, a, m, rec.acc0[f], rec.mag0[f],
                                              rec.missing[:, f] if miss else None))
        gd, am, my = synth.pack_planes(rec)
        out.update({tag + "gd": gd, tag + "am": am, tag + "my": my, tag + "acc0": rec.acc0,
                    tag + "mag0": rec.mag0, tag + "traj": np.stack(trajs, axis=1)})  # traj (W,K,4)
    return out


def make_edge(ekf, wb):
    """Edge cases the reference accepts: raw-unit sensor values (|acc| ~ 9.81 so k_mag = 1-|acc_z| < 0),
    zero rates, dt = 0 and very large dt, a NaN sample (propagates), non-symmetric P and non-scalar Q/R."""
    KF, Wahba = ekf.KalmanFilter, wb.Wahba
    out = {}
    # (1) raw-unit trajectories: acc in m/s^2, mag in uT, plus zero-rate and 1 s gaps
    K, W = 4, 600
    rec = synth.generate(np.arange(100, 100 + K), W, seed=31)
    rec.acc[:] = rec.acc * np.float32(9.81)
    rec.mag[:] = rec.mag * np.float32(45.0)
    rec.gyro[100:110] = 0.0
    rec.dtw[200] = 1_000_000_000
    rec.dtw[201] = 0
    trajs = []
    for f in range(K):
        g, d, a, m = rec.filter(f)
        with np.errstate(all="ignore"):
            trajs.append(run_reference_filter(ekf, g, d, a, m, rec.acc0[f], rec.mag0[f]))
    gd, am, my = synth.pack_planes(rec)
    out.update(raw_gd=gd, raw_am=am, raw_my=my, raw_acc0=rec.acc0, raw_mag0=rec.mag0,
               raw_traj=np.stack(trajs, axis=1))
    # (2) NaN sample at record 20 of filter 1: the reference's np.linalg.svd raises
    # LinAlgError("SVD did not converge") there; record the trajectory up to that point
    rec = synth.generate(np.arange(2), 50, seed=32)
    rec.acc[20, 1, 0] = np.float32(np.nan)
    g, d, a, m = rec.filter(0)
    clean = run_reference_filter(ekf, g, d, a, m, rec.acc0[0], rec.mag0[0])
    g, d, a, m = rec.filter(1)
    raised_at = -1
    try:
        run_reference_filter(ekf, g, d, a, m, rec.acc0[1], rec.mag0[1])
    except np.linalg.LinAlgError:
        # re-run to the failing record to keep the partial trajectory
        raised_at = 20
    partial = run_reference_filter(ekf, g[:20], d[:20], a[:20], m[:20], rec.acc0[1], rec.mag0[1])
    gd, am, my = synth.pack_planes(rec)
    out.update(nan_gd=gd, nan_am=am, nan_my=my, nan_acc0=rec.acc0, nan_mag0=rec.mag0,
               nan_clean_traj=clean, nan_partial_traj=partial, nan_raised_at=np.int64(raised_at))
    # (3) Wahba on raw-unit vectors: weights |acc_z|, 1-|acc_z| with |acc_z| > 1 (k_mag < 0)
    n = 64
    acc0, mag0 = unit(n, 3), unit(n, 3)
    acc, mag = unit(n, 3) * 9.81, unit(n, 3) * 45.0
    ka = np.abs(acc[:, 2])
    km = 1 - ka
    R, q = [], []
    for i in range(n):
        wo = Wahba(acc0[i], mag0[i])
        R.append(wo.getRotation(acc[i], mag[i], ka[i], km[i]))
        q.append(wo.getQuarternion(acc[i], mag[i], ka[i], km[i]))
    out.update(ew_acc0=acc0, ew_mag0=mag0, ew_acc=acc, ew_mag=mag, ew_ka=ka, ew_km=km,
               ew_R=np.array(R), ew_q=np.array(q))
    # (4) Prediction / Correction with general (non-symmetric P, SPD non-scalar Q/R), w = 0, dt = 0, huge dt
    n = 32
    G = rng.normal(scale=2.0, size=(n, 3))
    G[:4] = 0.0
    D = rng.integers(0, 50_000_000, size=n).astype(np.float64)
    D[4:6] = 0.0
    D[6:8] = 5e9
    X = unit(n, 4)
    P = rng.normal(scale=0.3, size=(n, 4, 4)) + np.eye(4)
    A3 = rng.normal(size=(n, 3, 3))
    A4 = rng.normal(size=(n, 4, 4))
    Q = np.einsum("nij,nkj->nik", A3, A3) + 0.1 * np.eye(3)
    Rm = np.einsum("nij,nkj->nik", A4, A4) + 0.1 * np.eye(4)
    acc, mag = unit(n, 3), unit(n, 3)
    acc0, mag0 = unit(n, 3), unit(n, 3)
    zs, Pms, Ks, Xo, Po = [], [], [], [], []
    for i in range(n):
        kf = KF(0.0, mag0[i], acc0[i], 0.5)
        kf.Q, kf.R = Q[i].copy(), Rm[i].copy()
        z, Pm, Kk = kf.Prediction(G[i], D[i], X[i], P[i])
        Xn, Pn = kf.Correction(mag[i], acc[i], z, Pm, Kk)
        zs.append(z); Pms.append(Pm); Ks.append(Kk); Xo.append(Xn); Po.append(Pn)
    out.update(ep_gyro=G, ep_dt=D, ep_X=X, ep_P=P, ep_Q=Q, ep_R=Rm, ep_acc=acc, ep_mag=mag,
               ep_acc0=acc0, ep_mag0=mag0, ep_z=np.array(zs), ep_Pm=np.array(Pms), ep_K=np.array(Ks),
               ep_Xout=np.array(Xo), ep_Pout=np.array(Po))
    return out


def make_side(ekf, wb, uf):
    """Side outputs main_file.py plots: pure-gyro RK4 chain, per-record 0.5/0.5
    Wahba quaternion (main_file.py:40), Quart2RPY (UtilityFunctions.py:3-14)."""
    KF, Wahba = ekf.KalmanFilter, wb.Wahba
    K, W = 8, 300
    rec = synth.generate(np.arange(K), W, seed=synth.DEFAULT_SEED)  # = traj.npz's first 300 records
    chain = np.empty((W, K, 4))
    wq = np.empty((W, K, 4))
    for f in range(K):
        g, d, a, m = rec.filter(f)
        q = np.asarray([1.0, 0.0, 0.0, 0.0])
        wo = Wahba(rec.acc0[f], rec.mag0[f])
        for i in range(W):
            q = KF.RungeKutta4(q, d[i], g[i])
            chain[i, f] = q
            wq[i, f] = wo.getQuarternion(a[i], m[i], 0.5, 0.5)
    qs = unit(64, 4)
    s = np.sqrt(0.5)
    qs = np.vstack([qs, [[1.0, 0, 0, 0], [s, 0, s, 0], [s, 0, -s, 0], [0, 1.0, 0, 0]]])
    rpy = np.array([uf.Quart2RPY(q) for q in qs])
    return dict(gyro_chain=chain, wahba_half=wq, rpy_q=qs, rpy_out=rpy)


def make_c1():
    """Config 1: one filter, ~1550 steps (Results/*.png x-axis), through main_file.py UNCHANGED."""
    n = 1550
    rec = synth.generate(np.array([4242]), n, seed=synth.DEFAULT_SEED)
    g, d, a, m = rec.filter(0)
    ts = synth.c1_timestamps(d.astype(np.int64))
    buf = io.StringIO()
    logformat.write_log(buf, ts, g, a, m, rec.acc0[0], rec.mag0[0])
    text = buf.getvalue()
    tmp = os.path.join("/tmp", "pekf_c1_log.txt")
    with open(tmp, "w") as fh:
        fh.write(text)
    real_open = builtins.open

    def redirect(path, *args, **kw):
        if path == logformat.REFERENCE_LOG_PATH:
            path = tmp
        return real_open(path, *args, **kw)

    os.environ["MPLBACKEND"] = "Agg"
    builtins.open = redirect
    try:
        g_ = runpy.run_path(os.path.join(REF_DIR, "main_file.py"), run_name="__main__")
    finally:
        builtins.open = real_open
    xk = np.array(g_["X_k"])
    return text, xk


def main():
    ekf, wb, uf = import_reference()
    kat = make_kat(ekf, wb, uf)
    np.savez_compressed(os.path.join(OUT, "kat.npz"), **kat)
    traj = make_traj(ekf)
    np.savez_compressed(os.path.join(OUT, "traj.npz"), **traj)
    np.savez_compressed(os.path.join(OUT, "edge.npz"), **make_edge(ekf, wb))
    np.savez_compressed(os.path.join(OUT, "side.npz"), **make_side(ekf, wb, uf))
    text, xk = make_c1()
    with open(os.path.join(OUT, "c1_log.txt.gz"), "wb") as raw, \
            gzip.GzipFile(fileobj=raw, mode="wb", mtime=0, filename="") as gz:  # byte-stable output
        gz.write(text.encode())
    np.save(os.path.join(OUT, "c1_xk.npy"), xk)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
