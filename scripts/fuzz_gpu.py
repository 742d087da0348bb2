#!/usr/bin/env python3
"""Randomised parity sweep of the fused stream kernel against the C oracle (GPU box).

Each case draws a batch (1-300 filters), a window (1-48 rows) and a run of 1-3 windows' worth of
records, cut into launches of random length at a random start row (launches of one record take the
online instantiation, longer ones the multi-record kernel; the rows wrap in the window).  It also
draws per-launch record counts, trajectory output, AoS or SoA state, FP64 or mixed precision, the
batched engine or the native filter handle, a random initial state, q and r, dt gaps up to 2 s,
missing magnetometer samples and escaped dts (negative, 2^31 ns and more, fractional).  Every
filter's expected state is the oracle run over exactly the records that filter applied, in order
(oracle/oracle_c.py, ExtendedKalmanFilter.py:58-80 as main_file.py:42-45 calls it).

Degenerate samples (zero or parallel acc / mag) are not drawn: there the reference's attitude is its
SVD's noise-chosen rotation and parity is a different property (tests/test_degenerate_samples.py).

usage: python3 scripts/fuzz_gpu.py [--cases N] [--seed S]   (exit status 1 on any mismatch)
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ekf_numpy, oracle_c  # noqa: E402  (the checkers)
from poseestimationkf_amd import engine, synth  # noqa: E402

TOL_F64 = 1e-9      # |X - X_oracle|, and |P - P_oracle| / max(1, r, max|P_oracle|): the FP64 path
TOL_MIXED_X = 2e-5  # the opt-in mixed-precision path (covariance in f32)
# A case whose covariance grows past this (long runs of Prediction-only records with large |w| dt:
# GetJacobian_A is not orthogonal, so P- grows by |A|^2 per record) is ill-conditioned: there the
# gain K = P-(P- + rI)^-1 rounds to I and X follows rounding noise.  Such cases, and those where
# the oracle finds S singular, are counted and not compared.
P_WELL = 1e6
# Where a single record is ill-conditioned in the reference's own arithmetic (e.g. RotationMatrix2Quart
# dividing by a small S), the two restatements of the reference -- the C oracle and the NumPy one,
# which differ only in rounding -- disagree too.  A filter beyond TOL_F64 is accepted when its error
# is within SPREAD x that disagreement, record by record, and reported as such.
SPREAD = 10.0


def _unit(rng, shape):
    v = rng.normal(size=shape)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def draw_case(rng):
    K = int(rng.integers(1, 301))
    W = int(rng.integers(1, 49))
    n_total = int(rng.integers(1, 3 * W + 1))
    dt_max = int(rng.choice([2, 20_000_000, 2_000_000_000]))
    gyro = rng.normal(scale=float(rng.choice([0.1, 1.0, 3.0])), size=(W, K, 3)).astype(np.float32)
    acc = (_unit(rng, (W, K, 3)) * rng.uniform(0.5, 12.0) + rng.normal(scale=0.02, size=(W, K, 3))).astype(np.float32)
    mag = (_unit(rng, (W, K, 3)) * rng.uniform(0.5, 60.0) + rng.normal(scale=0.02, size=(W, K, 3))).astype(np.float32)
    dtw = rng.integers(0, dt_max, size=(W, K), dtype=np.uint32)
    dtx = None
    if rng.random() < 0.3:  # escaped dts: the float64 side plane
        esc = rng.random((W, K)) < 0.2
        vals = rng.choice([-1.5e9, -37.0, 2.0 ** 31, 5.5e9, 1234.5, 0.25], size=(W, K))
        dtx = np.where(esc, vals, 0.0)
        dtw = np.where(esc, np.uint32(synth.DT_ESCAPE), dtw).astype(np.uint32)
    miss_p = float(rng.choice([0.0, 0.3, 0.9]))
    dtw |= np.where(rng.random((W, K)) < miss_p, np.uint32(synth.MISSING_BIT), np.uint32(0))
    rec = synth.Records(gyro, acc, mag, dtw, _unit(rng, (K, 3)) * rng.uniform(0.5, 12.0),
                        _unit(rng, (K, 3)) * rng.uniform(0.5, 60.0), dtx)
    # launches: random lengths summing to n_total, starting at a random row
    cuts = np.sort(rng.choice(np.arange(1, n_total), size=min(int(rng.integers(0, 4)), n_total - 1), replace=False))
    lens = np.diff(np.concatenate([[0], cuts, [n_total]])).astype(int)
    s = int(rng.integers(0, W))
    launches = []
    for L in lens:
        counts = rng.integers(0, L + 2, size=K).astype(np.int32) if rng.random() < 0.3 else None
        launches.append((s % W, int(L), counts, bool(rng.random() < 0.4)))
        s += int(L)
    X0 = P0 = None
    if rng.random() < 0.5:
        X0 = _unit(rng, (K, 4)) * rng.uniform(0.5, 2.0, size=(K, 1))
        A = rng.normal(scale=0.3, size=(K, 4, 4))
        P0 = A @ A.transpose(0, 2, 1) + 0.05 * np.eye(4)
    return dict(rec=rec, launches=launches, X0=X0, P0=P0, K=K, W=W,
                q=float(rng.choice([1.0, 0.25, 3.0])), r=float(rng.choice([0.1, 0.02, 1.5])),
                layout=str(rng.choice(["aos", "soa"])), precision="mixed" if rng.random() < 0.2 else "f64",
                handle=bool(rng.random() < 0.25))


def expected(case):
    """Per filter: the oracle over exactly the records it applied; trajectories per launch."""
    rec, K, W = case["rec"], case["K"], case["W"]
    X = np.tile([1.0, 0.0, 0.0, 0.0], (K, 1)) if case["X0"] is None else case["X0"].copy()
    P = np.tile(np.eye(4), (K, 1, 1)) if case["P0"] is None else case["P0"].copy()
    trajs = []
    for s, L, counts, want in case["launches"]:
        tr = np.empty((L, K, 4)) if want else None
        for b in range(K):
            c = L if counts is None else min(int(counts[b]), L)
            if c > 0:
                rows = (s + np.arange(c)) % W
                sub = synth.Records(rec.gyro[rows, b:b + 1], rec.acc[rows, b:b + 1], rec.mag[rows, b:b + 1],
                                    rec.dtw[rows, b:b + 1], rec.acc0[b:b + 1], rec.mag0[b:b + 1],
                                    None if rec.dtx is None else rec.dtx[rows, b:b + 1])
                Xb, Pb, tb = oracle_c.run(sub, q=case["q"], r=case["r"], X=X[b:b + 1], P=P[b:b + 1], want_traj=want)
                X[b], P[b] = Xb[0], Pb[0]
            if want:
                if c > 0:
                    tr[:c, b] = tb[0]
                tr[c:, b] = X[b]
        trajs.append(tr)
    return X, P, trajs


def _filter_records(case, b, rows):
    rec = case["rec"]
    return synth.Records(rec.gyro[rows, b:b + 1], rec.acc[rows, b:b + 1], rec.mag[rows, b:b + 1],
                         rec.dtw[rows, b:b + 1], rec.acc0[b:b + 1], rec.mag0[b:b + 1],
                         None if rec.dtx is None else rec.dtx[rows, b:b + 1])


def expected_numpy(case, b):
    """expected() for filter b through the NumPy restatement: (X (4,), P (4,4), [traj (L,4) or None])."""
    X = np.array([1.0, 0.0, 0.0, 0.0]) if case["X0"] is None else case["X0"][b].copy()
    P = np.eye(4) if case["P0"] is None else case["P0"][b].copy()
    trajs = []
    for s, L, counts, want in case["launches"]:
        c = L if counts is None else min(int(counts[b]), L)
        tr = np.empty((L, 4)) if want else None
        if c > 0:
            sub = _filter_records(case, b, (s + np.arange(c)) % case["W"])
            g, dt, a, m = sub.filter(0)
            X, P, t = ekf_numpy.run_filter(g, dt, a, m, sub.acc0[0], sub.mag0[0], q=case["q"], r=case["r"], X0=X,
                                           P0=P, missing=sub.missing[:, 0], record=want)
            if want:
                tr[:c] = np.asarray(t).reshape(c, 4)
        if want:
            tr[c:] = X
        trajs.append(tr)
    return X, P, trajs


def within_spread(case, Xg, Pg, tg, Xe, Pe, te, scale):
    """True when every filter beyond TOL_F64 is within SPREAD x the C / NumPy oracles' disagreement."""
    bad = set(np.nonzero(np.abs(Xg - Xe).max(axis=1) >= TOL_F64)[0])
    bad |= set(np.nonzero(np.abs(Pg - Pe).max(axis=(1, 2)) / scale >= TOL_F64)[0])
    for g, e in zip(tg, te):
        if e is not None:
            bad |= set(np.nonzero(np.abs(g - e).max(axis=(0, 2)) >= TOL_F64)[0])
    for b in sorted(bad):
        Xn, Pn, tn = expected_numpy(case, b)
        # per quantity: the final X, the final P, each trajectory row (largest component of each)
        pairs = [(np.abs(Xg[b] - Xe[b]).max(), np.abs(Xn - Xe[b]).max()),
                 (np.abs(Pg[b] - Pe[b]).max() / scale, np.abs(Pn - Pe[b]).max() / scale)]
        pairs += [(np.abs(g[:, b] - e[:, b]).max(axis=1), np.abs(n - e[:, b]).max(axis=1))
                  for g, e, n in zip(tg, te, tn) if e is not None]
        for err, spread in pairs:
            if np.any(err >= np.maximum(TOL_F64, SPREAD * spread)):
                return False
    return True


def run_gpu(case):
    rec = case["rec"]
    win = engine.IMUWindow.from_records(rec)
    if case["handle"]:
        f = engine.FilterHandle(rec.acc0, rec.mag0, q=case["q"], r=case["r"], precision=case["precision"],
                                layout=case["layout"])
    else:
        f = engine.BatchedEKF(case["K"], q=case["q"], r=case["r"], precision=case["precision"],
                              layout=case["layout"])
    if case["X0"] is not None:
        f.set_state(case["X0"], case["P0"])
    trajs = []
    for s, L, counts, want in case["launches"]:
        trajs.append(f.run(win, n_steps=L, step0=s, want_traj=want, counts=counts))
    X, P = f.get_state()
    if case["handle"]:
        f.close()
    return X, P, trajs


def detail(case, tg, te):
    """Where the trajectories differ: launch, row, filter, that filter's count and the record's flags."""
    rec = case["rec"]
    for li, ((s, L, counts, want), g, e) in enumerate(zip(case["launches"], tg, te)):
        if e is None:
            continue
        d = np.abs(g - e).max(axis=2)
        for t, b in zip(*np.nonzero(d > TOL_F64)):
            row = (s + t) % case["W"]
            c = L if counts is None else min(int(counts[b]), L)
            tn = expected_numpy(case, b)[2][li]
            print("launch %d row t=%d (window row %d) filter %d: |d| %.3e (C / NumPy oracles %.3e)  count %d  "
                  "missing %s  dt %.6g  |x| gpu %.17g oracle %.17g"
                  % (li, t, row, b, d[t, b], np.abs(tn[t] - e[t, b]).max(), c, bool(rec.missing[row, b]),
                     rec.dt_ns[row, b], np.linalg.norm(g[t, b]), np.linalg.norm(e[t, b])))


def describe(case):
    shapes = ",".join("%d@%d%s%s" % (L, s, "c" if c is not None else "", "t" if w else "")
                      for s, L, c, w in case["launches"])
    return "K=%d W=%d launches=[%s] %s %s %s q=%g r=%g esc=%s X0=%s" % (
        case["K"], case["W"], shapes, case["layout"], case["precision"], "handle" if case["handle"] else "batched",
        case["q"], case["r"], case["rec"].dtx is not None, case["X0"] is not None)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--only", type=int, default=None, help="run only case N of the sweep, with per-row detail")
    a = ap.parse_args(argv)
    oracle_c.lib()
    rng = np.random.default_rng(a.seed)
    fails, skipped, spread_ok, worst, t0 = 0, 0, 0, 0.0, time.time()
    for i in range(a.cases):
        if i and i % 25 == 0:
            print("%d cases, %d mismatches, %d ill-conditioned, worst FP64 error %.3e, %.0f s"
                  % (i, fails, skipped, worst, time.time() - t0), flush=True)
        case = draw_case(rng)
        if a.only is not None and i != a.only:
            continue
        try:
            Xe, Pe, te = expected(case)
        except np.linalg.LinAlgError:
            skipped += 1
            continue
        pmax = float(np.abs(Pe).max())
        if not (pmax < P_WELL):
            skipped += 1
            continue
        Xg, Pg, tg = run_gpu(case)
        ex = float(np.abs(Xg - Xe).max())
        ep = float(np.abs(Pg - Pe).max()) / max(1.0, case["r"], pmax)
        et = max([float(np.abs(g - e).max()) for g, e in zip(tg, te) if e is not None] or [0.0])
        if case["precision"] == "f64":
            ok = ex < TOL_F64 and ep < TOL_F64 and et < TOL_F64
            if not ok and within_spread(case, Xg, Pg, tg, Xe, Pe, te, max(1.0, case["r"], pmax)):
                ok, spread_ok = True, spread_ok + 1
                print("case %d: |dX| %.3e |dP|/scale %.3e |dtraj| %.3e, within %g x the C / NumPy oracles' own "
                      "disagreement  %s" % (i, ex, ep, et, SPREAD, describe(case)), flush=True)
            else:
                worst = max(worst, ex, ep, et)
        else:
            ok = ex < TOL_MIXED_X and et < TOL_MIXED_X
        if not ok:
            fails += 1
            print("MISMATCH case %d: |dX| %.3e |dP|/scale %.3e |dtraj| %.3e max|P| %.2e  %s"
                  % (i, ex, ep, et, pmax, describe(case)), flush=True)
        if a.only is not None:
            detail(case, tg, te)
    print("done: %d cases (%d compared, %d ill-conditioned), %d mismatches, %d within the oracles' spread, "
          "worst FP64 error otherwise %.3e" % (a.cases, a.cases - skipped, skipped, fails, spread_ok, worst))
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
