#!/usr/bin/env python3
"""Randomised sweep of the FP64-record launch (pekf_run_rec64_dev, engine.RecordWindow64) on the GPU box.

Cases are scripts/fuzz_gpu.py's (1-300 filters, 1-48-row windows, 1-3 windows' worth of records cut
into launches at a random start row, per-launch counts, trajectories, escaped time differences, a
random initial state, q and r), restricted to what FP64 records carry: every record has its
magnetometer sample (the missing flag is cleared), FP64 AoS state.  Each case is checked three ways:

* the same f32-representable values in a RecordWindow64: against the C oracle over exactly the
  records each filter applied (fuzz_gpu.expected, TOL_F64, the C / NumPy-spread rule), and bit for bit
  against the 40 B-record launch (pekf_run_dev) when every launch is of >= 2 records (the one-record
  launch of pekf_run_dev is the world-basis online kernel, which agrees to rounding only);
* float64 values (the f32 values moved off the f32 grid by a relative 1e-9): one launch over the whole
  run, four sampled filters against the NumPy restatement (ekf_numpy.run_filter on the float64 rows),
  held to TOL_F64 unless the reference itself is ill-conditioned there (rounding the records to f32
  moves its answer by more than 1e-6), which is counted.

usage: python3 scripts/fuzz_rec64.py [--cases N] [--seed S]   (exit status 1 on any mismatch)
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import fuzz_gpu as fg  # noqa: E402  (its cases and its oracle runs)
from oracle import ekf_numpy  # noqa: E402  (the checker)
from poseestimationkf_amd import engine, synth  # noqa: E402


def rec64_case(rng):
    case = fg.draw_case(rng)
    rec = case["rec"]
    rec.dtw &= np.uint32(synth.DT_MASK)          # FP64 records carry every magnetometer sample
    case.update(precision="f64", layout="aos", handle=False)
    return case


def dt_f64(rec):
    """The float64 dt of every row (the escaped ones from the side plane)."""
    dt = rec.dt_ns.astype(np.float64)
    return dt


def window64(rec, g=None, a=None, m=None):
    g = rec.gyro.astype(np.float64) if g is None else g
    a = rec.acc.astype(np.float64) if a is None else a
    m = rec.mag.astype(np.float64) if m is None else m
    return engine.RecordWindow64.from_arrays(g, dt_f64(rec), a, m, rec.acc0, rec.mag0)


def run(case, win):
    f = engine.BatchedEKF(case["K"], q=case["q"], r=case["r"])
    if case["X0"] is not None:
        f.set_state(case["X0"], case["P0"])
    trajs = [f.run(win, n_steps=L, step0=s, want_traj=want, counts=counts)
             for s, L, counts, want in case["launches"]]
    X, P = f.get_state()
    return X, P, trajs


def check_f64_values(case, rng, tally):
    """Float64 values off the f32 grid, one launch over the whole run: (problems, worst |dq|)."""
    rec, K, W = case["rec"], case["K"], case["W"]
    bump = lambda v: v.astype(np.float64) * (1.0 + 1e-9 * rng.standard_normal(v.shape))  # noqa: E731
    g, a, m = bump(rec.gyro), bump(rec.acc), bump(rec.mag)
    s0 = case["launches"][0][0]
    n = sum(L for _, L, _, _ in case["launches"])
    f = engine.BatchedEKF(K, q=case["q"], r=case["r"])
    if case["X0"] is not None:
        f.set_state(case["X0"], case["P0"])
    f.run(window64(rec, g, a, m), n_steps=n, step0=s0)
    X, _ = f.get_state()
    dt = dt_f64(rec)
    rows = (s0 + np.arange(n)) % W
    out, worst = [], 0.0
    for b in rng.choice(K, size=min(4, K), replace=False):
        X0 = None if case["X0"] is None else case["X0"][b]
        P0 = None if case["P0"] is None else case["P0"][b]
        chain = lambda gg, aa, mm: ekf_numpy.run_filter(gg[rows, b], dt[rows, b], aa[rows, b], mm[rows, b],  # noqa: E731
                                                        rec.acc0[b], rec.mag0[b], q=case["q"], r=case["r"], X0=X0,
                                                        P0=P0, record=False)[0]
        try:
            with np.errstate(all="ignore"):
                Xo = chain(g, a, m)
                r32 = lambda v: v.astype(np.float32).astype(np.float64)  # noqa: E731
                X32 = chain(r32(g), r32(a), r32(m))
        except np.linalg.LinAlgError:
            tally["singular"] += 1
            continue
        if not (np.isfinite(Xo).all() and np.isfinite(X32).all()) or not float(np.abs(X32 - Xo).max()) < 1e-6:
            tally["ill_conditioned"] += 1
            continue
        d = float(np.abs(X[b] - Xo).max())
        worst = max(worst, d)
        tally["checked"] += 1
        if not d < fg.TOL_F64:
            out.append("filter %d: FP64 values vs the NumPy restatement %.3e" % (b, d))
    return out, worst


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=100)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args(argv)
    rng = np.random.default_rng(a.seed)
    fails = bitwise = skipped = 0
    worst = worst64 = 0.0
    tally = dict(checked=0, ill_conditioned=0, singular=0)
    t0 = time.time()
    for i in range(a.cases):
        if i and i % 100 == 0:
            print("%d cases, %d mismatches, %d bit-identical to the 40 B launch, worst %.3e / %.3e (f32 / f64 "
                  "values), %.0f s" % (i, fails, bitwise, worst, worst64, time.time() - t0), flush=True)
        case = rec64_case(rng)
        try:
            Xe, Pe, te = fg.expected(case)
        except np.linalg.LinAlgError:
            skipped += 1
            continue
        Xg, Pg, tg = run(case, window64(case["rec"]))
        scale = max(1.0, case["r"], float(np.abs(Pe).max()))
        if not np.abs(Pe).max() < fg.P_WELL:
            skipped += 1
        else:
            err = max([float(np.abs(Xg - Xe).max()), float(np.abs(Pg - Pe).max()) / scale] +
                      [float(np.abs(g - e).max()) for g, e in zip(tg, te) if e is not None])
            if err >= fg.TOL_F64 and not fg.within_spread(case, Xg, Pg, tg, Xe, Pe, te, scale):
                fails += 1
                print("MISMATCH case %d vs the C oracle: %.3e  K=%d W=%d launches=%s" % (
                    i, err, case["K"], case["W"], [(s, L) for s, L, _, _ in case["launches"]]), flush=True)
            elif err < fg.TOL_F64:
                worst = max(worst, err)
        if all(L >= 2 for _, L, _, _ in case["launches"]):
            Xf, Pf, tf = run(case, engine.IMUWindow.from_records(case["rec"]))
            same = np.array_equal(Xf, Xg, equal_nan=True) and np.array_equal(Pf, Pg, equal_nan=True) and all(
                (x is None and y is None) or np.array_equal(x, y, equal_nan=True) for x, y in zip(tf, tg))
            if same:
                bitwise += 1
            else:
                fails += 1
                print("NOT BIT-IDENTICAL case %d to the 40 B-record launch  K=%d W=%d" % (i, case["K"], case["W"]),
                      flush=True)
        probs, w64 = check_f64_values(case, rng, tally)
        worst64 = max(worst64, w64)
        if probs:
            fails += 1
            print("F64 case %d: %s" % (i, "; ".join(probs)), flush=True)
    print("done: %d cases (%d not compared: singular or ill-conditioned covariance), %d mismatches, %d bit-identical "
          "to the 40 B launch; worst vs the C oracle %.3e; float64 values vs NumPy %.3e over %d filters (%d "
          "ill-conditioned, %d singular: not held to it)"
          % (a.cases, skipped, fails, bitwise, worst, worst64, tally["checked"], tally["ill_conditioned"],
             tally["singular"]))
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
