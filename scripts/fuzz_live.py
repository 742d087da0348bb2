#!/usr/bin/env python3
"""Randomised sweep of the fused front-end + filter kernel (pekf_live_ext_dev) against the split
pipeline it replaces (pekf_frontend_ext_dev writing records, then pekf_run_ext_dev with counts), on
the GPU box.  The two must agree bit for bit (NaN where both are NaN): same records, same filter
arithmetic, applied in the same order (pekf_live.hip's header).  The split pipeline's records of four
filters per case are also checked against the front-end restatement (oracle/frontend_numpy.py): the
same count, gyro samples and dt exactly, acc / mag within 1 f32 ulp (the kernel's reciprocal / rsqrt).

Each case draws 1-700 filters and 1-400 events per filter with per-filter type mixes (balanced,
gyro-heavy, mag-starved, or strict gyro/acc/mag triples in random order), gaps of 0 ns (duplicate
timestamps: the interpolation divides 0 by 0 as the C++ server does), 1-4 ms, or now and then a pause
of 2^30 ns and more or a clock stepping back (time events, escaped record dts), filters that never got
ready (NaN phase-2 means) and a random initial state.

The default FP64-record form (pekf_live_ext_dev without PEKF_EV_F32_RECORDS: the low-pass acc / mag
reach the filter unrounded, as in the server) is run on every case too: its counts and reference pairs
must equal the f32 form's, and the four filters' final X must agree with the unrounded oracle chain
(the restatement's float64 records -> oracle/ekf_numpy.py, the reference's own arithmetic) within
F64_TOL; NaN where the chain's SVD raises (a NaN record: duplicate timestamps interpolate 0/0).
check_f64 says which filters the reference's own ill-conditioning exempts.

--ev64 (round 6) adds FP64 events (PEKF_EV_F64_EVENTS: the server's own stod values) on every case: the
fused kernel must equal the FP64 split pipeline (pekf_frontend_ext_dev writing FP64 records, then
pekf_run_rec64_dev with counts) bit for bit, its counts and reference pairs the f32 form's, and the
four filters' final X the oracle chain fed the server's values (wire.server_values) within F64_TOL,
with the same exemptions as check_f64.

usage: python3 scripts/fuzz_live.py [--cases N] [--seed S] [--ev64]   (exit status 1 on any difference)
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ekf_numpy, frontend_numpy  # noqa: E402  (the checkers)
from poseestimationkf_amd import engine, synth, wire  # noqa: E402

KINDS = np.array([synth.EV_ACC, synth.EV_GYRO, synth.EV_MAG], np.uint32)
F64_TOL = 1e-9   # FP64 records vs the unrounded chain (tests/test_live.py asserts 1e-12 on smooth streams)


def draw_case(rng):
    K = int(rng.integers(1, 701))
    E = int(rng.integers(1, 401))
    mix = str(rng.choice(["balanced", "gyro", "magless", "triples"]))
    if mix == "triples":
        perms = np.array([[0, 1, 2], [0, 2, 1], [1, 0, 2], [1, 2, 0], [2, 0, 1], [2, 1, 0]])
        G = (E + 2) // 3
        types = KINDS[perms[rng.integers(0, 6, size=(G, K))]].transpose(0, 2, 1).reshape(3 * G, K)[:E]
    else:
        p = {"balanced": [0.4, 0.4, 0.2], "gyro": [0.2, 0.7, 0.1], "magless": [0.5, 0.48, 0.02]}[mix]
        types = KINDS[rng.choice(3, size=(E, K), p=p)]
    gaps = rng.integers(1_000_000, 4_000_001, size=(E, K)).astype(np.int64)
    gaps = np.where(rng.random((E, K)) < 0.03, 0, gaps)
    if rng.random() < 0.4:  # pauses past the event word's 30-bit gap, and a clock stepping back
        odd = rng.random((E, K)) < 0.01
        gaps = np.where(odd, rng.choice([1 << 30, 3_000_000_000, -5_000_000, -2_500_000_000], size=(E, K)), gaps)
    times = synth.T_INIT_NS + np.cumsum(gaps, axis=0)
    vals = rng.standard_normal((E, K, 3)).astype(np.float32)
    vals[..., 2] += np.where(types == synth.EV_ACC, 9.8, 0.0).astype(np.float32)
    init_acc = rng.normal(size=(K, 3)) + [0.0, 0.0, 9.8]
    init_mag = rng.normal(size=(K, 3)) * 20.0
    init_acc[rng.random(K) < 0.05] = np.nan  # never got ready: no records, state left as it was
    ev = dict(types=types, values=vals, times=times, init_acc=init_acc, init_mag=init_mag,
              t_init=np.full(K, synth.T_INIT_NS, np.int64))
    X0 = P0 = None
    if rng.random() < 0.5:
        X0 = rng.normal(size=(K, 4))
        X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
        A = rng.normal(scale=0.3, size=(K, 4, 4))
        P0 = A @ A.transpose(0, 2, 1) + 0.05 * np.eye(4)
    return dict(ev=ev, K=K, E=E, mix=mix, X0=X0, P0=P0)


def _ulps(a, b):
    """f32 ulps between a and b; NaN only where both are NaN (else a large number)."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    if (na != nb).any():
        return 1 << 30
    ia = a[~na].view(np.int32).astype(np.int64)
    ib = b[~nb].view(np.int32).astype(np.int64)
    return int(np.abs(ia - ib).max(initial=0))


def check_records(case, win, counts, cols):
    """Problems (strings) of the records of filters cols against the front-end restatement."""
    ev, out = case["ev"], []
    rec = win.download_filters(cols)
    for j, k in enumerate(cols):
        if not np.isfinite(ev["init_acc"][k]).all():
            continue  # never ready: the kernels emit nothing, the restatement knows no phase 2
        g, dt, a, m = frontend_numpy.run_frontend(ev["types"][:, k], ev["values"][:, k].astype(np.float64),
                                                  ev["times"][:, k], ev["init_acc"][k], ev["init_mag"][k],
                                                  ev["t_init"][k])
        r = len(dt)
        if counts[k] != r:
            out.append("filter %d: %d records, restatement %d" % (k, counts[k], r))
            continue
        if not np.array_equal(rec.gyro[:r, j], g.astype(np.float32)):
            out.append("filter %d: gyro" % k)
        if not np.array_equal(rec.dt_ns[:r, j], dt.astype(np.float64)):
            out.append("filter %d: dt" % k)
        u = max(_ulps(rec.acc[:r, j], a), _ulps(rec.mag[:r, j], m))
        if u > 1:
            out.append("filter %d: acc / mag %d ulps" % (k, u))
    return out


def split(case, cols=None):
    win, counts = engine.run_frontend(case["ev"])
    if cols is not None:
        case["record_problems"] = check_records(case, win, counts, cols)
    f = engine.BatchedEKF(case["K"])
    if case["X0"] is not None:
        f.set_state(case["X0"], case["P0"])
    if counts.max(initial=0) > 0:
        # at least two steps, so that the launch is the multi-record kernel k_live shares its arithmetic
        # with (a launch of one record takes the online kernel, which runs the step in the world basis
        # and agrees with it to rounding only); the counts keep every filter to its own records
        f.run(win, n_steps=max(2, int(counts.max())))
    X, P = f.get_state()
    return X, P, counts, win.refs.download((case["K"], 6), np.float64)


def fused(case, records="f32", events="f32"):
    f = engine.BatchedEKF(case["K"])
    if case["X0"] is not None:
        f.set_state(case["X0"], case["P0"])
    counts, refs = f.run_events(case["ev"], records=records, events=events)   # f32: the split pipeline's records
    X, P = f.get_state()
    return X, P, counts, refs


def split64(case):
    """The FP64-event split pipeline: FP64 records (a RecordWindow64), then pekf_run_rec64_dev with counts."""
    win, counts = engine.run_frontend(case["ev"], events="f64")
    f = engine.BatchedEKF(case["K"])
    if case["X0"] is not None:
        f.set_state(case["X0"], case["P0"])
    if counts.max(initial=0) > 0:
        f.run(win, n_steps=max(2, int(counts.max())))
    X, P = f.get_state()
    return X, P, counts, win.refs.download((case["K"], 6), np.float64)


def _chain(g, dt, a, m, refs_k, X0, P0):
    """The unrounded oracle chain's final X: NaN-filled if its SVD raises on a NaN record."""
    try:
        with np.errstate(all="ignore"):
            X, _, _ = ekf_numpy.run_filter(g, dt, a, m, refs_k[:3], refs_k[3:], X0=X0, P0=P0, record=False)
        return X, False
    except np.linalg.LinAlgError:
        return np.full(4, np.nan), True


def check_f64(case, got, cols, tally, server=False):
    """(problems, worst |dq|) of the FP64-record run's filters cols against the unrounded oracle chain.

    Two kinds of filter are not held to F64_TOL, each counted in `tally`: where the reference itself
    returns NaN from finite records (its RotationMatrix2Quart at an exactly-identity rotation takes a
    square root of -2e-16 -- the first record after duplicate timestamps interpolates to the phase-2
    means exactly; the kernel returns the well-conditioned value), and where the chain
    is ill-conditioned: rounding its records to f32 moves its answer by more than 1e-6 (a Comparator
    sign at q.z ~ 0, ExtendedKalmanFilter.py:73-75: either sign is the reference's answer).  A filter
    off by more than F64_TOL is held to 4x the spread of the reference's own answer under 1-ulp
    input noise instead (near-identity rotations) and counted as ulp-sensitive -- or counted as
    ill-conditioned when the reference's R->q broke down on one of its records (a non-unit quaternion:
    the branch formula at an all-but-identity rotation) or its answer turns NaN under that noise."""
    ev, out, worst = case["ev"], [], 0.0
    X, _, counts, refs = got
    for k in cols:
        if not np.isfinite(ev["init_acc"][k]).all():
            continue
        vals = wire.server_values(ev["values"][:, k]) if server else ev["values"][:, k].astype(np.float64)
        g, dt, a, m = frontend_numpy.run_frontend(ev["types"][:, k], vals,
                                                  ev["times"][:, k], ev["init_acc"][k], ev["init_mag"][k],
                                                  ev["t_init"][k])
        if len(dt) == 0:
            continue
        X0 = None if case["X0"] is None else case["X0"][k]
        P0 = None if case["P0"] is None else case["P0"][k]
        dt = dt.astype(np.float64)
        Xo, raised = _chain(g, dt, a, m, refs[k], X0, P0)

        def ulp_spread():
            # the reference's own answer under 1-ulp input noise (16 samples): near an identity Wahba
            # rotation its R->q divides rounding noise by the angle; NaN if any sample is
            pr = np.random.default_rng(k)
            sp = 0.0
            for _ in range(16):
                u = lambda v: v * (1 + 2.2e-16 * pr.standard_normal(np.shape(v)))  # noqa: E731
                Xn, _ = _chain(u(g), dt, u(a), u(m), u(refs[k]), X0, P0)
                sp = max(sp, float(np.abs(Xn - Xo).max())) if np.isfinite(Xn).all() else np.nan
            return sp
        if raised or np.isnan(X[k]).any():
            if raised and np.isnan(X[k]).all():
                continue                                  # both NaN: a NaN record (0 / 0 interpolation)
            if not raised and np.isnan(Xo).all() and np.isnan(X[k]).all():
                tally["reference_nan"] += 1               # both NaN from finite records: the reference's R->q
                continue                                  # at an exactly-identity rotation, taken by both
            if not raised and not np.isnan(Xo).any() and not ulp_spread() < 1e-6:
                tally["ill_conditioned"] += 1             # the kernel NaN where the reference's own answer
                continue                                  # is noise-driven (NaN or moved under 1-ulp noise)
            out.append("filter %d: NaN in one of kernel / chain (chain raised: %s)" % (k, raised))
            continue
        if np.isnan(Xo).any():
            tally["reference_nan"] += 1
            continue
        r32 = lambda v: v.astype(np.float32).astype(np.float64)  # noqa: E731
        X32, _ = _chain(r32(g), dt, r32(a), r32(m), refs[k], X0, P0)
        if not float(np.abs(X32 - Xo).max()) < 1e-6:
            tally["ill_conditioned"] += 1
            continue
        d = float(np.abs(X[k] - Xo).max())
        if d > F64_TOL:
            # the reference's RotationMatrix2Quart broke down on some record (Wahba.py:19-47 at an all-but-
            # identity rotation: its branch formula divides rounding noise by sqrt(noise) and returns a
            # non-unit "quaternion", |q| ~ 1e-8) -- the kernel returns the unit quaternion there (DESIGN.md
            # §4.1), and the trajectories meet again only as the filter forgets: exempt, counted
            qn = [np.linalg.norm(ekf_numpy.wahba_quat(refs[k][:3], refs[k][3:], a[i], m[i], abs(a[i][2]),
                                                      1 - abs(a[i][2]))) for i in range(len(dt))]
            if np.nanmax(np.abs(np.asarray(qn) - 1.0)) > 1e-6:
                tally["ill_conditioned"] += 1
                continue
            # such a filter is held to four times the reference's own 1-ulp spread, and counted; one whose
            # answer turns NaN under 1-ulp noise (an exactly-identity rotation one ulp away) is ill-conditioned
            sp = ulp_spread()
            if np.isnan(sp):
                tally["ill_conditioned"] += 1
                continue
            if d <= 4 * sp:
                tally["ulp_sensitive"] += 1
                continue
        worst = max(worst, d)
        tally["checked"] += 1
        if d > F64_TOL:
            out.append("filter %d: FP64 records vs the unrounded chain %.3e" % (k, d))
    return out, worst


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=100)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--ev64", action="store_true")
    a = ap.parse_args(argv)
    rng = np.random.default_rng(a.seed)
    fails, records, t0, worst64, worst_ev64 = 0, 0, time.time(), 0.0, 0.0
    tally = dict(checked=0, reference_nan=0, ill_conditioned=0, ulp_sensitive=0)
    tally64 = dict(checked=0, reference_nan=0, ill_conditioned=0, ulp_sensitive=0)
    for i in range(a.cases):
        if i and i % 25 == 0:
            print("%d cases, %d differ, %d records applied, FP64 records vs the unrounded chain <= %.3e, %.0f s"
                  % (i, fails, records, worst64, time.time() - t0), flush=True)
        case = draw_case(rng)
        cols = rng.choice(case["K"], size=min(4, case["K"]), replace=False)
        u, v = fused(case), split(case, cols)
        if case["record_problems"]:
            fails += 1
            print("RECORDS case %d: %s  K=%d E=%d mix=%s" % (i, "; ".join(case["record_problems"][:4]), case["K"],
                                                            case["E"], case["mix"]), flush=True)
        records += int(u[2].sum())
        w = fused(case, "f64")
        probs, d64 = check_f64(case, w, cols, tally)
        worst64 = max(worst64, d64)
        if not (np.array_equal(w[2], u[2]) and np.array_equal(w[3], u[3], equal_nan=True)):
            probs.append("counts / refs differ from the f32 form")
        if probs:
            fails += 1
            print("F64 case %d: %s  K=%d E=%d mix=%s" % (i, "; ".join(probs[:4]), case["K"], case["E"], case["mix"]),
                  flush=True)
        if a.ev64:
            x64, s64 = fused(case, "f64", "f64"), split64(case)
            probs, d = check_f64(case, x64, cols, tally64, server=True)
            worst_ev64 = max(worst_ev64, d)
            if not (np.array_equal(x64[2], u[2]) and np.array_equal(x64[3], u[3], equal_nan=True)):
                probs.append("FP64 events: counts / refs differ from the f32 form")
            if not all(np.array_equal(x, y, equal_nan=True) for x, y in zip(x64, s64)):
                probs.append("FP64 events: fused != FP64 split pipeline")
            if probs:
                fails += 1
                print("EV64 case %d: %s  K=%d E=%d mix=%s" % (i, "; ".join(probs[:4]), case["K"], case["E"],
                                                             case["mix"]), flush=True)
        same = all(np.array_equal(x, y, equal_nan=True) for x, y in zip(u, v))
        if not same:
            fails += 1
            names = ["%s (max |d| %.3e)" % (n, float(np.nanmax(np.abs(np.asarray(x, float) - np.asarray(y, float)))))
                     for n, x, y in zip(("X", "P", "counts", "refs"), u, v) if not np.array_equal(x, y, equal_nan=True)]
            print("DIFFERENT case %d: %s  K=%d E=%d mix=%s X0=%s" % (i, ", ".join(names), case["K"], case["E"],
                                                                     case["mix"], case["X0"] is not None), flush=True)
    print("done: %d cases, %d differ, %d records applied; FP64 records vs the unrounded chain <= %.3e over %d "
          "filters (%d where the reference returns NaN from finite records, %d ill-conditioned: not held to it; "
          "%d within 4x the reference's own spread under 1-ulp input noise)"
          % (a.cases, fails, records, worst64, tally["checked"], tally["reference_nan"], tally["ill_conditioned"],
             tally["ulp_sensitive"]))
    if a.ev64:
        print("FP64 events: fused = FP64 split pipeline bit for bit on every case; vs the oracle chain fed the "
              "server's values <= %.3e over %d filters (%d reference NaN, %d ill-conditioned, %d ulp-sensitive)"
              % (worst_ev64, tally64["checked"], tally64["reference_nan"], tally64["ill_conditioned"],
                 tally64["ulp_sensitive"]))
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
