#!/usr/bin/env python3
"""Randomised sweep of the batched per-call operators (pekf_predict / pekf_correct /
pekf_wahba_quaternion: the drop-ins' Prediction, Correction and getQuarternion) against the NumPy
restatement of the reference (oracle/ekf_numpy.py, bit-identical to ExtendedKalmanFilter.py /
Wahba.py), item by item, on the GPU box.

Each case draws 1-3,000 items with random gyro rates, dts of 0-2 s (fractional ns too), quaternions
of norm 0.5-2, covariances that are SPD or general (non-symmetric, as the reference accepts any
4x4), Q and R scalar or full SPD, raw-magnitude or unit acc / mag samples and reference pairs, and
Wahba weights of either sign.  An item passes within 1e-12 x max(1, |value|), or, where the item is
ill-conditioned in the reference's own arithmetic, within 10 x the disagreement between the two
restatements of the reference (the C oracle and the NumPy one differ only in rounding); a Wahba
quaternion also within 100 ulps of B's largest singular value over s2 + s3 (the SVD's own bound).

usage: python3 scripts/fuzz_percall.py [--cases N] [--seed S]   (exit status 1 on any mismatch)
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
from poseestimationkf_amd import engine  # noqa: E402

TOL = 1e-12
SPREAD = 10.0


def _unit(rng, shape):
    v = rng.normal(size=shape)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _spd(rng, n, k, scalar_p):
    A = rng.normal(scale=0.5, size=(n, k, k))
    M = A @ A.transpose(0, 2, 1) + 0.05 * np.eye(k)
    s = rng.uniform(0.01, 3.0, size=(n, 1, 1)) * np.eye(k)
    return np.where((rng.random(n) < scalar_p)[:, None, None], s, M)


def draw_case(rng):
    n = int(rng.integers(1, 3001))
    gyro = rng.normal(scale=float(rng.choice([0.1, 1.0, 3.0])), size=(n, 3))
    dt = rng.uniform(0, float(rng.choice([2e7, 2e9])), size=n)
    dt = np.where(rng.random(n) < 0.5, np.floor(dt), dt)
    X = _unit(rng, (n, 4)) * rng.uniform(0.5, 2.0, size=(n, 1))
    P = _spd(rng, n, 4, 0.0)
    P = np.where((rng.random(n) < 0.3)[:, None, None], P + rng.normal(scale=0.1, size=(n, 4, 4)), P)
    Q, R = _spd(rng, n, 3, 0.5), _spd(rng, n, 4, 0.5)
    raw = rng.random() < 0.5
    sa, sm = (9.8, 45.0) if raw else (1.0, 1.0)
    acc = (_unit(rng, (n, 3)) + rng.normal(scale=0.05, size=(n, 3))) * sa
    mag = (_unit(rng, (n, 3)) + rng.normal(scale=0.05, size=(n, 3))) * sm
    acc0, mag0 = _unit(rng, (n, 3)) * sa, _unit(rng, (n, 3)) * sm
    ka = rng.uniform(-1.0, 2.0, size=n)
    return dict(n=n, gyro=gyro, dt=dt, X=X, P=P, Q=Q, R=R, acc=acc, mag=mag, acc0=acc0, mag0=mag0, ka=ka, km=1.0 - ka,
                raw=raw)


def _ok(err, ref, spread):
    scale = np.maximum(1.0, np.abs(ref))
    return bool(np.all(err <= np.maximum(TOL * scale, SPREAD * spread)))


def check(c):
    """Problems (strings) of one case."""
    out = []
    z, Pm, K = engine.predict(c["gyro"], c["dt"], c["X"], c["P"], c["Q"], c["R"])
    Xc, Pc = engine.correct(c["mag"], c["acc"], z, Pm, K, c["acc0"], c["mag0"])
    qw = engine.wahba_quaternion(c["acc0"], c["mag0"], c["acc"], c["mag"], c["ka"], c["km"])
    for i in range(c["n"]):
        zn, Pn, Kn = ekf_numpy.predict(c["gyro"][i], c["dt"][i], c["X"][i], c["P"][i], c["Q"][i], c["R"][i])
        Xn, Pcn = ekf_numpy.correct(c["mag"][i], c["acc"][i], z[i], Pm[i], K[i], c["acc0"][i], c["mag0"][i])
        qn = ekf_numpy.wahba_quat(c["acc0"][i], c["mag0"][i], c["acc"][i], c["mag"][i], c["ka"][i], c["km"][i])
        for name, g, e in (("z", z[i], zn), ("P-", Pm[i], Pn), ("K", K[i], Kn), ("X", Xc[i], Xn), ("P", Pc[i], Pcn),
                           ("q_wahba", qw[i], qn)):
            err = np.abs(g - e)
            if np.all(err <= TOL * np.maximum(1.0, np.abs(e))):
                continue
            # the C restatement on the same inputs: how far the reference's own rounding moves this item
            if name in ("z", "P-", "K"):
                zc, Pcc, Kc = oracle_c.predict(c["gyro"][i], c["dt"][i], c["X"][i], c["P"][i], c["Q"][i], c["R"][i])
                alt = {"z": zc, "P-": Pcc, "K": Kc}[name]
            elif name in ("X", "P"):
                Xo, Po = oracle_c.correct(c["mag"][i], c["acc"][i], z[i], Pm[i], K[i], c["acc0"][i], c["mag0"][i])
                alt = {"X": Xo, "P": Po}[name]
            else:
                alt = oracle_c.wahba_quat(c["acc0"][i], c["mag0"][i], c["acc"][i], c["mag"][i], c["ka"][i], c["km"][i])
            spread = np.abs(alt - e)
            if name == "q_wahba":
                # the rotation of an SVD moves by ~ |dB| / (s2 + s3) for a perturbation dB of B
                # (LAPACK's error bound for the singular subspaces); the kernel's closed-form 3x3 SVD
                # and the reference's gesdd round differently, so allow that bound at a few ulps of B
                B = (c["ka"][i] * np.outer(c["acc0"][i], c["acc"][i]) + c["km"][i] * np.outer(c["mag0"][i], c["mag"][i]))
                sv = np.linalg.svd(B, compute_uv=False)
                spread = np.maximum(spread, 10 * np.finfo(float).eps * sv[0] / max(sv[1] + sv[2], 1e-300))
            if not _ok(err, e, spread):
                out.append("item %d %s: |d| %.3e (C / NumPy %.3e)" % (i, name, err.max(), np.abs(alt - e).max()))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args(argv)
    oracle_c.lib()
    rng = np.random.default_rng(a.seed)
    fails, items, t0 = 0, 0, time.time()
    for i in range(a.cases):
        c = draw_case(rng)
        items += c["n"]
        problems = check(c)
        if problems:
            fails += 1
            print("MISMATCH case %d (n=%d raw=%s): %s" % (i, c["n"], c["raw"], "; ".join(problems[:4])), flush=True)
        print("%d cases, %d items, %d mismatching cases, %.0f s" % (i + 1, items, fails, time.time() - t0), flush=True)
    print("done: %d cases, %d items, %d mismatching cases" % (a.cases, items, fails))
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
