"""Golden vectors for time differences that do not fit the 31-bit record word, made by importing the
REFERENCE itself (run in the survey container only; /root/reference does not exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_gaps_golden.py

The reference's Prediction takes any float64 T - previousT (ExtendedKalmanFilter.py:32,62): pauses of
seconds, a clock that steps back, a fractional difference of float64 timestamps.  This runs
main_file.py's loop (its classes, unchanged: KalmanFilter(T0, ...), setQ(1), setR(0.1), Prediction +
Correction per record, ExtendedKalmanFilter.py:6-80, main_file.py:19-47) over synthetic streams whose
absolute timestamps carry such differences, and stores inputs and X trajectories only.

Output: tests/golden/gaps.npz
  gyro/acc/mag (W,K,3) f32, dt (W,K) float64 (= T[i] - T[i-1] as the reference forms it),
  acc0/mag0 (K,3), t0 (K,) float64, traj (W,K,4) the reference's X after every record.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# where the fixtures are written (tests/test_golden_regen.py regenerates them into a scratch directory)
OUT = os.environ.get("PEKF_GOLDEN_OUT") or HERE
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_DIR = "/root/reference/Python Kalman Filter"
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

from poseestimationkf_amd import synth  # noqa: E402

ODD = [5e9, -2e7, 1e7 + 0.5, float(0x7FFFFFFF), 3.3e10, 0.0, 2147483648.0, -1.5]


def main():
    sys.path.insert(0, REF_DIR)
    import ExtendedKalmanFilter as ekf  # noqa: E402  (the reference module)

    K, W = 6, 300
    rec = synth.generate(np.arange(200, 200 + K), W, seed=77)
    dt = rec.dt_ns.copy()
    rng = np.random.default_rng(77)
    for k in range(K):
        rows = rng.choice(W, size=12, replace=False)
        for j, r in enumerate(rows):
            dt[r, k] = ODD[(j + k) % len(ODD)]
    dt[:, 3] = 5e9                      # one filter that pauses before every record
    t0 = 1.0e12 + 1e6 * np.arange(K)
    traj = np.empty((W, K, 4))
    for k in range(K):
        kf = ekf.KalmanFilter(t0[k], rec.mag0[k], rec.acc0[k], 0.5)
        kf.setQ(1)
        kf.setR(0.1)
        X, P = np.asarray([1., 0., 0., 0.]), np.identity(4)
        T = t0[k]
        for i in range(W):
            Tn = T + dt[i, k]
            assert Tn - T == dt[i, k]   # the reference's T - previousT is exactly the stored dt
            T = Tn
            g, a, m = (v[i, k].astype(np.float64) for v in (rec.gyro, rec.acc, rec.mag))
            z, P, Kk = kf.Prediction(g, T, X, P)
            X, P = kf.Correction(m, a, z, P, Kk)
            traj[i, k] = X
    np.savez_compressed(os.path.join(OUT, "gaps.npz"), gyro=rec.gyro, acc=rec.acc, mag=rec.mag, dt=dt,
                        acc0=rec.acc0, mag0=rec.mag0, t0=t0, traj=traj)
    print("gaps.npz", os.path.getsize(os.path.join(OUT, "gaps.npz")))


if __name__ == "__main__":
    main()
