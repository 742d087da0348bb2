"""Filter handle (pekf_filter_*): B KalmanFilter objects with device-resident state.

update() is main_file.py:42-45 per filter from FP64 host arrays; it shares ekf_record_step with
the stream kernel (the stream kernel in the reference frame's basis, update() in the world basis),
so on f32-representable records it agrees with pekf_run_dev to rounding, and on general FP64
records it is checked against the NumPy restatement of the reference.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ekf_numpy as npo
from poseestimationkf_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


ROUNDING = 1e-13  # per-record (world basis) vs multi-record (reference-frame basis) launches


def _close(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max()) < ROUNDING


@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_update_loop_matches_stream_run(eng, layout):
    K, N = 300, 40
    rec = synth.generate(np.arange(K), N, seed=31, missing=True)
    ref = eng.BatchedEKF(K)
    tr = ref.run(eng.IMUWindow.from_records(rec), want_traj=True)
    t0 = np.arange(K, dtype=np.int64) * 1000 + 5_000_000_000
    h = eng.FilterHandle(rec.acc0, rec.mag0, q=1.0, r=0.1, t0_ns=t0, layout=layout)
    t = t0.copy()
    for i in range(N):
        t += (rec.dtw[i] & 0x7FFFFFFF).astype(np.int64)
        X = h.update(rec.gyro[i].astype(np.float64), t, rec.acc[i].astype(np.float64), rec.mag[i].astype(np.float64),
                     missing=(rec.dtw[i] >> 31).astype(np.uint8))
        assert _close(X, tr[i]), i
    Xr, Pr = ref.get_state()
    Xh, Ph = h.get_state()
    assert _close(Xh, Xr) and _close(Ph, Pr)


def test_update_fp64_records_against_numpy_restatement(eng):
    """Inputs that are not f32-representable (the reference's FP64 path) vs oracle/ekf_numpy.py."""
    K, N = 12, 60
    rng = np.random.default_rng(5)
    rec = synth.generate(np.arange(K), N, seed=2)
    gyro = rec.gyro.astype(np.float64) + rng.normal(scale=1e-9, size=rec.gyro.shape)
    acc = rec.acc.astype(np.float64) + rng.normal(scale=1e-9, size=rec.acc.shape)
    mag = rec.mag.astype(np.float64) + rng.normal(scale=1e-9, size=rec.mag.shape)
    dt = (rec.dtw & 0x7FFFFFFF).astype(np.int64)
    h = eng.FilterHandle(rec.acc0, rec.mag0)
    t = np.zeros(K, np.int64)
    for i in range(N):
        t += dt[i]
        X = h.update(gyro[i], t, acc[i], mag[i])
    assert np.array_equal(h.get_time(), t)  # previousT advanced to each filter's last T (:67)
    h.set_time(t - 5)
    assert np.array_equal(h.get_time(), t - 5)
    h.set_time(t)
    for k in range(K):
        Xo, Po, _ = npo.run_filter(gyro[:, k], dt[:, k].astype(np.float64), acc[:, k], mag[:, k], rec.acc0[k],
                                   rec.mag0[k], record=False)
        assert np.abs(X[k] - Xo).max() < 1e-9
        assert np.abs(h.get_state()[1][k] - Po).max() < 1e-9


def test_handle_run_and_state_roundtrip(eng):
    K, W = 130, 24
    rec = synth.generate(np.arange(K), W, seed=6)
    win = eng.IMUWindow.from_records(rec)
    a = eng.BatchedEKF(K)
    a.run(win, n_steps=W)
    h = eng.FilterHandle(rec.acc0, rec.mag0, layout="soa")
    h.run(win, n_steps=W)
    (Xa, Pa), (Xh, Ph) = a.get_state(), h.get_state()
    assert _same(Xa, Xh) and _same(Pa, Ph)
    h.set_state(X=np.tile([1.0, 0, 0, 0], (K, 1)))       # X only: P is kept
    X2, P2 = h.get_state()
    assert _same(P2, Ph) and np.all(X2[:, 0] == 1.0)
    h.set_state(P=np.tile(np.eye(4), (K, 1, 1)))
    assert _same(h.get_state()[1], np.tile(np.eye(4), (K, 1, 1)))
    h.close()
