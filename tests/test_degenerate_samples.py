"""Samples that leave Wahba's B rank-deficient: a zero accelerometer or magnetometer sample, or the two
exactly parallel (Wahba.py:8-17, B = |acc_z| acc0 acc^T + (1 - |acc_z|) mag0 mag^T = w v^T).

The reference stays finite there: np.linalg.svd returns some rotation taking v/|v| to w/|w|, chosen by
the rounding noise of B's zero singular values, so no other evaluation reproduces that particular one
(the C oracle's Jacobi SVD picks another: CPU test below).  What is defined is the optimum itself,
tr(R^T B) = |w||v|, and every rotation attaining it is a correct answer.  The build takes the shortest
arc (pekf_math.hpp: wahba_current_rank1 / wahba_rank1_rotation).  Both samples zero (B = 0) gives NaN,
as the reference does (its SVD returns the identity, and RotationMatrix2Quart divides 0 by 0 there).

GPU: the per-call Wahba operators and the pure-Wahba side output attain the reference's optimum (a pair
parallel to within 1e-12 counts as rank 1 there).  The fused kernels (multi-record, one-record, handle,
the fused front-end + filter) detect a zero sample for free -- it makes their Wahba chain NaN, and the
rare fallback branch, taken for NaN too, solves the rank-1 problem from the record re-read from memory
-- and stay finite through such records.  An exactly parallel pair is not caught there (its Gram-Schmidt
remainder is rounding noise, not zero), so that record's measurement is an arbitrary finite attitude,
as arbitrary as the reference's noise-chosen one.  Either way the trajectories equal the reference
before the first such record and are back on it within 1e-9 thirty records after (the Kalman gain
forgets a measurement geometrically: ~4x per record here).  Before this handling a zero sample turned
a fused filter's state into NaN for the rest of its stream."""
import numpy as np
import pytest

from oracle import ekf_numpy
from poseestimationkf_amd import synth

ACC0, MAG0 = np.array([0.0, 0.1, 0.99]), np.array([0.5, 0.0, -0.86])


def _ref_rotation(acc0, mag0, acc, mag, ka, km):
    B = ka * np.outer(acc0, acc) + km * np.outer(mag0, mag)            # Wahba.py:11-13
    u, s, vh = np.linalg.svd(B)
    return u @ np.diag([1, 1, np.linalg.det(u) * np.linalg.det(vh)]) @ vh, B


def _quat_rotm(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


CASES = {   # (acc, mag) of the current sample, (acc0, mag0) of the reference pair
    "zero acc": ([0.0, 0.0, 0.0], [0.45, 0.05, -0.88], ACC0, MAG0),
    "zero mag": ([0.02, 0.1, 0.98], [0.0, 0.0, 0.0], ACC0, MAG0),
    "acc parallel to mag": ([0.1, -0.2, 0.95], [0.2, -0.4, 1.9], ACC0, MAG0),
    "reference pair parallel": ([0.02, 0.1, 0.98], [0.45, 0.05, -0.88], ACC0, 2.0 * ACC0),
}


def _degenerate_stream(K=8, W=120, seed=9):
    rec = synth.generate(np.arange(K), W, seed=seed)
    marks = {}
    rec.acc[20, 0] = 0.0                          # zero acc
    rec.mag[35, 1] = 0.0                          # zero mag
    rec.mag[50, 2] = 2.0 * rec.acc[50, 2]         # mag exactly parallel to acc
    rec.acc[15, 3] = 0.0                          # two degenerate records in one filter
    rec.mag[60, 3] = 0.0
    rec.acc[70, 4] = rec.mag[70, 4]               # acc equal to mag
    for k, rows in {0: [20], 1: [35], 2: [50], 3: [15, 60], 4: [70]}.items():
        marks[k] = rows
    return rec, marks


def test_reference_is_finite_and_oracles_disagree_only_there(oracle_c):
    """CPU: the reference (the NumPy restatement, bit-identical to it) stays finite through rank-1
    records; the C oracle's SVD chooses another optimal rotation there, and the two trajectories
    meet again within 1e-9 thirty records later."""
    rec, marks = _degenerate_stream()
    _, _, tro = oracle_c.run(rec, want_traj=True)
    for k, rows in marks.items():
        g, d, a, m = rec.filter(k)
        _, _, tr = ekf_numpy.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k])
        assert np.isfinite(tr).all()
        err = np.abs(tr - tro[k]).max(axis=1)
        assert err[:rows[0]].max() < 1e-12
        assert err[rows[-1] + 30:].max() < 1e-9
    for name, (acc, mag, a0, m0) in CASES.items():
        ka = abs(acc[2])
        R, B = _ref_rotation(np.asarray(a0), np.asarray(m0), np.asarray(acc), np.asarray(mag), ka, 1 - ka)
        assert np.isfinite(R).all(), name
        assert np.linalg.matrix_rank(B, tol=1e-12) == 1, name


# ------------------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


@pytest.mark.gpu
def test_percall_wahba_attains_the_reference_optimum(eng):
    """Wahba.getQuarternion per call on rank-1 B: a unit quaternion whose rotation attains the
    reference's tr(R^T B) (the optimum) and maps B's row direction onto its column direction."""
    names = list(CASES)
    acc = np.array([CASES[n][0] for n in names])
    mag = np.array([CASES[n][1] for n in names])
    a0 = np.array([CASES[n][2] for n in names])
    m0 = np.array([CASES[n][3] for n in names])
    ka = np.abs(acc[:, 2])
    q = eng.wahba_quaternion(a0, m0, acc, mag, ka, 1 - ka)
    Rg = eng.wahba_rotation(a0, m0, acc, mag, ka, 1 - ka).reshape(-1, 3, 3)
    for i, name in enumerate(names):
        R, B = _ref_rotation(a0[i], m0[i], acc[i], mag[i], ka[i], 1 - ka[i])
        best = np.trace(R.T @ B)
        for Rx in (Rg[i], _quat_rotm(q[i])):
            assert np.isfinite(Rx).all(), name
            assert np.abs(Rx @ Rx.T - np.eye(3)).max() < 1e-12 and abs(np.linalg.det(Rx) - 1) < 1e-12, name
            assert abs(np.trace(Rx.T @ B) - best) <= 1e-12 * max(1.0, abs(best)), name
        assert abs(np.linalg.norm(q[i]) - 1) < 1e-12, name
    # both samples zero: B = 0, NaN as the reference
    z = np.zeros((1, 3))
    assert np.isnan(eng.wahba_quaternion(ACC0[None], MAG0[None], z, z, np.zeros(1), np.ones(1))).all()
    Rr, _ = _ref_rotation(ACC0, MAG0, z[0], z[0], 0.0, 1.0)
    assert np.array_equal(Rr, np.eye(3))   # the reference's R2Q of the identity is 0/0


def _check_trajectory(tr, rec, marks, what):
    for k in range(rec.dtw.shape[1]):
        g, d, a, m = rec.filter(k)
        _, _, want = ekf_numpy.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k])
        assert np.isfinite(tr[:, k]).all(), (what, k)
        assert np.abs(np.linalg.norm(tr[:, k], axis=1) - 1).max() < 1e-12, (what, k)
        err = np.abs(tr[:, k] - want).max(axis=1)
        rows = marks.get(k)
        if rows is None:
            assert err.max() < 1e-9, (what, k)
        else:
            assert err[:rows[0]].max() < 1e-9, (what, k)
            assert err[rows[-1] + 30:].max() < 1e-9, (what, k, err[rows[-1]:rows[-1] + 40])


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_fused_kernel_through_rank1_records(eng, layout):
    rec, marks = _degenerate_stream()
    K, W = rec.dtw.shape[1], rec.dtw.shape[0]
    win = eng.IMUWindow.from_records(rec)
    tr = eng.BatchedEKF(K, layout=layout).run(win, want_traj=True)
    _check_trajectory(tr, rec, marks, "multi-record " + layout)
    f = eng.BatchedEKF(K, layout=layout)        # the headline launch shape: no trajectory
    f.run(win)
    assert np.abs(f.get_state()[0] - tr[-1]).max() < 1e-12
    f1 = eng.BatchedEKF(K, layout=layout)       # one-record launches (online serving)
    tr1 = np.empty_like(tr)
    for t in range(W):
        f1.run(win, n_steps=1, step0=t)
        tr1[t] = f1.get_state()[0]
    _check_trajectory(tr1, rec, marks, "one-record " + layout)


@pytest.mark.gpu
def test_handle_updates_through_rank1_records(eng):
    rec, marks = _degenerate_stream()
    K, W = rec.dtw.shape[1], rec.dtw.shape[0]
    h = eng.FilterHandle(rec.acc0, rec.mag0)
    t = np.zeros(K, np.int64)
    tr = np.empty((W, K, 4))
    for i in range(W):
        t += (rec.dtw[i] & np.uint32(synth.DT_MASK)).astype(np.int64)
        tr[i] = h.update(rec.gyro[i], t, rec.acc[i], rec.mag[i])
    _check_trajectory(tr, rec, marks, "handle")


@pytest.mark.gpu
def test_wahba_side_output_through_rank1_records(eng):
    """The pure-Wahba side output (main_file.py:40, weights 0.5 / 0.5) is a unit quaternion at every
    record and attains the reference's optimum at the rank-1 ones."""
    rec, marks = _degenerate_stream()
    win = eng.IMUWindow.from_records(rec)
    q = win.wahba_quaternions()
    # (unit to the side output's own accuracy: one Newton step on the rsqrt seed, ~1e-12 near the identity)
    assert np.isfinite(q).all() and np.abs(np.linalg.norm(q, axis=2) - 1).max() < 1e-10
    for k, rows in marks.items():
        for r in rows:
            a, m = rec.acc[r, k].astype(np.float64), rec.mag[r, k].astype(np.float64)
            R, B = _ref_rotation(rec.acc0[k], rec.mag0[k], a, m, 0.5, 0.5)
            assert abs(np.trace(_quat_rotm(q[r, k]).T @ B) - np.trace(R.T @ B)) < 1e-10, (k, r)


@pytest.mark.gpu
def test_dropin_loop_through_rank1_records(eng, monkeypatch):
    """main_file.py's loop through the drop-in modules (per-call kernels) over the same streams: finite,
    equal to the reference before the first rank-1 record, back on it 30 records after."""
    import os
    import sys

    from .conftest import ROOT
    rec, marks = _degenerate_stream()
    monkeypatch.syspath_prepend(os.path.join(ROOT, "poseestimationkf_amd", "dropin"))
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "_bootstrap"):
        sys.modules.pop(m, None)
    from ExtendedKalmanFilter import KalmanFilter
    W = rec.dtw.shape[0]
    for k in (0, 1, 3):
        g, d, a, m = rec.filter(k)
        _, _, want = ekf_numpy.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k])
        kf = KalmanFilter(0.0, rec.mag0[k], rec.acc0[k], 0.5)
        kf.setQ(1)
        kf.setR(0.1)
        X, P, T, got = np.asarray([1., 0., 0., 0.]), np.identity(4), 0.0, np.empty((W, 4))
        for i in range(W):
            T = T + d[i]
            z, Pm, Kk = kf.Prediction(g[i], T, X, P)
            X, P = kf.Correction(m[i], a[i], z, Pm, Kk)
            got[i] = X
        err = np.abs(got - want).max(axis=1)
        assert np.isfinite(got).all(), k
        assert err[:marks[k][0]].max() < 1e-11 and err[marks[k][-1] + 30:].max() < 1e-9, k
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "_bootstrap"):
        sys.modules.pop(m, None)


@pytest.mark.gpu
def test_degenerate_reference_pair_in_the_fused_kernels(eng):
    """A reference pair that does not span a plane leaves the filter's frame undefined, and with it
    every record's Wahba attitude (the reference's are its SVD's noise-chosen rotations, record after
    record).  The fused kernels, which run each filter in that frame, return NaN for a zero vector and
    an unspecified unit quaternion for an exactly parallel pair; the other filters
    of the launch are untouched."""
    rec = synth.generate(np.arange(4), 40, seed=4)
    rec.mag0[1] = 2.0 * rec.acc0[1]      # mag0 parallel to acc0
    rec.mag0[2] = 0.0                    # zero mag0
    win = eng.IMUWindow.from_records(rec)
    f = eng.BatchedEKF(4)
    f.run(win)
    X = f.get_state()[0]
    assert np.isnan(X[2]).all()
    assert np.isfinite(X[1]).all() and abs(np.linalg.norm(X[1]) - 1) < 1e-9
    for k in (0, 3):
        g, d, a, m = rec.filter(k)
        Xo = ekf_numpy.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k], record=False)[0]
        assert np.abs(X[k] - Xo).max() < 1e-9
