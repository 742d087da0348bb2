"""n = 1 per-call operators through the resident service kernel vs one launch per call.

The drop-in modules make one call per record (main_file.py:38-45).  By default those calls are
answered by a resident one-wave kernel polling pinned host memory (csrc/pekf_percall.hip,
`Service`); PEKF_PERCALL_LAUNCH launches k_call1 per call.  Both run the same device functions,
so results must agree bit for bit with each other and with the batched kernels' rows.  The service
spreads Prediction's products and Correction's P - K P over its wave's lanes, one entry per lane with
the expression the serial body uses (csrc/pekf_percall.hip, svc_predict_wave / svc_correct_wave), so
a randomised sweep over general operands checks that bit-identity too.
"""
from __future__ import annotations

import ctypes
import threading
import time

import numpy as np
import pytest

from poseestimationkf_amd._lib import PEKF_ERR_INVALID, lib


def test_mode_api_rejects_unknown_modes():
    assert lib.pekf_set_percall_mode(7) == PEKF_ERR_INVALID
    m = ctypes.c_int(-1)
    assert lib.pekf_get_percall_mode(ctypes.byref(m)) == 0 and m.value in (0, 1)


def test_dropin_module_exposes_the_mode_switch(monkeypatch):
    """The switch is reachable from the module main_file.py imports (no GPU needed to set the mode)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    monkeypatch.syspath_prepend(os.path.join(root, "poseestimationkf_amd", "dropin"))
    sys.modules.pop("ExtendedKalmanFilter", None)
    import ExtendedKalmanFilter as ekf
    prev = ekf.percall_mode()
    try:
        assert ekf.percall_mode(ekf.PERCALL_LAUNCH) == ekf.PERCALL_LAUNCH
        m = ctypes.c_int(-1)
        assert lib.pekf_get_percall_mode(ctypes.byref(m)) == 0 and m.value == ekf.PERCALL_LAUNCH
        assert ekf.percall_mode(ekf.PERCALL_SERVICE) == ekf.PERCALL_SERVICE
    finally:
        ekf.percall_mode(prev)
        for name in ("ExtendedKalmanFilter", "Wahba", "_bootstrap"):
            sys.modules.pop(name, None)


@pytest.fixture()
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    prev = engine.percall_mode()
    yield engine
    engine.percall_mode(prev)


def _pc(kat, i):
    p = [kat[k][i] for k in ("pc_gyro", "pc_dt", "pc_X", "pc_P", "pc_Q", "pc_R")]
    c = [kat[k][i] for k in ("pc_mag", "pc_acc", "pc_z", "pc_Pm", "pc_K", "pc_acc0", "pc_mag0")]
    w = [kat[k][i] for k in ("wahba_acc0", "wahba_mag0", "wahba_acc", "wahba_mag", "wahba_ka", "wahba_km")]
    return p, c, w


def _one_each(eng, kat, idx, every_op=False):
    out = []
    for i in idx:
        p, c, w = _pc(kat, i)
        r = eng.predict(*p) + eng.correct(*c) + (eng.wahba_quaternion(*w),)
        if every_op:  # the other n = 1 entry points go the same way
            j = i % 64
            r += (eng.wahba_rotation(*w), eng.rk4(kat["rk4_q0"][i], kat["rk4_dt"][i], kat["rk4_w"][i]),
                  eng.jacobian_a(kat["jac_w"][j]), eng.jacobian_b(kat["jac_q"][j]),
                  eng.comparator(kat["cmp_q1"][j], kat["cmp_q2"][j]), eng.rotmat_to_quat(kat["r2q_M"][i]))
        out.append(r)
    return out


def _same(a, b):
    for r1, r2 in zip(a, b):
        assert len(r1) == len(r2)
        for x, y in zip(r1, r2):
            assert np.array_equal(x, y, equal_nan=True)


@pytest.mark.gpu
def test_service_and_launch_identical_and_match_batched_rows(eng, kat):
    idx = range(0, 256, 7)
    eng.percall_mode(eng.PERCALL_SERVICE)
    svc = _one_each(eng, kat, idx, every_op=True)
    eng.percall_mode(eng.PERCALL_LAUNCH)
    lau = _one_each(eng, kat, idx, every_op=True)
    _same(svc, lau)
    full_p = eng.predict(*[kat[k] for k in ("pc_gyro", "pc_dt", "pc_X", "pc_P", "pc_Q", "pc_R")])
    for j, i in enumerate(idx):
        for f, x in zip(full_p, svc[j][:3]):
            assert np.array_equal(f[i], x.reshape(f[i].shape))


@pytest.mark.gpu
def test_service_survives_idle_exit_and_device_sync(eng, kat):
    eng.percall_mode(eng.PERCALL_SERVICE)
    ref = _one_each(eng, kat, [3])
    time.sleep(0.03)               # past the service's 5 ms idle limit: the kernel has left
    _same(ref, _one_each(eng, kat, [3]))
    time.sleep(0.003)              # between half and the whole idle limit: restarted deliberately
    _same(ref, _one_each(eng, kat, [3]))
    assert lib.pekf_device_sync() == 0   # stops the resident kernel first, so this returns at once
    _same(ref, _one_each(eng, kat, [3]))


@pytest.mark.gpu
def test_service_errors_like_the_reference(eng):
    eng.percall_mode(eng.PERCALL_SERVICE)
    with pytest.raises(np.linalg.LinAlgError):
        eng.predict(np.zeros(3), 1e7, [1.0, 0, 0, 0], np.zeros((4, 4)), np.zeros((3, 3)), np.zeros((4, 4)))
    with pytest.raises(np.linalg.LinAlgError):
        eng.correct([np.nan, 0, 1], [0, 0, 1.0], [1.0, 0, 0, 0], np.eye(4), np.eye(4) * 0.5, [0, 0, 1.0], [1.0, 0, 0])
    # and the service still answers afterwards
    z, _, _ = eng.predict(np.zeros(3), 1e7, [1.0, 0, 0, 0], np.eye(4), np.eye(3), np.eye(4) * 0.1)
    assert np.array_equal(z[0], np.array([1.0, 0, 0, 0]))


@pytest.mark.gpu
def test_service_from_several_threads(eng, kat):
    eng.percall_mode(eng.PERCALL_SERVICE)
    idx = list(range(64))
    ref = _one_each(eng, kat, idx)
    results, errors = {}, []

    def worker(t):
        try:
            for _ in range(5):
                results[t] = _one_each(eng, kat, idx[t::4])
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors
    for t in range(4):
        _same(ref[t::4], results[t])


def _rand_operands(rng):
    """One predict + correct operand set: general (non-symmetric) P, K; Q, R scalar or full; samples of
    any magnitude; now and then a NaN, an inf or an exactly singular S (the reference raises)."""
    g = rng.normal(0, 2, 3)
    dt = float(rng.choice([rng.uniform(0, 2e9), rng.integers(0, 2**31), 0.0]))
    X = rng.normal(0, 1, 4)
    P = rng.normal(0, 1, (4, 4)) if rng.random() < 0.5 else np.eye(4) * rng.uniform(0.1, 3)
    Q = np.eye(3) * rng.uniform(0.1, 2) if rng.random() < 0.5 else rng.normal(0, 1, (3, 3))
    R = np.eye(4) * rng.uniform(0.01, 1) if rng.random() < 0.7 else rng.normal(0, 1, (4, 4))
    mag, acc = rng.normal(0, 1, 3) * rng.uniform(0.1, 10), rng.normal(0, 1, 3) * rng.uniform(0.1, 10)
    z, Pm, K = rng.normal(0, 1, 4), rng.normal(0, 1, (4, 4)), rng.normal(0, 1, (4, 4))
    a0, m0 = rng.normal(0, 1, 3), rng.normal(0, 1, 3)
    u = rng.random()
    if u < 0.03:
        P[rng.integers(4), rng.integers(4)] = np.nan
    elif u < 0.06:
        K[rng.integers(4), rng.integers(4)] = np.inf
    elif u < 0.09:  # S = P- + R singular: zero rates and covariances
        g, P, Q, R = np.zeros(3), np.zeros((4, 4)), np.zeros((3, 3)), np.zeros((4, 4))
    return (g, dt, X, P, Q, R), (mag, acc, z, Pm, K, a0, m0)


def _call(fn, *args):
    try:
        return tuple(np.array(r, copy=True) for r in fn(*args))
    except np.linalg.LinAlgError as e:
        return ("LinAlgError", str(e))


@pytest.mark.gpu
def test_service_wave_spread_bit_identical_to_launch_on_random_operands(eng):
    rng = np.random.default_rng(20261017)
    cases = [_rand_operands(rng) for _ in range(300)]
    got = {}
    for mode in (eng.PERCALL_SERVICE, eng.PERCALL_LAUNCH):
        eng.percall_mode(mode)
        got[mode] = [(_call(eng.predict, *p), _call(eng.correct, *c)) for p, c in cases]
    raised = 0
    for a, b in zip(got[eng.PERCALL_SERVICE], got[eng.PERCALL_LAUNCH]):
        for x, y in zip(a, b):
            if isinstance(x[0], str):
                raised += 1
                assert x == y
                continue
            assert len(x) == len(y)
            for u, v in zip(x, y):
                assert np.array_equal(u, v, equal_nan=True)
    assert raised > 0  # the singular and non-finite cases were exercised
