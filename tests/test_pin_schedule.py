"""The schedules of the multi-record kernel against the compiler's own order (PEKF_RUN_PIN=0), bit for
bit, and against the oracle (csrc/pekf_step.hpp):
* PIN (k_run<..., PIN = true>: the Schur inverse computed in the basic block of the Wahba chain; the
  default for FP64 launches without trajectories or counts), PEKF_RUN_PIN=1 PEKF_RUN_HOIST=0;
* HOIST (the Correction's state-independent half ahead of the missing-magnetometer branch; selected
  on top of PIN for launches of at most one wave per SIMD), PEKF_RUN_PIN=1 PEKF_RUN_HOIST=1."""
import numpy as np
import pytest

from oracle import ekf_numpy as npo
from poseestimationkf_amd import synth

pytestmark = pytest.mark.gpu

PREC_GUARD = 1e-9


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


SCHEDULES = {"default": ("0", "0"), "pin": ("1", "0"), "hoist": ("1", "1")}


def _run(eng, monkeypatch, sched, K, win, n, step0=0, layout="aos", X0=None, P0=None, chunks=None):
    pin, hoist = SCHEDULES[sched]
    monkeypatch.setenv("PEKF_RUN_PIN", pin)
    monkeypatch.setenv("PEKF_RUN_HOIST", hoist)
    f = eng.BatchedEKF(K, layout=layout)
    if X0 is not None:
        f.set_state(X0, P0)
    for n_i, s_i in chunks or [(n, step0)]:
        f.run(win, n_steps=n_i, step0=s_i)
    return f.get_state()


def _same(a, b):
    assert np.array_equal(a, b, equal_nan=True), float(np.nanmax(np.abs(a - b)))


def _schedules(eng, monkeypatch, *args, **kw):
    """(X, P) of the PIN schedule, after checking that HOIST and the default order give the same bits."""
    Xs, Ps = _run(eng, monkeypatch, "pin", *args, **kw)
    for other in ("hoist", "default"):
        X1, P1 = _run(eng, monkeypatch, other, *args, **kw)
        _same(Xs, X1)
        _same(Ps, P1)
    return Xs, Ps


@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_pin_bit_identical_ragged_missing_wrapping(eng, monkeypatch, oracle_c, layout):
    # 300 filters (a ragged last block); 30 % missing magnetometer records; 150 records from row 5 of a 64-row window (two wraps)
    K, W = 300, 64
    rec = synth.generate(np.arange(K), W, seed=99, missing=True)
    win = eng.IMUWindow.from_records(rec)
    Xs, Ps = _schedules(eng, monkeypatch, K, win, 150, 5, layout)
    Xo, Po, _ = oracle_c.run(rec, n_steps=150, step0=5)
    assert float(np.abs(Xs - Xo).max()) < PREC_GUARD


@pytest.mark.parametrize("n", [1, 2, 3])
def test_pin_short_launches(eng, monkeypatch, n):
    # 1 record takes the one-record kernel; 2 and 3 exercise the loop's odd / even exits
    K, W = 128, 8
    rec = synth.generate(np.arange(K), W, seed=4)
    win = eng.IMUWindow.from_records(rec)
    _schedules(eng, monkeypatch, K, win, n)


def test_pin_far_measurements_take_the_fallback(eng, monkeypatch):
    """Random initial attitudes: early measurements with |Y.z| < 1/4 take the reference's branch
    formula and flip, the branch the PIN schedule moves the Schur inverse ahead of."""
    K, W = 256, 30
    rec = synth.generate(np.arange(K), W, seed=11)
    rng = np.random.default_rng(3)
    X0 = rng.normal(size=(K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.broadcast_to(np.identity(4), (K, 4, 4)).copy()
    win = eng.IMUWindow.from_records(rec)
    Xs, Ps = _schedules(eng, monkeypatch, K, win, W, X0=X0, P0=P0)
    for k in range(0, K, 17):
        g, d, a, m = rec.filter(k)
        _, _, want = npo.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k], X0=X0[k], P0=P0[k])
        assert float(np.abs(Xs[k] - want[-1]).max()) < PREC_GUARD, k


def test_pin_non_unit_state_and_chunks(eng, monkeypatch):
    """A non-unit initial X (its |X|^2 enters the first record) and a run split over two launches."""
    K, W = 64, 20
    rec = synth.generate(np.arange(K), W, seed=13)
    rng = np.random.default_rng(5)
    X0 = rng.normal(size=(K, 4))
    X0 *= (rng.uniform(0.3, 3.0, size=K) / np.linalg.norm(X0, axis=1))[:, None]
    P0 = np.broadcast_to(np.identity(4) * 0.3, (K, 4, 4)).copy()
    win = eng.IMUWindow.from_records(rec)
    for chunks in ([(W, 0)], [(7, 0), (13, 7)]):
        _schedules(eng, monkeypatch, K, win, None, X0=X0, P0=P0, chunks=chunks)


def test_pin_config2_sampled(eng, monkeypatch, oracle_c):
    """Config 2's batch (65,536 filters: one wave per SIMD, so the library picks PIN + HOIST) over a
    64-row window, 200 records: bit-identical to every other schedule, sampled filters against the oracle."""
    K, W, N = 65536, 64, 200
    win = eng.IMUWindow(K, W).synthesize(seed=synth.DEFAULT_SEED, missing=True)
    monkeypatch.delenv("PEKF_RUN_PIN", raising=False)
    monkeypatch.delenv("PEKF_RUN_HOIST", raising=False)
    f = eng.BatchedEKF(K)
    f.run(win, n_steps=N)
    Xa, Pa = f.get_state()
    X1, P1 = _schedules(eng, monkeypatch, K, win, N)
    _same(Xa, X1)
    _same(Pa, P1)
    cols = np.array([0, 63, 64, 40000, K - 1])
    rec = synth.generate(cols, W, seed=synth.DEFAULT_SEED, missing=True)
    Xo, _, _ = oracle_c.run(rec, n_steps=N)
    assert float(np.abs(Xa[cols] - Xo).max()) < PREC_GUARD
