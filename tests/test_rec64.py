"""The fused launch over FP64 records (pekf_run_rec64_dev, engine.RecordWindow64): inputs
that are float64 to begin with -- recorded logs, which the reference parses into float64
(ReadFile.py:14-21) -- reach the filter unrounded, where the 40 B stream record rounds them to f32.

* f32-representable values: bit for bit the 40 B-record launch (pekf_run_dev), the same step arithmetic;
* config 1's log (natively parsed, float64) against the reference's own X_k (main_file.py:38-47);
* float64 records with odd time differences against the NumPy restatement (oracle/ekf_numpy.py);
* ragged logs in one launch (per-filter counts), each against its own reference run."""
import gzip
import os

import numpy as np
import pytest

from oracle import ekf_numpy as npo
from poseestimationkf_amd import logformat, synth

from .conftest import GOLDEN

pytestmark = pytest.mark.gpu

ATOL_F64 = 1e-10   # FP64 kernel arithmetic vs the reference's on the same float64 records (observed ~1e-13)


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _rec64_of(eng, rec):
    """The RecordWindow64 holding exactly the values of a 40 B-record synth.Records."""
    return eng.RecordWindow64.from_arrays(rec.gyro.astype(np.float64), rec.dt_ns, rec.acc.astype(np.float64),
                                          rec.mag.astype(np.float64), rec.acc0, rec.mag0)


@pytest.mark.parametrize("want_traj,ragged", [(False, False), (True, False), (False, True), (True, True)])
def test_rec64_bit_identical_to_the_f32_record_launch(eng, want_traj, ragged):
    K, W = 300, 64     # a ragged last block; 150 records from row 5 wrap the window twice
    rec = synth.generate(np.arange(K), W, seed=41)
    counts = np.random.default_rng(2).integers(0, 151, size=K).astype(np.int32) if ragged else None
    out = []
    for win in (eng.IMUWindow.from_records(rec), _rec64_of(eng, rec)):
        f = eng.BatchedEKF(K)
        tr = f.run(win, n_steps=150, step0=5, want_traj=want_traj, counts=counts)
        out.append(f.get_state() + ((tr,) if want_traj else ()))
    for a, b in zip(*out):
        assert np.array_equal(a, b, equal_nan=True)


def test_rec64_config1_log_vs_reference(eng, tmp_path):
    """Config 1's log, parsed into float64 (pekf_log_read64), through the fused kernel: the reference's own
    X_k (c1_xk.npy, main_file.py run unchanged) within FP64 rounding -- against 5.4e-8 through the 40 B
    record (test_gpu_parity.py::test_fused_run_on_native_parsed_c1_log)."""
    log = tmp_path / "KalmanFilter.txt"
    with gzip.open(os.path.join(GOLDEN, "c1_log.txt.gz"), "rt") as fh:
        log.write_text(fh.read())
    win = eng.RecordWindow64.from_logs([str(log), str(log)])
    tr = eng.BatchedEKF(2).run(win, want_traj=True)
    want = np.load(os.path.join(GOLDEN, "c1_xk.npy"))[1:]
    err = float(np.abs(tr[:, 0] - want).max())
    print("C1 via float64 log ingest + FP64-record kernel: max |dq| = %.3e" % err)
    assert err < ATOL_F64
    assert np.array_equal(tr[:, 0], tr[:, 1])


def test_rec64_float64_records_and_odd_dts_vs_numpy(eng):
    """Records that are not f32 values, and time differences the 40 B record would escape: pauses of
    seconds, a clock stepping back, fractional nanoseconds -- dt is the float64 itself here."""
    K, W = 96, 120
    rng = np.random.default_rng(8)
    g = rng.normal(scale=0.5, size=(W, K, 3))
    a = rng.normal(scale=0.3, size=(W, K, 3)) + [0.0, 0.0, 9.8]
    m = rng.normal(scale=2.0, size=(W, K, 3)) + [20.0, 1.0, -40.0]
    dt = rng.choice([1.0e7, 2.5e7 + 0.25, 3.2e9, -4.0e6], p=[0.7, 0.2, 0.05, 0.05], size=(W, K))
    a0 = rng.normal(scale=0.3, size=(K, 3)) + [0.0, 0.0, 9.8]
    m0 = rng.normal(scale=2.0, size=(K, 3)) + [20.0, 1.0, -40.0]
    win = eng.RecordWindow64.from_arrays(g, dt, a, m, a0, m0)
    f = eng.BatchedEKF(K)
    tr = f.run(win, want_traj=True)
    worst = 0.0
    for k in range(0, K, 7):
        _, _, want = npo.run_filter(g[:, k], dt[:, k], a[:, k], m[:, k], a0[k], m0[k])
        worst = max(worst, float(np.abs(tr[:, k] - want).max()))
    print("FP64 records with odd dts vs the NumPy restatement: max |dq| = %.3e" % worst)
    assert worst < ATOL_F64


def test_rec64_ragged_logs_in_one_launch(eng, tmp_path):
    """Three logs of different lengths (written in the server's format, std::to_string's 6 decimals) in
    one launch: each filter applies exactly its own records and matches the reference loop run on its
    own log through the Python reader (logformat, ReadFile.py's float64)."""
    rng = np.random.default_rng(12)
    paths = []
    for i, n in enumerate((37, 120, 64)):
        ts = 1_000_000_000 + np.cumsum(rng.integers(5_000_000, 20_000_000, size=n + 1))
        p = tmp_path / ("log%d.txt" % i)
        logformat.write_log(str(p), ts, rng.normal(scale=0.3, size=(n, 3)),
                            rng.normal(scale=0.2, size=(n, 3)) + [0, 0, 9.8], rng.normal(size=(n, 3)) + [20, 1, -40],
                            [0.1, 0.2, 9.8], [20.0, 1.0, -40.0])
        paths.append(str(p))
    win = eng.RecordWindow64.from_logs(paths)
    assert win.window == 120 and win.counts.tolist() == [37, 120, 64]
    f = eng.BatchedEKF(3)
    f.run(win)
    X, _ = f.get_state()
    for k, p in enumerate(paths):
        g, dt, a, m, a0, m0 = logformat.log_to_arrays(logformat.read_log(p))
        Xo, _, _ = npo.run_filter(g, dt, a, m, a0, m0, record=False)
        assert float(np.abs(X[k] - Xo).max()) < ATOL_F64, k


def test_rec64_nan_record_poisons_only_its_filter(eng):
    """A NaN sample, where the reference's SVD raises LinAlgError (Wahba.py:14): inside a batch the filter
    cannot raise, so that filter's state turns NaN (pekf.h, as pekf_run_dev) and every other filter is
    unaffected -- equal to the same launch without the bad filter."""
    K, W = 128, 40
    rng = np.random.default_rng(21)
    g = rng.normal(scale=0.5, size=(W, K, 3))
    a = rng.normal(scale=0.3, size=(W, K, 3)) + [0.0, 0.0, 9.8]
    m = rng.normal(scale=2.0, size=(W, K, 3)) + [20.0, 1.0, -40.0]
    dt = np.full((W, K), 1.0e7)
    a0 = np.tile([0.1, 0.2, 9.8], (K, 1))
    m0 = np.tile([20.0, 1.0, -40.0], (K, 1))
    bad = a.copy()
    bad[17, 77, 1] = np.nan
    out = []
    for acc in (a, bad):
        f = eng.BatchedEKF(K)
        f.run(eng.RecordWindow64.from_arrays(g, dt, acc, m, a0, m0))
        out.append(f.get_state()[0])
    assert np.isnan(out[1][77]).all()
    keep = np.arange(K) != 77
    assert np.array_equal(out[0][keep], out[1][keep]) and np.isfinite(out[0]).all()


def test_rec64_side_outputs(eng):
    """The pure-gyro chain and the per-record 0.5/0.5 Wahba (main_file.py:40) over FP64 records: bit for bit
    the 40 B-record kernels on f32-representable values, and against the NumPy restatement
    (RungeKutta4 chained, Wahba.getQuarternion) on float64 records with odd time differences."""
    K, W = 130, 48
    rec = synth.generate(np.arange(K), W, seed=43)
    w32, w64 = eng.IMUWindow.from_records(rec), _rec64_of(eng, rec)
    for a, b in zip(w32.gyro_chain(n_steps=70, step0=3, want_traj=True),
                    w64.gyro_chain(n_steps=70, step0=3, want_traj=True)):
        assert np.array_equal(a, b)
    assert np.array_equal(w32.wahba_quaternions(n_steps=60, step0=9), w64.wahba_quaternions(n_steps=60, step0=9))

    rng = np.random.default_rng(44)
    K, W = 40, 50
    g = rng.normal(scale=0.5, size=(W, K, 3))
    a = rng.normal(scale=0.3, size=(W, K, 3)) + [0.0, 0.0, 9.8]
    m = rng.normal(scale=2.0, size=(W, K, 3)) + [20.0, 1.0, -40.0]
    dt = rng.choice([1.0e7, 2.5e7 + 0.25, 3.2e9, -4.0e6], p=[0.7, 0.2, 0.05, 0.05], size=(W, K))
    a0 = rng.normal(scale=0.3, size=(K, 3)) + [0.0, 0.0, 9.8]
    m0 = rng.normal(scale=2.0, size=(K, 3)) + [20.0, 1.0, -40.0]
    win = eng.RecordWindow64.from_arrays(g, dt, a, m, a0, m0)
    qf, tr = win.gyro_chain(want_traj=True)
    wq = win.wahba_quaternions()
    eg = ew = 0.0
    for k in range(0, K, 3):
        q = np.array([1.0, 0, 0, 0])
        for i in range(W):
            q = npo.rk4(q, dt[i, k], g[i, k])
            eg = max(eg, float(np.abs(tr[i, k] - q).max()))
            ew = max(ew, float(np.abs(wq[i, k] - npo.wahba_quat(a0[k], m0[k], a[i, k], m[i, k], 0.5, 0.5)).max()))
    print("FP64 records: gyro chain %.3e, 0.5/0.5 Wahba %.3e vs the NumPy restatement" % (eg, ew))
    assert eg < 1e-12 and ew < 1e-10
    assert np.array_equal(qf, tr[-1])


def test_rec64_fallback_branch_bit_identical(eng):
    """The rare fallback branch, which re-reads the record from memory (k_run64's reload, one row behind
    the cursor, wrapping at the window's start): degenerate samples (zero acc / mag, a parallel pair)
    and filters started at random attitudes (measurements far from the prediction), over a window
    replayed twice from a mid-window start -- bit for bit the 40 B-record launch on the same values."""
    from .test_degenerate_samples import _degenerate_stream
    rec, _ = _degenerate_stream(K=8, W=120, seed=9)
    K, W = 8, 120
    rng = np.random.default_rng(3)
    X0 = rng.normal(size=(K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.broadcast_to(np.identity(4), (K, 4, 4)).copy()
    out = []
    for win in (eng.IMUWindow.from_records(rec), _rec64_of(eng, rec)):
        f = eng.BatchedEKF(K)
        f.set_state(X0, P0)
        tr = f.run(win, n_steps=2 * W + 7, step0=W - 3, want_traj=True)
        out.append(f.get_state() + (tr,))
    for a, b in zip(*out):
        assert np.array_equal(a, b, equal_nan=True)
    assert np.isfinite(out[1][2]).all()
