"""HIP path (libpekf.so on an MI355X, through the C ABI) vs the oracle and the reference's golden vectors.

Tolerance: the north_star asks for quaternions within 1e-5 absolute of the NumPy reference
(ATOL_Q).  The kernels compute in FP64, so observed errors are ~1e-13; PREC_GUARD catches
a precision regression long before the 1e-5 contract would.
"""
import gzip
import os
import sys

import numpy as np
import pytest

from oracle import ekf_numpy as npo
from poseestimationkf_amd import synth

from .conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

ATOL_Q = 1e-5       # north_star: quaternion trajectories within 1e-5 absolute of NumPy
PREC_GUARD = 1e-9   # FP64 kernel vs FP64 oracle: regression guard, far inside ATOL_Q


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _maxerr(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    return float(np.nanmax(np.abs(a - b), initial=0.0))


def test_device_is_gfx950(eng):
    assert eng.device_name(0).startswith("gfx950")


# ------------------------------------------------------------ per-call operators vs golden KATs

def test_rk4(eng, kat):
    got = eng.rk4(kat["rk4_q0"], kat["rk4_dt"], kat["rk4_w"])
    assert _maxerr(got, kat["rk4_out"]) < 1e-14


def test_jacobians_norm_comparator(eng, kat):
    assert np.array_equal(eng.jacobian_a(kat["jac_w"]), kat["jac_a"])
    assert np.array_equal(eng.jacobian_b(kat["jac_q"]), kat["jac_b"])
    assert _maxerr(eng.norm(kat["norm_in"]), kat["norm_out"]) < 1e-14
    assert _maxerr(eng.comparator(kat["cmp_q1"], kat["cmp_q2"]), kat["cmp_out"]) < 1e-15


def test_r2q_bit_exact(eng, kat):
    got = eng.rotmat_to_quat(kat["r2q_M"])
    assert np.array_equal(got, kat["r2q_out"], equal_nan=True)


def test_wahba(eng, kat):
    args = [kat[k] for k in ("wahba_acc0", "wahba_mag0", "wahba_acc", "wahba_mag", "wahba_ka", "wahba_km")]
    R = eng.wahba_rotation(*args)
    q = eng.wahba_quaternion(*args)
    km = kat["wahba_km"]
    tol = np.maximum(1e-12, 1e-15 / np.abs(km))  # LAPACK's own error grows like eps/k_mag
    assert (np.abs(R - kat["wahba_R"]).reshape(len(km), -1).max(axis=1) <= tol).all()
    assert (np.abs(q - kat["wahba_q"]).max(axis=1) <= tol).all()
    assert np.allclose(q[-1], [0, 0, 0, 1], atol=1e-15)  # WahbaProblem_singularValue.py:4-24


def test_predict_correct(eng, kat):
    z, Pm, K = eng.predict(kat["pc_gyro"], kat["pc_dt"], kat["pc_X"], kat["pc_P"], kat["pc_Q"], kat["pc_R"])
    assert _maxerr(z, kat["pc_z"]) < 1e-14
    assert _maxerr(Pm, kat["pc_Pm"]) < 1e-14
    assert _maxerr(K, kat["pc_K"]) < 1e-12
    X, P = eng.correct(kat["pc_mag"], kat["pc_acc"], kat["pc_z"], kat["pc_Pm"], kat["pc_K"],
                       kat["pc_acc0"], kat["pc_mag0"])
    assert _maxerr(X, kat["pc_Xout"]) < 1e-11
    assert _maxerr(P, kat["pc_Pout"]) < 1e-13


def test_predict_singular_raises(eng):
    with pytest.raises(np.linalg.LinAlgError):
        eng.predict(np.zeros(3), 1e7, [1.0, 0, 0, 0], np.zeros((4, 4)), np.zeros((3, 3)), np.zeros((4, 4)))


def test_predict_singular_item_in_a_batch_raises(eng, kat):
    args = [kat[k][:100].copy() for k in ("pc_gyro", "pc_dt", "pc_X", "pc_P", "pc_Q", "pc_R")]
    args[3][77] = 0.0
    args[4][77] = 0.0
    args[5][77] = 0.0
    with pytest.raises(np.linalg.LinAlgError):
        eng.predict(*args)


@pytest.mark.parametrize("start,n", [(0, 1), (0, 2), (0, 63), (0, 64), (0, 65), (3, 130), (7, 249)])
def test_percall_items_independent_of_tiling(eng, kat, start, n):
    """The batched per-call kernels move operands in 64-item wave tiles (csrc/pekf_tile.hpp):
    any slice -- short last tile, unaligned start, n = 1 (the by-value k_call1 launch) -- gives
    the rows of the full-batch call bit for bit."""
    sl = slice(start, start + n)
    pc = [kat[k] for k in ("pc_gyro", "pc_dt", "pc_X", "pc_P", "pc_Q", "pc_R")]
    full = eng.predict(*pc)
    part = eng.predict(*[a[sl] for a in pc])
    for f, p in zip(full, part):
        assert np.array_equal(f[sl], p)
    cc = [kat[k] for k in ("pc_mag", "pc_acc", "pc_z", "pc_Pm", "pc_K", "pc_acc0", "pc_mag0")]
    for f, p in zip(eng.correct(*cc), eng.correct(*[a[sl] for a in cc])):
        assert np.array_equal(f[sl], p)
    wa = [kat[k] for k in ("wahba_acc0", "wahba_mag0", "wahba_acc", "wahba_mag", "wahba_ka", "wahba_km")]
    assert np.array_equal(eng.wahba_quaternion(*wa)[sl], eng.wahba_quaternion(*[a[sl] for a in wa]))
    assert np.array_equal(eng.wahba_rotation(*wa)[sl], eng.wahba_rotation(*[a[sl] for a in wa]))
    rk = [kat[k] for k in ("rk4_q0", "rk4_dt", "rk4_w")]
    assert np.array_equal(eng.rk4(*rk)[sl], eng.rk4(*[a[sl] for a in rk]))
    assert np.array_equal(eng.rotmat_to_quat(kat["r2q_M"])[sl], eng.rotmat_to_quat(kat["r2q_M"][sl]),
                          equal_nan=True)
    jq = np.concatenate([kat["jac_q"]] * 4)
    assert np.array_equal(eng.jacobian_b(jq)[sl], eng.jacobian_b(jq[sl]))   # W = 12: the general slot path


def test_empty_batch_is_noop(eng):
    assert eng.rk4(np.zeros((0, 4)), np.zeros(0), np.zeros((0, 3))).shape == (0, 4)


# ------------------------------------------------------------ fused kernel vs reference trajectories

@pytest.mark.parametrize("tag", ["", "miss_"])
def test_fused_run_matches_reference_trajectory(eng, traj, tag):
    win = eng.IMUWindow.from_planes(traj[tag + "gd"], traj[tag + "am"], traj[tag + "my"],
                                    traj[tag + "acc0"], traj[tag + "mag0"])
    f = eng.BatchedEKF(win.batch, q=1.0, r=0.1)
    tr = f.run(win, want_traj=True)
    err = _maxerr(tr, traj[tag + "traj"])
    print("fused vs reference (%s): max |dq| = %.3e" % (tag or "full", err))
    assert err < ATOL_Q
    assert err < PREC_GUARD


@pytest.mark.parametrize("tag", ["", "miss_"])
def test_fused_mixed_precision_within_tolerance(eng, traj, tag):
    """Opt-in covariance-in-FP32 path: quaternions must still meet the 1e-5 contract."""
    win = eng.IMUWindow.from_planes(traj[tag + "gd"], traj[tag + "am"], traj[tag + "my"],
                                    traj[tag + "acc0"], traj[tag + "mag0"])
    tr = eng.BatchedEKF(win.batch, precision="mixed").run(win, want_traj=True)
    err = _maxerr(tr, traj[tag + "traj"])
    print("mixed precision vs reference (%s): max |dq| = %.3e" % (tag or "full", err))
    assert err < ATOL_Q
    assert err < 1e-6


def test_device_generator_bit_identical_to_host(eng):
    K, W = 1000, 48
    win = eng.IMUWindow(K, W).synthesize(seed=synth.DEFAULT_SEED, first_filter=123, missing=True)
    dev = win.download_filters(np.arange(K))
    host = synth.generate(np.arange(123, 123 + K), W, seed=synth.DEFAULT_SEED, missing=True)
    for name in ("gyro", "acc", "mag"):
        assert np.array_equal(getattr(dev, name).view(np.uint32), getattr(host, name).view(np.uint32)), name
    assert np.array_equal(dev.dtw, host.dtw)
    assert np.array_equal(dev.acc0, host.acc0) and np.array_equal(dev.mag0, host.mag0)


def test_cyclic_window_ragged_batch_and_chunking(eng, oracle_c):
    K, W = 300, 64  # 300 filters: not a multiple of the 256-lane block
    rec = synth.generate(np.arange(K), W, seed=99, missing=True)
    win = eng.IMUWindow.from_records(rec)
    f = eng.BatchedEKF(K)
    f.run(win, n_steps=150, step0=5)            # wraps the window twice
    Xg, Pg = f.get_state()
    Xo, Po, _ = oracle_c.run(rec, n_steps=150, step0=5)
    assert _maxerr(Xg, Xo) < PREC_GUARD
    assert _maxerr(Pg, Po) < PREC_GUARD
    # chunked launches continue where a single launch would be.  Each launch boundary rotates the
    # state out of and back into the reference frame's basis and converts N <-> P, so the chunked
    # run rounds differently at the boundary; the gain K = I - r S^-1 damps such ulp-level
    # differences within a few records.  Checked to a rounding-level tolerance,
    # not bit for bit: the agreement must not depend on the seed or the noise scales.
    g = eng.BatchedEKF(K)
    g.run(win, n_steps=70, step0=5)
    g.run(win, n_steps=80, step0=75)
    X2, P2 = g.get_state()
    assert _maxerr(X2, Xg) <= 1e-15
    assert _maxerr(P2, Pg) <= 1e-15 * max(1.0, float(np.abs(Pg).max()))


def test_set_state_roundtrip_and_resume(eng, oracle_c):
    K, W = 64, 40
    rec = synth.generate(np.arange(K), W, seed=5)
    win = eng.IMUWindow.from_records(rec)
    X0, P0, _ = oracle_c.run(rec, n_steps=17)          # start from a mid-run state
    f = eng.BatchedEKF(K)
    f.set_state(X0, P0)
    Xs, Ps = f.get_state()
    assert np.array_equal(Xs, X0) and np.array_equal(Ps, P0)
    f.run(win, n_steps=23, step0=17)
    Xo, _, _ = oracle_c.run(rec, n_steps=40)
    assert _maxerr(f.get_state()[0], Xo) < PREC_GUARD


@pytest.mark.parametrize("q,r", [(0.37, 2.5), (4.0, 0.01), (1e-3, 1.0)])
def test_fused_run_other_noise_scales(eng, oracle_c, q, r):
    """setQ(q) / setR(r) other than main_file.py's (1, 0.1): the fused algebra uses Q = qI, R = rI."""
    K, W = 128, 300
    rec = synth.generate(np.arange(K), W, seed=17, missing=True)
    f = eng.BatchedEKF(K, q=q, r=r)
    tr = f.run(eng.IMUWindow.from_records(rec), want_traj=True)
    Xo, Po, to = oracle_c.run(rec, q=q, r=r, want_traj=True)
    assert _maxerr(tr.transpose(1, 0, 2), to) < PREC_GUARD
    assert _maxerr(f.get_state()[1], Po) < PREC_GUARD * max(1.0, r)
    # the instantiation without trajectory output (q_W recomputed, the covariance carried as N
    # with beta = sqrt(2) r, X unnormalised between records) in two chunks
    g = eng.BatchedEKF(K, q=q, r=r)
    win = eng.IMUWindow.from_records(rec)
    g.run(win, n_steps=120)
    g.run(win, n_steps=W - 120, step0=120)
    X, P = g.get_state()
    assert _maxerr(X, Xo) < PREC_GUARD
    assert _maxerr(P, Po) < PREC_GUARD * max(1.0, r)
    assert np.abs(np.linalg.norm(X, axis=1) - 1.0).max() < 1e-13


def test_scale_c2_batch_sampled_against_oracle(eng, oracle_c):
    """Config-2 batch (65,536 filters) on a device-generated window; 64 sampled filters re-run on the host."""
    B, W, N = 65536, 128, 384
    win = eng.IMUWindow(B, W).synthesize(seed=synth.DEFAULT_SEED)
    f = eng.BatchedEKF(B)
    f.run(win, n_steps=N)
    X, P = f.get_state()
    assert np.isfinite(X).all()
    assert np.abs(np.linalg.norm(X, axis=1) - 1).max() < 1e-12   # size-independent property
    assert np.abs(P - P.transpose(0, 2, 1)).max() == 0.0          # stored symmetric
    cols = np.linspace(0, B - 1, 64).astype(np.int64)
    rec = synth.generate(cols, W, seed=synth.DEFAULT_SEED)
    Xo, _, _ = oracle_c.run(rec, n_steps=N)
    err = _maxerr(X[cols], Xo)
    print("C2 sampled parity: max |dq| = %.3e" % err)
    assert err < ATOL_Q and err < PREC_GUARD


@pytest.mark.parametrize("name,batch,missing", [("C2", 65536, False), ("C3", 1 << 20, False),
                                                ("C5", 1 << 20, True)])
def test_full_size_configs_sampled_against_oracle(eng, oracle_c, name, batch, missing):
    """BASELINE.json configs 2/3/5 at full size (10,000 records over a 1,024-record resident window):
    64 filters spread over the batch re-run by the C oracle; every filter's X stays unit-norm."""
    W, N = 1024, 10000
    win = eng.IMUWindow(batch, W).synthesize(seed=synth.DEFAULT_SEED, missing=missing)
    f = eng.BatchedEKF(batch)
    f.run(win, n_steps=N)
    X, P = f.get_state()
    assert np.isfinite(X).all() and np.isfinite(P).all()
    assert np.abs(np.linalg.norm(X, axis=1) - 1).max() < 1e-12
    eig = np.linalg.eigvalsh(P[:: max(1, batch // 4096)])
    assert eig.min() > 0                                 # covariance stays positive definite
    if not missing:                                      # after a correction P = r I - r^2 S^-1 < r I
        assert eig.max() < 0.1 + 1e-12
    cols = np.linspace(0, batch - 1, 64).astype(np.int64)
    rec = synth.generate(cols, W, seed=synth.DEFAULT_SEED, missing=missing)
    Xo, _, _ = oracle_c.run(rec, n_steps=N)
    err = _maxerr(X[cols], Xo)
    print("%s full size (%d filters x %d records): sampled max |dq| = %.3e" % (name, batch, N, err))
    assert err < ATOL_Q and err < PREC_GUARD


@pytest.mark.parametrize("W,step0,n", [(1, 0, 7), (2, 1, 7), (3, 2, 8)])
def test_tiny_windows_replayed(eng, oracle_c, W, step0, n):
    """Windows of 1-3 rows replayed for more records than they hold (every record advances the row
    cursor past the window's end), odd and even launch lengths, against the C oracle."""
    K = 96
    rec = synth.generate(np.arange(K), W, seed=17 + W)
    win = eng.IMUWindow.from_records(rec)
    f = eng.BatchedEKF(K)
    f.run(win, n_steps=n, step0=step0)
    Xg, Pg = f.get_state()
    Xo, Po, _ = oracle_c.run(rec, n_steps=n, step0=step0)
    assert _maxerr(Xg, Xo) < PREC_GUARD
    assert _maxerr(Pg, Po) < PREC_GUARD


def test_row_chunks_wrap_and_offset_start(eng, oracle_c):
    """Records are read through descriptors of a chunk of rows with the row offset in soffset
    (RowCursor, csrc/pekf_step.hpp).  At 16M filters a row of the 16 B planes is 256 MiB, so a chunk
    is 8 rows: a 13-row window started at row 5 and run for 30 records crosses chunk ends inside the
    window, the window's short last chunk and wraps twice; a second launch resumes at row 9."""
    B, W = 1 << 24, 13
    win = eng.IMUWindow(B, W).synthesize(seed=5)
    f = eng.BatchedEKF(B)
    f.run(win, n_steps=30, step0=5)
    f.run(win, n_steps=11, step0=9)
    X = f.X.download((B, 4), np.float64)
    cols = np.array([0, 1, 63, 64, 12345, B // 2, B - 65, B - 1])
    rec = synth.generate(cols, W, seed=5)
    Xo, Po, _ = oracle_c.run(rec, n_steps=30, step0=5)
    Xo, _, _ = oracle_c.run(rec, n_steps=11, step0=9, X=Xo, P=Po)
    err = _maxerr(X[cols], Xo)
    print("row chunks (16M filters, 8-row chunks, 13-row window): max |dq| = %.3e" % err)
    assert err < ATOL_Q and err < PREC_GUARD


def test_batch_of_one(eng, traj):
    sl = slice(0, 1)
    win = eng.IMUWindow.from_planes(traj["gd"][:, sl], traj["am"][:, sl], traj["my"][:, sl],
                                    traj["acc0"][sl], traj["mag0"][sl])
    tr = eng.BatchedEKF(1).run(win, want_traj=True)
    assert _maxerr(tr, traj["traj"][:, sl]) < PREC_GUARD


# ------------------------------------------------------------ config 1: the drop-in modules

def test_dropin_main_file_loop_on_c1_log(eng, tmp_path, monkeypatch):
    """main_file.py:11-47 on the config-1 log, through the drop-in modules, vs main_file's own X_k."""
    log = tmp_path / "KalmanFilter.txt"
    with gzip.open(os.path.join(GOLDEN, "c1_log.txt.gz"), "rt") as fh:
        log.write_text(fh.read())
    monkeypatch.setenv("PEKF_LOG_PATH", str(log))
    monkeypatch.syspath_prepend(os.path.join(ROOT, "poseestimationkf_amd", "dropin"))
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "ReadFile", "_bootstrap"):
        sys.modules.pop(m, None)
    from ExtendedKalmanFilter import KalmanFilter
    from ReadFile import getData
    from UtilityFunctions import DimensionalSplit, norm
    from Wahba import Wahba

    g = getData()
    w = Wahba(g.acc_0, g.mag_0)
    k = KalmanFilter(g.timestamp[0][0], g.mag_0, g.acc_0, 0.5)
    k.setQ(1)
    k.setR(0.1)
    P = np.identity(4)
    g.timestamp = g.timestamp[1:]
    X = np.asarray([1., 0., 0., 0.])
    X_k = [X]
    for i in range(len(g.acc_1)):
        z_k, P, K_k = k.Prediction(g.gyro[i], g.timestamp[i][0], X, P)
        w.getQuarternion(g.acc_1[i], g.mag_1[i], 0.5, 0.5)
        X, P = k.Correction(g.mag_1[i], g.acc_1[i], z_k, P, K_k)
        X_k.append(X)
    want = np.load(os.path.join(GOLDEN, "c1_xk.npy"))
    err = _maxerr(np.array(X_k), want)
    print("C1 drop-in vs main_file.py: max |dq| = %.3e over %d steps" % (err, len(X_k) - 1))
    assert err < ATOL_Q and err < PREC_GUARD
    assert len(DimensionalSplit(X_k)) == 4
    assert abs(norm(X_k[-1]) - 1.0) < 1e-14


def test_fused_run_on_native_parsed_c1_log(eng, tmp_path):
    """Config 1 through the batched path: log -> pekf_log_read (f32 records) -> fused kernel."""
    log = tmp_path / "KalmanFilter.txt"
    with gzip.open(os.path.join(GOLDEN, "c1_log.txt.gz"), "rt") as fh:
        log.write_text(fh.read())
    win = eng.IMUWindow.from_logs([str(log), str(log)])  # two filters, same trace
    tr = eng.BatchedEKF(2).run(win, want_traj=True)
    want = np.load(os.path.join(GOLDEN, "c1_xk.npy"))[1:]
    err = _maxerr(tr[:, 0], want)
    print("C1 via native log ingest + fused kernel: max |dq| = %.3e (inputs rounded to f32)" % err)
    # the batched stream path stores the log's float64 samples as f32 (the 40 B record): measured 5.4e-8
    # against the reference's own X_k (NumPy restatement on the same f32-rounded records: 5.380e-8), so
    # the bound is that rounding, not the north_star's 1e-5 (the drop-in loop keeps FP64: 1.1e-13)
    assert err < 1e-7
    assert np.array_equal(tr[:, 0], tr[:, 1])


def test_dropin_returns_fresh_arrays_and_keeps_inputs(eng, monkeypatch):
    monkeypatch.syspath_prepend(os.path.join(ROOT, "poseestimationkf_amd", "dropin"))
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "_bootstrap"):
        sys.modules.pop(m, None)
    from ExtendedKalmanFilter import KalmanFilter
    k = KalmanFilter(0.0, [0.5, 0.0, -0.86], [0.0, 0.1, 0.99], 0.5)
    k.setQ(1)
    k.setR(0.1)
    X, P = np.asarray([1., 0., 0., 0.]), np.identity(4)
    Xc, Pc = X.copy(), P.copy()
    z, Pm, K = k.Prediction([0.1, -0.2, 0.3], 1e7, X, P)
    assert np.array_equal(X, Xc) and np.array_equal(P, Pc) and k.previousT == 1e7
    X1, P1 = k.Correction([0.5, 0.01, -0.86], [0.01, 0.1, 0.99], z, Pm, K)
    want = npo.correct([0.5, 0.01, -0.86], [0.01, 0.1, 0.99], z, Pm, K, [0.0, 0.1, 0.99], [0.5, 0.0, -0.86])
    assert _maxerr(X1, want[0]) < 1e-13 and _maxerr(P1, want[1]) < 1e-13
    assert X1 is not z and P1 is not Pm


def test_dropin_north_star_aliases_equal_real_names(eng, monkeypatch):
    """KalmanFilter.predict / update and Wahba.solve (the north_star's call surface) are the
    reference's Prediction / Correction / getQuarternion (ExtendedKalmanFilter.py:58,70, Wahba.py:49):
    bit for bit the same results, and previousT advances the same way."""
    monkeypatch.syspath_prepend(os.path.join(ROOT, "poseestimationkf_amd", "dropin"))
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "_bootstrap"):
        sys.modules.pop(m, None)
    from ExtendedKalmanFilter import KalmanFilter
    from Wahba import Wahba
    assert KalmanFilter.predict is KalmanFilter.Prediction and KalmanFilter.update is KalmanFilter.Correction
    assert Wahba.solve is Wahba.getQuarternion
    acc0, mag0 = [0.0, 0.1, 0.99], [0.5, 0.0, -0.86]
    k1, k2 = KalmanFilter(0.0, mag0, acc0, 0.5), KalmanFilter(0.0, mag0, acc0, 0.5)
    for k in (k1, k2):
        k.setQ(1)
        k.setR(0.1)
    rng = np.random.default_rng(11)
    X1 = X2 = np.asarray([1., 0., 0., 0.])
    P1 = P2 = np.identity(4)
    for i in range(20):
        g, a, m = rng.normal(0, 0.3, 3), rng.normal([0, 0.1, 0.99], 0.02), rng.normal([0.5, 0, -0.86], 0.02)
        t = 1e7 * (i + 1)
        z1, Pm1, K1 = k1.Prediction(g, t, X1, P1)
        z2, Pm2, K2 = k2.predict(g, t, X2, P2)
        assert np.array_equal(z1, z2) and np.array_equal(Pm1, Pm2) and np.array_equal(K1, K2)
        assert k1.previousT == k2.previousT == t
        X1, P1 = k1.Correction(m, a, z1, Pm1, K1)
        X2, P2 = k2.update(m, a, z2, Pm2, K2)
        assert np.array_equal(X1, X2) and np.array_equal(P1, P2)
        w = Wahba(acc0, mag0)
        assert np.array_equal(w.solve(a, m, 0.5, 0.5), w.getQuarternion(a, m, 0.5, 0.5))
    want = npo.correct(m, a, z1, Pm1, K1, acc0, mag0)
    assert _maxerr(X2, want[0]) < 1e-11   # raw samples: k_mag = 1 - |acc_z| ~ 0.01, LAPACK's bound ~ eps / k_mag


@pytest.mark.gpu
def test_fused_measurement_far_from_prediction(eng):
    """Filters started at random attitudes, so early Wahba measurements Y lie anywhere relative to
    the prediction z, including |Y.z| < 1/4 where the fused kernel leaves Y = normalise(4qq^T z) for
    the reference's branch formula and strict '<' flip (ExtendedKalmanFilter.py:73-75)."""
    K, W = 256, 30
    rec = synth.generate(np.arange(K), W, seed=11)
    rng = np.random.default_rng(3)
    X0 = rng.normal(size=(K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.broadcast_to(np.identity(4), (K, 4, 4)).copy()
    f = eng.BatchedEKF(K)
    f.set_state(X0, P0)
    tr = f.run(eng.IMUWindow.from_records(rec), want_traj=True)
    Q, R = np.identity(3), np.identity(4) * 0.1
    far = 0
    for k in range(K):
        g, d, a, m = rec.filter(k)
        z, _, _ = npo.predict(g[0], d[0], X0[k], P0[k], Q, R)
        y = npo.wahba_quat(rec.acc0[k], rec.mag0[k], a[0], m[0], abs(a[0][2]), 1 - abs(a[0][2]))
        far += abs(float(np.dot(y, z))) < 0.25
        _, _, want = npo.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k], X0=X0[k], P0=P0[k])
        assert _maxerr(tr[:, k], want) < PREC_GUARD, k
    assert far >= 20  # the fallback lanes really ran


@pytest.mark.gpu
def test_fused_non_unit_initial_state(eng):
    """A state set to a non-unit X (set_state) keeps its |X|^2 in the first record's Jb term and RK4
    normalisation (ExtendedKalmanFilter.py:60-62), as the reference; unit states snap |X|^2 to 1."""
    K, W = 64, 20
    rec = synth.generate(np.arange(K), W, seed=13)
    rng = np.random.default_rng(5)
    X0 = rng.normal(size=(K, 4))
    X0 *= (rng.uniform(0.3, 3.0, size=K) / np.linalg.norm(X0, axis=1))[:, None]
    X0[::4] /= np.linalg.norm(X0[::4], axis=1, keepdims=True)          # some exactly-normalised rows
    P0 = np.broadcast_to(np.identity(4) * 0.3, (K, 4, 4)).copy()
    f = eng.BatchedEKF(K)
    f.set_state(X0, P0)
    tr = f.run(eng.IMUWindow.from_records(rec), want_traj=True)
    _, Pf = f.get_state()
    for k in range(K):
        g, d, a, m = rec.filter(k)
        _, Pk, want = npo.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k], X0=X0[k], P0=P0[k])
        assert _maxerr(tr[:, k], want) < PREC_GUARD, k
        assert _maxerr(Pf[k], Pk) < PREC_GUARD, k


@pytest.mark.gpu
def test_fused_arbitrary_reference_frames(eng):
    """Reference pairs (acc0, mag0) in arbitrary directions: every filter's Wahba reference frame,
    and with it the basis the multi-record kernel runs the filter in (its quaternion q_W, all four
    of Shepperd's branches), differs; records stay in the body frame, so the filters start far from
    the attitude they converge to."""
    from scipy.spatial.transform import Rotation
    K, W = 256, 40
    rec = synth.generate(np.arange(K), W, seed=23)
    Rk = Rotation.random(K, random_state=7).as_matrix()
    rec.acc0[:] = np.einsum("kij,kj->ki", Rk, rec.acc0)
    rec.mag0[:] = np.einsum("kij,kj->ki", Rk, rec.mag0)
    tr = eng.BatchedEKF(K).run(eng.IMUWindow.from_records(rec), want_traj=True)
    for k in range(K):
        g, d, a, m = rec.filter(k)
        _, _, want = npo.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k])
        assert _maxerr(tr[:, k], want) < PREC_GUARD, k
