"""Edge cases the reference accepts (tests/golden/edge.npz, generated from the reference):
raw-unit sensor values (|acc| ~ 9.81 so the Wahba weight k_mag = 1-|acc_z| < 0), zero rates,
dt = 0 and 1-5 s gaps, a NaN sample (the reference raises LinAlgError from np.linalg.svd),
non-symmetric P and non-scalar Q/R in the per-call operators."""
import os

import numpy as np
import pytest

from oracle import ekf_numpy as npo
from poseestimationkf_amd import synth

from .conftest import GOLDEN

ATOL_Q = 1e-5
PREC_GUARD = 1e-9


@pytest.fixture(scope="module")
def edge():
    with np.load(os.path.join(GOLDEN, "edge.npz")) as z:
        return {k: z[k] for k in z.files}


def _rec(e, tag):
    return synth.unpack_planes(e[tag + "gd"], e[tag + "am"], e[tag + "my"], e[tag + "acc0"], e[tag + "mag0"])


def _wahba_args(e):
    return [e[k] for k in ("ew_acc0", "ew_mag0", "ew_acc", "ew_mag", "ew_ka", "ew_km")]


# ------------------------------------------------------------------ oracle (CPU)

def test_raw_unit_inputs_really_give_negative_k_mag(edge):
    rec = _rec(edge, "raw_")
    assert (1 - np.abs(rec.acc[..., 2].astype(np.float64)) < 0).mean() > 0.3
    assert (edge["ew_km"] < 0).mean() > 0.3


def test_numpy_port_raw_trajectory_bit_exact(edge):
    rec = _rec(edge, "raw_")
    for f in range(rec.acc0.shape[0]):
        g, d, a, m = rec.filter(f)
        with np.errstate(all="ignore"):
            _, _, tr = npo.run_filter(g, d, a, m, rec.acc0[f], rec.mag0[f])
        assert np.array_equal(tr, edge["raw_traj"][:, f])


def test_c_oracle_raw_trajectory(edge, oracle_c):
    rec = _rec(edge, "raw_")
    _, _, tr = oracle_c.run(rec, want_traj=True)
    assert np.abs(tr.transpose(1, 0, 2) - edge["raw_traj"]).max() < 1e-10


def test_c_oracle_wahba_negative_weights(edge, oracle_c):
    R = np.array([oracle_c.wahba_rotation(*a) for a in zip(*_wahba_args(edge))])
    assert np.abs(R - edge["ew_R"]).max() < 1e-12


def test_nan_sample_raises_in_reference(edge):
    assert int(edge["nan_raised_at"]) == 20
    rec = _rec(edge, "nan_")
    g, d, a, m = rec.filter(1)
    with pytest.raises(np.linalg.LinAlgError):
        npo.run_filter(g, d, a, m, rec.acc0[1], rec.mag0[1])


# ------------------------------------------------------------------ HIP path (GPU)

@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["f64", "mixed"])
def test_fused_raw_unit_trajectory(eng, edge, precision):
    win = eng.IMUWindow.from_planes(edge["raw_gd"], edge["raw_am"], edge["raw_my"], edge["raw_acc0"],
                                    edge["raw_mag0"])
    tr = eng.BatchedEKF(win.batch, precision=precision).run(win, want_traj=True)
    err = float(np.abs(tr - edge["raw_traj"]).max())
    print("fused %s, raw-unit inputs (k_mag < 0, zero rates, dt = 0 / 1 s): max |dq| = %.3e" % (precision, err))
    assert err < ATOL_Q
    if precision == "f64":
        assert err < PREC_GUARD


@pytest.mark.gpu
def test_fused_nan_sample_poisons_only_its_filter(eng, edge):
    win = eng.IMUWindow.from_planes(edge["nan_gd"], edge["nan_am"], edge["nan_my"], edge["nan_acc0"],
                                    edge["nan_mag0"])
    tr = eng.BatchedEKF(win.batch).run(win, want_traj=True)
    assert np.abs(tr[:, 0] - edge["nan_clean_traj"]).max() < PREC_GUARD
    assert np.abs(tr[:20, 1] - edge["nan_partial_traj"]).max() < PREC_GUARD
    assert np.isnan(tr[20:, 1]).all()


@pytest.mark.gpu
def test_percall_wahba_negative_weights(eng, edge):
    R = eng.wahba_rotation(*_wahba_args(edge))
    q = eng.wahba_quaternion(*_wahba_args(edge))
    assert np.abs(R - edge["ew_R"]).max() < 1e-12
    assert np.abs(q - edge["ew_q"]).max() < 1e-12


@pytest.mark.gpu
def test_percall_general_predict_correct(eng, edge):
    e = edge
    z, Pm, K = eng.predict(e["ep_gyro"], e["ep_dt"], e["ep_X"], e["ep_P"], e["ep_Q"], e["ep_R"])
    assert np.abs(z - e["ep_z"]).max() < 1e-14
    assert np.abs(Pm - e["ep_Pm"]).max() < 1e-13
    assert np.abs(K - e["ep_K"]).max() < 1e-12
    X, P = eng.correct(e["ep_mag"], e["ep_acc"], e["ep_z"], e["ep_Pm"], e["ep_K"], e["ep_acc0"], e["ep_mag0"])
    assert np.abs(X - e["ep_Xout"]).max() < 1e-12
    assert np.abs(P - e["ep_Pout"]).max() < 1e-13


@pytest.mark.gpu
def test_percall_nan_raises_like_numpy_svd(eng):
    acc0, mag0 = [0.0, 0.0, 1.0], [0.5, 0.0, -0.866]
    with pytest.raises(np.linalg.LinAlgError, match="SVD did not converge"):
        eng.wahba_quaternion(acc0, mag0, [np.nan, 0.0, 1.0], [0.5, 0.0, -0.86], [1.0], [0.0])
    with pytest.raises(np.linalg.LinAlgError, match="SVD did not converge"):
        eng.correct([0.5, 0.0, -0.86], [np.nan, 0.0, 1.0], [1.0, 0, 0, 0], np.eye(4), np.eye(4) * 0.5, acc0, mag0)
    # NaN in P does not raise in np.linalg.inv (LAPACK only checks for exact-zero pivots): it propagates
    z, Pm, K = eng.predict([0.1, 0.2, 0.3], 1e7, [1.0, 0, 0, 0], np.full((4, 4), np.nan), np.eye(3), np.eye(4) * 0.1)
    assert np.isnan(K).all() and np.isfinite(z).all()


@pytest.mark.gpu
def test_fused_empty_launches_are_noops(eng):
    from poseestimationkf_amd._lib import lib
    f = eng.BatchedEKF(8)
    win = eng.IMUWindow(8, 4).synthesize()
    X0, P0 = f.get_state()
    f.run(win, n_steps=0)
    X1, P1 = f.get_state()
    assert np.array_equal(X0, X1) and np.array_equal(P0, P1)
    assert lib.pekf_run_dev(0, 10, 4, 0, None, None, None, None, None, None, 1.0, 0.1, None, None, 0, None) == 0
