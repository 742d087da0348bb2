"""ctypes bindings to oracle/build/libekf_oracle.so -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
as the checker.  See ekf_oracle.c for the reference lines each entry restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libekf_oracle.so")

_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_up = ctypes.POINTER(ctypes.c_uint32)
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_rk4.argtypes = [_dp, ctypes.c_double, _dp, _dp]
        L.oracle_jacobian_a.argtypes = [_dp, _dp]
        L.oracle_jacobian_b.argtypes = [_dp, _dp]
        L.oracle_norm4.argtypes = [_dp]
        L.oracle_norm4.restype = ctypes.c_double
        L.oracle_inv4.argtypes = [_dp, _dp]
        L.oracle_predict.argtypes = [_dp, ctypes.c_double, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.oracle_correct.argtypes = [_dp] * 9
        L.oracle_wahba_rotation.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_double, ctypes.c_double, _dp]
        L.oracle_wahba_quat.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_double, ctypes.c_double, _dp]
        L.oracle_rotm_to_quat.argtypes = [_dp, _dp]
        L.oracle_run.argtypes = [ctypes.c_int64] * 4 + [_fp, _up, _dp, _dp, _dp, ctypes.c_double,
                                                         ctypes.c_double, _dp, _dp, _dp]
        _lib = L
    return _lib


def _d(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if n is not None:
        assert a.size == n, (a.shape, n)
    return a


def _p(a):
    return a.ctypes.data_as(_dp)


def rk4(q0, dt_ns, w):
    out = np.empty(4)
    lib().oracle_rk4(_p(_d(q0, 4)), float(dt_ns), _p(_d(w, 3)), _p(out))
    return out


def jacobian_a(w):
    out = np.empty((4, 4))
    lib().oracle_jacobian_a(_p(_d(w, 3)), _p(out))
    return out


def jacobian_b(q):
    out = np.empty((4, 3))
    lib().oracle_jacobian_b(_p(_d(q, 4)), _p(out))
    return out


def predict(gyro, dt_ns, X, P, Q, R):
    z, Pm, K = np.empty(4), np.empty((4, 4)), np.empty((4, 4))
    st = lib().oracle_predict(_p(_d(gyro, 3)), float(dt_ns), _p(_d(X, 4)), _p(_d(P, 16)),
                              _p(_d(Q, 9)), _p(_d(R, 16)), _p(z), _p(Pm), _p(K))
    if st:
        raise np.linalg.LinAlgError("Singular matrix")
    return z, Pm, K


def correct(mag, acc, z, P, K, acc0, mag0):
    X, Po = np.empty(4), np.empty((4, 4))
    lib().oracle_correct(_p(_d(mag, 3)), _p(_d(acc, 3)), _p(_d(z, 4)), _p(_d(P, 16)), _p(_d(K, 16)),
                         _p(_d(acc0, 3)), _p(_d(mag0, 3)), _p(X), _p(Po))
    return X, Po


def wahba_rotation(acc0, mag0, acc, mag, k_acc, k_mag):
    R = np.empty((3, 3))
    lib().oracle_wahba_rotation(_p(_d(acc0, 3)), _p(_d(mag0, 3)), _p(_d(acc, 3)), _p(_d(mag, 3)),
                                float(k_acc), float(k_mag), _p(R))
    return R


def wahba_quat(acc0, mag0, acc, mag, k_acc, k_mag):
    q = np.empty(4)
    lib().oracle_wahba_quat(_p(_d(acc0, 3)), _p(_d(mag0, 3)), _p(_d(acc, 3)), _p(_d(mag, 3)),
                            float(k_acc), float(k_mag), _p(q))
    return q


def rotm_to_quat(M):
    q = np.empty(4)
    lib().oracle_rotm_to_quat(_p(_d(M, 9)), _p(q))
    return q


def run(records, n_steps=None, step0=0, q=1.0, r=0.1, X=None, P=None, want_traj=False):
    """Run every filter of a synth.Records window through the oracle.

    Returns (X (K,4), P (K,4,4), traj (K,n_steps,4) or None).  Step t reads record (step0+t) % W.
    """
    W, K = records.dtw.shape
    n_steps = W if n_steps is None else int(n_steps)
    rec = np.empty((K, W, 9), np.float32)
    rec[..., 0:3] = records.gyro.transpose(1, 0, 2)
    rec[..., 3:6] = records.acc.transpose(1, 0, 2)
    rec[..., 6:9] = records.mag.transpose(1, 0, 2)
    dtw = np.ascontiguousarray(records.dtw.T, dtype=np.uint32)
    dtx_rec = getattr(records, "dtx", None)
    dtx = None if dtx_rec is None else np.ascontiguousarray(np.asarray(dtx_rec, np.float64).T)
    Xs = np.tile(np.array([1.0, 0, 0, 0]), (K, 1)) if X is None else np.array(X, np.float64, copy=True)
    Ps = np.tile(np.eye(4), (K, 1, 1)) if P is None else np.array(P, np.float64, copy=True)
    traj = np.empty((K, n_steps, 4)) if want_traj else None
    acc0 = _d(records.acc0)
    mag0 = _d(records.mag0)
    st = lib().oracle_run(K, n_steps, W, step0, rec.ctypes.data_as(_fp), dtw.ctypes.data_as(_up),
                          _p(dtx) if dtx is not None else None,
                          _p(acc0), _p(mag0), float(q), float(r), _p(Xs), _p(Ps),
                          _p(traj) if want_traj else None)
    if st:
        raise np.linalg.LinAlgError("Singular matrix")
    return Xs, Ps, traj
