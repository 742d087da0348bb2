"""Drop-in for the reference module ``ExtendedKalmanFilter`` (Python Kalman Filter/ExtendedKalmanFilter.py).

``KalmanFilter`` keeps the reference's constructor, attributes (previousT, wahba, Q, R,
eps), methods and return tuples, so ``main_file.py`` runs unchanged against it.  X, P, z
and K are caller-owned values: every call returns fresh arrays and never mutates its
inputs (main_file.py:39-44 keeps the returned X in a list).  The arithmetic runs in the
per-call gfx950 kernels of libpekf.so (k_predict, k_correct, k_rk4, ...); the two per-record
methods go through the CPython binding ``_fastcall`` (same C entry points, less call overhead).  For many
filters at once use ``poseestimationkf_amd.engine.BatchedEKF`` (the fused kernel).
``predict`` / ``update`` are aliases of ``Prediction`` / ``Correction`` (the north_star's names).

Per-record calls are answered by a resident kernel that polls pinned host memory and leaves 5 ms
after the last call; a device-wide synchronisation elsewhere in the process may wait for it.  To
launch one kernel per call instead (identical results): ``PEKF_PERCALL=launch`` in the environment,
or ``percall_mode(PERCALL_LAUNCH)`` from this module.
"""
import numpy as np
from _bootstrap import engine as _eng
from _bootstrap import fastcall as _fc
from Wahba import Wahba

# the per-call service switch (include/pekf.h: pekf_set_percall_mode), re-exported for the drop-in's users
percall_mode = _eng.percall_mode
PERCALL_SERVICE, PERCALL_LAUNCH = _eng.PERCALL_SERVICE, _eng.PERCALL_LAUNCH


class KalmanFilter:
    def __init__(self, T0, mag_0, acc_0, eps):          # ExtendedKalmanFilter.py:6-11
        self.previousT = T0
        self.wahba = Wahba(acc_0, mag_0)
        self.Q = np.identity(3)
        self.R = np.identity(4)
        self.eps = eps

    def setQ(self, q):                                   # :12-13
        self.Q *= q

    def setR(self, r):                                   # :14-15
        self.R *= r

    def Comparator(self, q1, q2):                        # :16-23
        return _eng.comparator(q1, q2)[0]

    @staticmethod
    def RungeKutta4(q_0, T, w):                          # :25-41 (T in ns)
        return _eng.rk4(q_0, T, w)[0]

    def GetJacobian_A(self, w):                          # :43-48
        return _eng.jacobian_a(w)[0]

    def GetJacobian_B(self, q):                          # :51-56
        return _eng.jacobian_b(q)[0]

    def Prediction(self, Gyro, T, X_k, P_k):             # :58-68
        dt = T - self.previousT                          # same float64 op as :62
        z, P, K = _fc.predict(Gyro, dt, X_k, P_k, self.Q, self.R)    # LinAlgError if S singular
        self.previousT = T                               # :67, only after a successful step
        return z, P, K

    def Correction(self, Mag, Acc, z_k, P_k, K_k):       # :70-80
        return _fc.correct(Mag, Acc, z_k, P_k, K_k, self.wahba.w_initial_acc, self.wahba.w_initial_mag)

    # the north_star's call surface (BASELINE.json): predict()/update() are the same methods as the
    # reference's Prediction (:58) / Correction (:70) -- aliases, not wrappers, so they are the same code
    predict = Prediction
    update = Correction
