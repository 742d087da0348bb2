"""Diagnostic: where the drop-in n = 1 call time goes (Python conversion vs ctypes vs the C entry)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poseestimationkf_amd import engine  # noqa: E402
from poseestimationkf_amd._lib import lib  # noqa: E402


def med(fn, n=400):
    for _ in range(50):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


g, dt, X, P, Q, R = np.array([0.1, -0.2, 0.3]), np.array([1e7]), np.array([1.0, 0, 0, 0]), np.eye(4), np.eye(3), np.eye(4) * 0.1
z, Pm, K = np.empty(4), np.empty((4, 4)), np.empty((4, 4))
args = [a.ctypes.data for a in (g, dt, X, P, Q, R, z, Pm, K)]
print("ctypes pekf_predict (pre-built pointers): %.1f us" % med(lambda: lib.pekf_predict(1, *args)))
print("ctypes pekf_abi_version (no-op):          %.1f us" % med(lambda: lib.pekf_abi_version()))
print("engine.predict (lists in):                %.1f us" % med(lambda: engine.predict([0.1, -0.2, 0.3], 1e7, X, P, Q, R)))
print("engine.correct:                           %.1f us" % med(lambda: engine.correct([0.5, 0, -0.86], [0, 0.1, 0.99], X, P, P, [0, 0, 1.0], [0.5, 0, -0.86])))
