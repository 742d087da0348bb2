"""Drop-in for the reference module ``UtilityFunctions`` (Python Kalman Filter/UtilityFunctions.py).

``norm`` (the hot-path helper, :16-21) and ``Quart2RPY`` (:3-14) run on the device (k_norm,
k_rpy).  ``DimensionalSplit`` (:24-34) is the reference's list-transpose plot helper, plain
host code as there.
"""
import numpy as np
from _bootstrap import engine as _eng


def Quart2RPY(q):
    """Quaternion [w,x,y,z] -> roll, pitch, yaw in degrees (UtilityFunctions.py:3-14)."""
    return _eng.quat_to_rpy(np.asarray(q, dtype=np.float64)[:4])[0]


def norm(a):
    """Euclidean norm, sequential sum of squares (UtilityFunctions.py:16-21)."""
    return np.float64(_eng.norm(np.asarray(a, dtype=np.float64).reshape(1, -1))[0])


def DimensionalSplit(S):
    """Transpose a list of equal-length sequences into per-component lists (UtilityFunctions.py:24-34)."""
    return [[row[i] for row in S] for i in range(len(S[0]))]
