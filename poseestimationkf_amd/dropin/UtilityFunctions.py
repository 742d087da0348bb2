"""Drop-in for the reference module ``UtilityFunctions`` (Python Kalman Filter/UtilityFunctions.py).

``norm`` (the hot-path helper, :16-21) runs on the device (k_norm).  ``Quart2RPY`` (:3-14)
and ``DimensionalSplit`` (:24-34) are the reference's display/plot helpers, off the hot
path; they are plain host code here as there.
"""
import math

import numpy as np
from _bootstrap import engine as _eng


def Quart2RPY(q):
    """Quaternion [w,x,y,z] -> roll, pitch, yaw in degrees (UtilityFunctions.py:3-14)."""
    w, x, y, z = (float(v) for v in q[:4])
    roll = math.atan2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y))
    pitch = math.asin(2 * (w * y - z * x))
    yaw = math.atan2(2 * (w * z + x * y), 1 - 2 * (y * y + z * z))
    return np.asarray([roll, pitch, yaw]) * 180.0 / np.pi


def norm(a):
    """Euclidean norm, sequential sum of squares (UtilityFunctions.py:16-21)."""
    return np.float64(_eng.norm(np.asarray(a, dtype=np.float64).reshape(1, -1))[0])


def DimensionalSplit(S):
    """Transpose a list of equal-length sequences into per-component lists (UtilityFunctions.py:24-34)."""
    return [[row[i] for row in S] for i in range(len(S[0]))]
