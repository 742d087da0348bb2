"""The live server's text log: emit and ingest.

Format (Kalman Filter Server/PoseEstimator/KalmanFilter.cpp): one tagged line per
``WriteTextFile`` call (:335-340), numbers via ``std::to_string`` (i.e. ``%f`` for
doubles, plain integers for the ``long long`` timestamps):

    mag_0 : x,y,z                       set_mag_0            :26-29
    acc_0 : x,y,z                       set_acc_0            :30-33
    q_gyro : 1.0, 0.0, 0.0, 0.0         compute_initial_params :58-67
    X_k : 1.0, 0.0, 0.0, 0.0
    Wahba_quart : 1.0, 0.0, 0.0, 0.0
  per step:
    gyro : x,y,z                        SetAngularVelocity   :265-277
    T : <previousT>                     (first step only)    :136-141
    T : <T>                                                  :150-151
    q_gyro : w,x,y,z                                         :152-153
    Mag_1 : x,y,z                       SetMagnetometerMeasurements :279-290
    Acc_1 : x,y,z                       SetAccelerometerMeasurements :292-303
    X_k : w,x,y,z                       Correction           :180-183
    Wahba_quart : w,x,y,z

``read_log`` parses by substring tag with exactly the precedence of the offline
reader (Python Kalman Filter/ReadFile.py:27-45): ``q_gyro`` is tested before ``gyro``
and any line containing a capital ``T`` that matched nothing earlier is a timestamp.
"""
from __future__ import annotations

import io
import os
from dataclasses import dataclass, field

import numpy as np

REFERENCE_LOG_PATH = "D:/GITProjects/Kalman Filtering Server/PoseEstimationKF/Sensor_CSV/KalmanFilter.txt"
LOG_PATH_ENV = "PEKF_LOG_PATH"


def _vec(v):
    return ",".join("%f" % float(x) for x in v)


def write_log(fh, timestamps, gyro, acc, mag, acc0, mag0, q_gyro=None, x_k=None, wahba=None):
    """Write a single-filter trace in the server's log format.

    timestamps: n+1 absolute ns values (T0 then one per step); gyro/acc/mag: (n,3);
    q_gyro / x_k / wahba: optional (n,4) side channels (written as zeros when absent).
    """
    n = len(gyro)
    assert len(timestamps) == n + 1
    zeros = np.zeros((n, 4))
    q_gyro = zeros if q_gyro is None else q_gyro
    x_k = zeros if x_k is None else x_k
    wahba = zeros if wahba is None else wahba
    out = fh if hasattr(fh, "write") else open(fh, "w")
    try:
        out.write("mag_0 : %s\n" % _vec(mag0))
        out.write("acc_0 : %s\n" % _vec(acc0))
        out.write("q_gyro : 1.0, 0.0, 0.0, 0.0\n")
        out.write("X_k : 1.0, 0.0, 0.0, 0.0\n")
        out.write("Wahba_quart : 1.0, 0.0, 0.0, 0.0\n")
        for i in range(n):
            out.write("gyro : %s\n" % _vec(gyro[i]))
            if i == 0:
                out.write("T : %d\n" % int(timestamps[0]))
            out.write("T : %d\n" % int(timestamps[i + 1]))
            out.write("q_gyro : %s\n" % _vec(q_gyro[i]))
            out.write("Mag_1 : %s\n" % _vec(mag[i]))
            out.write("Acc_1 : %s\n" % _vec(acc[i]))
            out.write("X_k : %s\n" % _vec(x_k[i]))
            out.write("Wahba_quart : %s\n" % _vec(wahba[i]))
    finally:
        if out is not fh:
            out.close()


def write_log_native(path, timestamps, gyro, acc, mag, acc0, mag0, q_gyro=None, x_k=None, wahba=None):
    """write_log through libpekf's pekf_log_write (the same bytes, C++ on the host, for long traces)."""
    from ._lib import check, lib

    def arr(a, shape, dtype=np.float64):
        return None if a is None else np.ascontiguousarray(np.asarray(a, dtype).reshape(shape))
    n = len(gyro)
    t = arr(timestamps, (n + 1,), np.int64)
    g, a, m = arr(gyro, (n, 3)), arr(acc, (n, 3)), arr(mag, (n, 3))
    a0, m0 = arr(acc0, (3,)), arr(mag0, (3,))
    sides = [arr(x, (n, 4)) for x in (q_gyro, x_k, wahba)]
    ptr = lambda x: None if x is None else x.ctypes.data  # noqa: E731
    check(lib.pekf_log_write(os.fsencode(path), n, ptr(t), ptr(g), ptr(a), ptr(m), ptr(a0), ptr(m0),
                             *[ptr(x) for x in sides]))


def _values(line):
    return [float(tok) for tok in line.split(":")[1].split(",")]


@dataclass
class LogData:
    """Same attribute names and list-of-lists shapes as the reference's ``getData``."""
    mag_0: list = field(default_factory=list)
    mag_1: list = field(default_factory=list)
    acc_0: list = field(default_factory=list)
    acc_1: list = field(default_factory=list)
    gyro: list = field(default_factory=list)
    timestamp: list = field(default_factory=list)
    quart_wahba: list = field(default_factory=list)
    quart_xk: list = field(default_factory=list)
    quart_gyro: list = field(default_factory=list)


def parse_lines(lines, into=None):
    d = LogData() if into is None else into
    for line in lines:
        if "mag_0" in line:
            d.mag_0 = _values(line)
        elif "acc_0" in line:
            d.acc_0 = _values(line)
        elif "Acc_1" in line:
            d.acc_1.append(_values(line))
        elif "Mag_1" in line:
            d.mag_1.append(_values(line))
        elif "q_gyro" in line:
            d.quart_gyro.append(_values(line))
        elif "gyro" in line:
            d.gyro.append(_values(line))
        elif "T" in line:
            d.timestamp.append(_values(line))
        elif "Wahba_quart" in line:
            d.quart_wahba.append(_values(line))
        elif "X_k" in line:
            d.quart_xk.append(_values(line))
    return d


def read_log(path=None, into=None):
    """Parse a log file; default path: $PEKF_LOG_PATH, else the reference's hard-coded path."""
    if path is None:
        path = os.environ.get(LOG_PATH_ENV, REFERENCE_LOG_PATH)
    if isinstance(path, io.TextIOBase):
        return parse_lines(path.readlines(), into)
    with open(path) as fh:
        return parse_lines(fh.readlines(), into)


def log_to_arrays(d: LogData):
    """LogData -> float64 arrays (gyro, dt_ns, acc, mag, acc0, mag0) for one filter.

    dt_ns follows the reference exactly: T[i] - previousT in float64 (ExtendedKalmanFilter.py:62),
    previousT starting at the first timestamp (main_file.py:19-20,25).
    """
    ts = [t[0] for t in d.timestamp]
    n = len(d.acc_1)
    dt = np.empty(n)
    prev = ts[0]
    for i in range(n):
        dt[i] = ts[i + 1] - prev
        prev = ts[i + 1]
    return (np.asarray(d.gyro[:n], np.float64), dt, np.asarray(d.acc_1, np.float64),
            np.asarray(d.mag_1, np.float64), np.asarray(d.acc_0, np.float64), np.asarray(d.mag_0, np.float64))
