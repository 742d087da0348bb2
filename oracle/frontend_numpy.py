"""Restatement of the live server's pre-processing front-end -- TEST INFRASTRUCTURE ONLY.

PARITY PARTLY PINNED: the source is C++ (Kalman Filter Server/PoseEstimator/Parser.cpp,
KalmanFilter.cpp) that needs Eigen, conio.h and winsock, so it cannot be
built here and ships no fixtures; this file restates its phase-3 logic by reading the code.
The low-pass stage (`lpf_step`) is pinned bit for bit by the reference's own Python
`Test.py:20-35` (the same alpha = 0.1 recurrence from a zero state, run unchanged to produce
tests/golden/lpf_testpy.npz); the state machine, interpolation and normalisation are
unpinned.  Used only by tests/test_frontend.py as the checker of pekf_frontend_dev
(SURVEY.md §8f-2).

Per filter, events (type '0' acc, '1' gyro, '2' mag; 3 values; integer ns time) go through
Parser::WriteKalmanFilterMeasurement (Parser.cpp:148-219):
  * before a gyro sample: acc -> acc_0, mag -> mag_0; gyro -> gyro, gyro_is_set;
  * after it: acc -> acc_1 (set), mag -> mag_1 (set); a new gyro replaces the gyro and, if
    set, shifts acc_1 -> acc_0 and mag_1 -> mag_0, clearing both flags;
  * once acc_1 and mag_1 are both set: ExecuteKalmanFilter (Parser.cpp:229-257), then
    acc_0 <- acc_1, mag_0 <- mag_1 and all flags cleared.
ExecuteKalmanFilter linearly interpolates acc and mag to the gyro time (Parser.cpp:259-267),
normalises both (Parser.cpp:221-228), low-pass filters them into Mag_1 / Acc_1 with
alpha = 0.1 from a zero state (KalmanFilter.cpp:16-18,21-24,279-303) and runs the filter step
with dt = time_gyro - previousT (KalmanFilter.cpp:306-308).  The record it produces is
exactly what the server logs (gyro, T, Mag_1, Acc_1) and what the offline filter consumes.
Before phase 3, acc_0 / mag_0 hold the phase-2 means at the initialisation time
(Parser.cpp:44-53), which is also previousT (KalmanFilter.cpp:9-14).
"""
from __future__ import annotations

import numpy as np

ACC, GYRO, MAG = 0, 1, 2
OTHER, NONE = 3, 4  # a message no sensor takes; no message at all (padding)


def _interp(t1, t2, t3, y1, y2):
    """Parser::LinearInterpolationSensor (Parser.cpp:259-267)."""
    with np.errstate(divide="ignore", invalid="ignore"):  # C++ double: x / 0 is inf / nan, not an error
        return [np.float64(y2[i] - y1[i]) / np.float64(float(t2) - float(t1)) * (float(t3) - float(t1)) + y1[i]
                for i in range(3)]


def lpf_step(prev, x, alpha):
    """alpha * x + (1 - alpha) * prev per component (KalmanFilter.cpp:285,298; Test.py:29-35)."""
    return [alpha * x[i] + (1 - alpha) * prev[i] for i in range(3)]


def lpf(samples, alpha=0.1):
    """The low-pass over a sample sequence from a zero state: (n, 3) -> (n, 3)."""
    out, prev = [], [0.0, 0.0, 0.0]
    for x in np.asarray(samples, np.float64):
        prev = lpf_step(prev, x, alpha)
        out.append(prev)
    return np.array(out)


def _normalise(v):
    """Parser::NormalizeValues (Parser.cpp:221-228)."""
    d = np.sqrt(np.float64((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]))
    with np.errstate(divide="ignore", invalid="ignore"):
        return [v[0] / d, v[1] / d, v[2] / d]


def run_frontend(types, values, times, init_acc, init_mag, t_init, alpha=0.1):
    """One filter's phase-3 events -> records.

    types (E,) int, values (E,3) float64, times (E,) int64 ns; init_acc / init_mag: phase-2
    means (raw), t_init: initialisation time.  Returns (gyro (R,3), dt_ns (R,), acc (R,3),
    mag (R,3)) as float64 -- the values the server logs as gyro / T / Acc_1 / Mag_1.
    """
    acc0, t_acc0 = list(map(float, init_acc)), int(t_init)
    mag0, t_mag0 = list(map(float, init_mag)), int(t_init)
    acc1 = mag1 = gyro = None
    t_acc1 = t_mag1 = t_gyro = 0
    gyro_set = acc1_set = mag1_set = False
    lpf_acc = [0.0, 0.0, 0.0]
    lpf_mag = [0.0, 0.0, 0.0]
    prev_t = int(t_init)
    out_g, out_dt, out_a, out_m = [], [], [], []
    for k in range(len(types)):
        ty, v, t = int(types[k]), [float(x) for x in values[k]], int(times[k])
        if not gyro_set:
            if ty == ACC:
                acc0, t_acc0 = v, t
            elif ty == MAG:
                mag0, t_mag0 = v, t
            elif ty == GYRO:
                gyro, t_gyro = v, t
                gyro_set = True
        else:
            if ty == ACC:
                acc1, t_acc1, acc1_set = v, t, True
            elif ty == MAG:
                mag1, t_mag1, mag1_set = v, t, True
            elif ty == GYRO:
                gyro, t_gyro = v, t
                if acc1_set:
                    acc0, t_acc0 = acc1, t_acc1
                if mag1_set:
                    mag0, t_mag0 = mag1, t_mag1
                acc1_set = mag1_set = False
        if acc1_set and mag1_set:
            gyro_set = acc1_set = mag1_set = False
            a = _normalise(_interp(t_acc0, t_acc1, t_gyro, acc0, acc1))
            m = _normalise(_interp(t_mag0, t_mag1, t_gyro, mag0, mag1))
            lpf_mag = lpf_step(lpf_mag, m, alpha)
            lpf_acc = lpf_step(lpf_acc, a, alpha)
            out_g.append(gyro)
            out_dt.append(t_gyro - prev_t)
            out_a.append(lpf_acc)
            out_m.append(lpf_mag)
            prev_t = t_gyro
            acc0, t_acc0 = acc1, t_acc1
            mag0, t_mag0 = mag1, t_mag1
    return (np.asarray(out_g, np.float64).reshape(-1, 3), np.asarray(out_dt, np.int64),
            np.asarray(out_a, np.float64).reshape(-1, 3), np.asarray(out_m, np.float64).reshape(-1, 3))


def initial_values(types, values, times, n_avg=100):
    """One filter's phase-2 events -> dict(ready, acc, mag, gyro (means), var_acc, var_mag, var_gyro, t_init).

    Parser::ProcessString phase '2' (Parser.cpp:36-58): while any sensor is not initialised, the
    event goes to initialMeanAndCovariance (:84-140) -- the first n_avg samples of its type are
    averaged (InitialValues::setValuesforAverage: a sequential float64 sum; compute_mean_and_variance:
    sum / n, then sum((x - mean)^2) / (n - 1), InitialValues.cpp:20-66) and the sensor counts as
    initialised at its next sample; the first event after all three are initialised builds the
    KalmanFilter at its time, and every later one moves acc_0 / mag_0's time and previousT to its
    own (:41-62).  PARITY UNPINNED (C++ source that cannot be built here, no fixtures).
    Every message counts, whatever its type (a Type char no sensor matches, here 3, adds no sample but
    builds the filter or moves its time once all three are initialised); type NONE (4) is no message
    (stream padding) and is skipped."""
    keys = (ACC, GYRO, MAG)
    sums = {k: [0.0, 0.0, 0.0] for k in keys}
    samples = {k: [] for k in keys}
    done = {k: False for k in keys}
    kalman, t_last = False, None
    for ty, v, t in zip(types, values, times):
        ty, t = int(ty), int(t)
        if ty == NONE:
            continue
        if not all(done.values()):
            if ty in sums:
                if len(samples[ty]) < n_avg:
                    x = [float(c) for c in v]
                    samples[ty].append(x)
                    for j in range(3):
                        sums[ty][j] += x[j]
                else:
                    done[ty] = True
        else:
            kalman, t_last = True, t
    out = dict(ready=kalman, t_init=t_last)
    for k, name in ((ACC, "acc"), (MAG, "mag"), (GYRO, "gyro")):
        if not kalman:
            out[name] = out["var_" + name] = [float("nan")] * 3
            continue
        mean = [sums[k][j] / n_avg for j in range(3)]
        var = [0.0, 0.0, 0.0]
        for x in samples[k]:
            for j in range(3):
                var[j] += (x[j] - mean[j]) * (x[j] - mean[j])
        out[name] = mean
        out["var_" + name] = [var[j] / (n_avg - 1) for j in range(3)]
    return out
