"""Synthetic IMU streams: host (NumPy) mirror of the device generator ``pekf_synth_dev``.

The reference's input trace (``Sensor_CSV/KalmanFilter.txt``, read at
Python Kalman Filter/ReadFile.py:24) was never committed, so every workload here
is synthetic (SURVEY.md §8d "Synthetic inputs").  Each filter ``b`` owns a
Philox4x32-10 stream keyed by ``(seed, b)`` with counter ``(step, slot, 0, 0)``,
and every floating-point operation below is a single IEEE-754 correctly rounded
op (+ - * / sqrt, no fused multiply-add), so this host mirror and the HIP kernel
in ``csrc/pekf_synth.hip`` produce bit-identical streams.  Any shard can
therefore regenerate any subset of filters on the host to check the GPU result.

Per filter:
  * reference vectors acc0 = normalise([0,0,1] + n), mag0 = normalise([cos60°,0,-sin60°] + n)
    (the phone's initial calibration means, KFS/Parser.cpp:48-49), rounded to f32;
  * true body rate w is AR(1): w <- 0.98 w + N(0, 0.3²) rad/s; the true attitude q is
    advanced with the closed form of the RK4 step (body-frame rate, same convention as
    ExtendedKalmanFilter.py:27-30);
  * gyro = w + N(0, 0.02²); acc = normalise(R(q)^T acc0 + N(0,0.02²)); mag likewise;
  * dt_ns ~ U{4e6 .. 2e7} (variable in every config); optional Bernoulli(0.3)
    "magnetometer missing" flag (config 5) in bit 31 of the dt word.
Noise is the sum of 4 uniforms (Irwin-Hall), rescaled to the stated sigma.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

DEFAULT_SEED = 20261015

_MASK = np.uint64(0xFFFFFFFF)
_PM0 = np.uint64(0xD2511F53)
_PM1 = np.uint64(0xCD9E8D57)
_PW0 = np.uint64(0x9E3779B9)
_PW1 = np.uint64(0xBB67AE85)

INIT_STEP = 0xFFFFFFFF        # counter word used for the per-filter reference vectors
DT_MIN_NS = 4_000_000
DT_SPAN_NS = 16_000_001       # dt_ns = DT_MIN_NS + x % DT_SPAN_NS  -> [4e6, 2e7]
MISS_THRESH = 5_033_165       # (x >> 8) < 0.3 * 2^24
MISSING_BIT = 0x80000000
DT_MASK = 0x7FFFFFFF
DT_ESCAPE = 0x7FFFFFFF        # dt field of all ones: the record's dt is in the float64 side plane (dtx)

SQRT3 = 1.7320508075688772    # correctly rounded sqrt(3)
SIN60 = 0.8660254037844386    # correctly rounded sqrt(3)/2


@dataclass(frozen=True)
class SynthParams:
    """Noise levels and dynamics; the scales are passed verbatim to the device kernel."""
    sigma_ref: float = 0.05
    sigma_w: float = 0.3
    sigma_gyro: float = 0.02
    sigma_acc: float = 0.02
    sigma_mag: float = 0.02
    ar_w: float = 0.98

    def scales(self):
        """Irwin-Hall(4) has variance 1/3: scale = sqrt(3) * sigma (one rounding each)."""
        return (SQRT3 * self.sigma_ref, SQRT3 * self.sigma_w, SQRT3 * self.sigma_gyro,
                SQRT3 * self.sigma_acc, SQRT3 * self.sigma_mag)


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al., SC'11), vectorised; all inputs uint32-valued arrays."""
    c0, c1, c2, c3, k0, k1 = (np.asarray(v, dtype=np.uint64) & _MASK for v in (c0, c1, c2, c3, k0, k1))
    for rnd in range(10):
        if rnd:
            k0 = (k0 + _PW0) & _MASK
            k1 = (k1 + _PW1) & _MASK
        p0 = _PM0 * c0
        p1 = _PM1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & _MASK,
                          (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & _MASK)
    return c0, c1, c2, c3


def _noise(words, scale):
    u = [(w >> np.uint64(8)).astype(np.float64) * (2.0 ** -24) for w in words]
    return ((((u[0] + u[1]) + u[2]) + u[3]) - 2.0) * scale


def _normalise3(x, y, z):
    n = np.sqrt((x * x + y * y) + z * z)
    return x / n, y / n, z / n


def reference_vectors(ids, seed=DEFAULT_SEED, params=SynthParams()):
    """Per-filter (acc0, mag0) as float64 arrays of shape (K,3) holding f32-representable values."""
    ids = np.asarray(ids, dtype=np.uint64)
    s_ref = params.scales()[0]
    n = [_noise(philox4x32(INIT_STEP, s, 0, 0, seed, ids), s_ref) for s in range(6)]
    a = _normalise3(0.0 + n[0], 0.0 + n[1], 1.0 + n[2])
    m = _normalise3(0.5 + n[3], 0.0 + n[4], -SIN60 + n[5])
    acc0 = np.stack([v.astype(np.float32) for v in a], axis=1).astype(np.float64)
    mag0 = np.stack([v.astype(np.float32) for v in m], axis=1).astype(np.float64)
    return acc0, mag0


def _body(q, v):
    """R(q)^T v for unit q = [w,x,y,z] mapping body -> world; columns of R dotted with v."""
    w, x, y, z = q
    r00 = 1.0 - 2.0 * (y * y + z * z)
    r01 = 2.0 * (x * y - w * z)
    r02 = 2.0 * (x * z + w * y)
    r10 = 2.0 * (x * y + w * z)
    r11 = 1.0 - 2.0 * (x * x + z * z)
    r12 = 2.0 * (y * z - w * x)
    r20 = 2.0 * (x * z - w * y)
    r21 = 2.0 * (y * z + w * x)
    r22 = 1.0 - 2.0 * (x * x + y * y)
    return ((r00 * v[0] + r10 * v[1]) + r20 * v[2],
            (r01 * v[0] + r11 * v[1]) + r21 * v[2],
            (r02 * v[0] + r12 * v[1]) + r22 * v[2])


def _measure(q, ref, words3, scale):
    b = _body(q, ref)
    a = [b[i] + _noise(words3[i], scale) for i in range(3)]
    a = _normalise3(*a)
    f = [v.astype(np.float32) for v in a]
    # keep |z| < 1 and z != 0 in f32 so the Wahba weights |z|, 1-|z| never vanish
    # (a vanishing weight makes B rank-1 and the reference's SVD rotation ill-defined)
    big = np.abs(f[2]) >= np.float32(1.0)
    f[2] = np.where(big, np.copysign(np.float32(0.99999994), f[2]), f[2])
    f[2] = np.where(f[2] == np.float32(0.0), np.float32(1e-30), f[2]).astype(np.float32)
    return f


@dataclass
class Records:
    """Per-filter record view of a window: arrays indexed [step, filter, ...]."""
    gyro: np.ndarray   # (W,K,3) float32
    acc: np.ndarray    # (W,K,3) float32
    mag: np.ndarray    # (W,K,3) float32
    dtw: np.ndarray    # (W,K)   uint32: dt_ns | MISSING_BIT
    acc0: np.ndarray   # (K,3)   float64
    mag0: np.ndarray   # (K,3)   float64
    dtx: np.ndarray = None  # (W,K) float64 dt side plane, or None: the dt of records whose dt field is DT_ESCAPE

    @property
    def dt_ns(self):
        """(W,K) float64 T - previousT of every record (the side plane's value for an escaped one)."""
        field = self.dtw & DT_MASK
        dt = field.astype(np.float64)
        if self.dtx is not None:
            dt = np.where(field == DT_ESCAPE, self.dtx, dt)
        return dt

    @property
    def missing(self):
        return (self.dtw & MISSING_BIT) != 0

    def filter(self, k):
        """(gyro, dt_ns, acc, mag) float64 arrays of filter column k, for the oracle."""
        return (self.gyro[:, k].astype(np.float64), self.dt_ns[:, k],
                self.acc[:, k].astype(np.float64), self.mag[:, k].astype(np.float64))


def generate(ids, window, seed=DEFAULT_SEED, missing=False, params=SynthParams()):
    """Generate `window` steps for the filters `ids` (host mirror of pekf_synth_dev)."""
    ids = np.asarray(ids, dtype=np.uint64)
    K = ids.shape[0]
    acc0, mag0 = reference_vectors(ids, seed, params)
    _, s_w, s_g, s_a, s_m = params.scales()
    w = [np.zeros(K) for _ in range(3)]
    q = [np.ones(K), np.zeros(K), np.zeros(K), np.zeros(K)]
    gyro = np.empty((window, K, 3), np.float32)
    acc = np.empty((window, K, 3), np.float32)
    mag = np.empty((window, K, 3), np.float32)
    dtw = np.empty((window, K), np.uint32)
    a_ref = [acc0[:, i] for i in range(3)]
    m_ref = [mag0[:, i] for i in range(3)]
    for t in range(window):
        ph = lambda slot: philox4x32(t, slot, 0, 0, seed, ids)  # noqa: E731
        s0 = ph(0)
        dt = np.uint64(DT_MIN_NS) + s0[0] % np.uint64(DT_SPAN_NS)
        word = dt.astype(np.uint32)
        if missing:
            flag = (s0[1] >> np.uint64(8)) < np.uint64(MISS_THRESH)
            word = np.where(flag, word | np.uint32(MISSING_BIT), word).astype(np.uint32)
        dtw[t] = word
        for i in range(3):
            w[i] = params.ar_w * w[i] + _noise(ph(1 + i), s_w)
        h = dt.astype(np.float64) * 1e-9
        th2 = 0.25 * ((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2])
        x = (h * h) * th2
        ca = (1.0 - x * 0.5) + (x * x) / 24.0
        cb = h * (1.0 - x / 6.0)
        r0 = 0.5 * ((-(w[0] * q[1]) - w[1] * q[2]) - w[2] * q[3])
        r1 = 0.5 * ((w[0] * q[0] + w[2] * q[2]) - w[1] * q[3])
        r2 = 0.5 * ((w[1] * q[0] - w[2] * q[1]) + w[0] * q[3])
        r3 = 0.5 * ((w[2] * q[0] + w[1] * q[1]) - w[0] * q[2])
        q = [ca * q[0] + cb * r0, ca * q[1] + cb * r1, ca * q[2] + cb * r2, ca * q[3] + cb * r3]
        n = np.sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3])
        q = [c / n for c in q]
        for i in range(3):
            gyro[t, :, i] = (w[i] + _noise(ph(4 + i), s_g)).astype(np.float32)
        a = _measure(q, a_ref, [ph(7), ph(8), ph(9)], s_a)
        m = _measure(q, m_ref, [ph(10), ph(11), ph(12)], s_m)
        for i in range(3):
            acc[t, :, i] = a[i]
            mag[t, :, i] = m[i]
    return Records(gyro, acc, mag, dtw, acc0, mag0)


# ---------------------------------------------------------------------------------------------
# HBM stream layout (see DESIGN.md "Data layout"): three planes per step, filter-minor.
#   plane GD : float4 {gx, gy, gz, bits(dt word)}   [window][batch]
#   plane AM : float4 {ax, ay, az, mx}              [window][batch]
#   plane MY : float2 {my, mz}                      [window][batch]
# 40 B per filter-step; a wavefront reads 1 KiB + 1 KiB + 512 B per step, fully coalesced.
# ---------------------------------------------------------------------------------------------

def pack_planes(rec: Records):
    """Records -> (gd (W,K,4) f32, am (W,K,4) f32, my (W,K,2) f32) contiguous planes."""
    W, K = rec.dtw.shape
    gd = np.empty((W, K, 4), np.float32)
    gd[..., :3] = rec.gyro
    gd[..., 3] = rec.dtw.view(np.float32)
    am = np.empty((W, K, 4), np.float32)
    am[..., :3] = rec.acc
    am[..., 3] = rec.mag[..., 0]
    my = np.ascontiguousarray(rec.mag[..., 1:3])
    return gd, am, my


def unpack_planes(gd, am, my, acc0, mag0, dtx=None):
    """Inverse of pack_planes (used to pull sampled filters back off the device)."""
    gyro = np.ascontiguousarray(gd[..., :3])
    dtw = np.ascontiguousarray(gd[..., 3]).view(np.uint32)
    acc = np.ascontiguousarray(am[..., :3])
    mag = np.concatenate([am[..., 3:4], my], axis=-1)
    return Records(gyro, acc, mag, dtw, np.asarray(acc0, np.float64), np.asarray(mag0, np.float64),
                   None if dtx is None else np.asarray(dtx, np.float64))


def refs_array(acc0, mag0):
    """Per-filter constants block for the fused kernel: (K,6) float64 [acc0 xyz, mag0 xyz]."""
    return np.ascontiguousarray(np.concatenate([acc0, mag0], axis=1), dtype=np.float64)


# ---------------------------------------------------------------------------------------------
# Raw phone events for the server front-end: what the Android client sends in
# phase 3 (ASC/SensorActivities.java:50-88, wire format ASC/MessageSender.java:217-233) --
# asynchronous accelerometer (m/s^2), gyroscope (rad/s) and magnetometer (uT) samples with
# integer ns timestamps.  Event planes: EV float4 {x, y, z, bits(type)} and ET int64 [E][K].
# ---------------------------------------------------------------------------------------------
EV_ACC, EV_GYRO, EV_MAG = 0, 1, 2
G_MS2, B_UT = 9.81, 45.0
T_INIT_NS = 1_000_000_000_000


def generate_events(ids, n_events, seed=DEFAULT_SEED, params=SynthParams()):
    """Per filter: n_events events, type ~ {acc 0.4, gyro 0.4, mag 0.2}, gaps U{1..4} ms.

    Returns dict(types (E,K) uint32, values (E,K,3) float32, times (E,K) int64,
    init_acc / init_mag (K,3) float64 = raw phase-2 means, t_init (K,) int64)."""
    ids = np.asarray(ids, dtype=np.uint64)
    K = ids.shape[0]
    acc0, mag0 = reference_vectors(ids, seed, params)
    _, s_w, s_g, s_a, s_m = params.scales()
    w = [np.zeros(K) for _ in range(3)]
    q = [np.ones(K), np.zeros(K), np.zeros(K), np.zeros(K)]
    types = np.empty((n_events, K), np.uint32)
    vals = np.empty((n_events, K, 3), np.float32)
    times = np.empty((n_events, K), np.int64)
    t = np.full(K, T_INIT_NS, np.int64)
    key = np.uint64(seed) ^ np.uint64(0x5EED)
    for e in range(n_events):
        ph = lambda slot: philox4x32(e, slot, 1, 0, key, ids)  # noqa: E731  (c2 = 1: event streams)
        s0 = ph(0)
        u = (s0[0] >> np.uint64(8)).astype(np.float64) * (2.0 ** -24)
        ty = np.where(u < 0.4, EV_ACC, np.where(u < 0.8, EV_GYRO, EV_MAG)).astype(np.uint32)
        gap = 1_000_000 + (s0[1] % np.uint64(3_000_001)).astype(np.int64)
        t = t + gap
        for i in range(3):
            w[i] = 0.995 * w[i] + _noise(ph(1 + i), 0.5 * s_w)
        h = gap.astype(np.float64) * 1e-9
        th2 = 0.25 * ((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2])
        x = (h * h) * th2
        ca = (1.0 - x * 0.5) + (x * x) / 24.0
        cb = h * (1.0 - x / 6.0)
        r = [0.5 * ((-(w[0] * q[1]) - w[1] * q[2]) - w[2] * q[3]),
             0.5 * ((w[0] * q[0] + w[2] * q[2]) - w[1] * q[3]),
             0.5 * ((w[1] * q[0] - w[2] * q[1]) + w[0] * q[3]),
             0.5 * ((w[2] * q[0] + w[1] * q[1]) - w[0] * q[2])]
        q = [ca * q[i] + cb * r[i] for i in range(4)]
        n = np.sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3])
        q = [c / n for c in q]
        ba = _body(q, [acc0[:, i] for i in range(3)])
        bm = _body(q, [mag0[:, i] for i in range(3)])
        for i in range(3):
            g_val = w[i] + _noise(ph(4 + i), s_g)
            a_val = G_MS2 * (ba[i] + _noise(ph(7 + i), s_a))
            m_val = B_UT * (bm[i] + _noise(ph(10 + i), s_m))
            vals[e, :, i] = np.where(ty == EV_ACC, a_val, np.where(ty == EV_GYRO, g_val, m_val)).astype(np.float32)
        types[e] = ty
        times[e] = t
    return dict(types=types, values=vals, times=times, init_acc=G_MS2 * acc0, init_mag=B_UT * mag0,
                t_init=np.full(K, T_INIT_NS, np.int64))


EV_DT_BITS = 30  # event word = (ns since the previous event << 2) | type
EV_TIME = 3      # a time event: word == 3, x / y = the float64 clock step (include/pekf.h PEKF_EV_TIME)
EV_OTHER = 3     # in an event dict: a message of no sensor type (the server parses it, no sensor takes it)
EV_NONE = 4      # in an event dict: no message at all (padding of a short stream), only its time


def pack_events(ev):
    """generate_events dict -> EV float4 plane (E',K,4) f32 {x, y, z, bits(word)}.

    16 B per event: the word carries the 2-bit type and the ns gap to the filter's previous
    event (the first one: to t_init).  A gap the 30-bit field cannot hold (a pause of 2^30 ns or
    more, or a clock that steps back) becomes a time event -- word 3, the gap as a float64 in the
    x / y bits -- followed by the event itself with gap 0; every filter's stream is then padded to
    the longest with zero-step time events (E' = E + the most time events any filter needs).
    Type EV_OTHER (3, a message no sensor takes: it still counts as a message in phase 2, as every
    message the server parses does, KFS/Parser.cpp:36-62) needs a nonzero gap field, since word 3 is
    the time event: at a gap of 0 (or one the field cannot hold) it goes after a time event of
    gap - 1 ns with a gap field of 1.  Type EV_NONE (4, no message) is packed as a time event of its
    gap: the clock moves, no message is seen."""
    E, K = ev["types"].shape
    types = np.asarray(ev["types"], np.uint64)
    if types.size and int(types.max()) > EV_NONE:
        raise ValueError("event types are 0 acc, 1 gyro, 2 mag, 3 a message of no sensor type, 4 no message")
    values = np.asarray(ev["values"], np.float32)
    times = np.asarray(ev["times"], np.int64)
    prev = np.concatenate([np.asarray(ev["t_init"], np.int64)[None, :], times[:-1]], axis=0)
    gap = times - prev
    none = types == EV_NONE
    long_gap = (gap < 0) | (gap >= (1 << EV_DT_BITS))
    other0 = (types == EV_OTHER) & (long_gap | (gap == 0))
    insert = (long_gap | other0) & ~none             # a time event goes before the event
    gap_field = np.where(insert, other0.astype(np.int64), gap) if insert.any() else gap
    word = ((gap_field.astype(np.uint64) << np.uint64(2)) | types).astype(np.uint32)
    vals = values
    if none.any():  # an EV_NONE entry is itself a time event: x / y the float64 step
        word[none] = EV_TIME
        vals = values.copy()
        vals[none, :2] = gap[none].astype(np.float64).view(np.uint32).reshape(-1, 2).view(np.float32)
        vals[none, 2] = 0.0
    if not insert.any():
        planes = np.empty((E, K, 4), np.float32)
        planes[..., :3] = vals
        planes[..., 3] = word.view(np.float32)
        return planes
    shift = np.cumsum(insert, axis=0)              # time events inserted up to and including event e
    planes = np.zeros((E + int(shift[-1].max()), K, 4), np.float32)
    planes[..., 3] = np.uint32(EV_TIME).reshape(1).view(np.float32)[0]   # padding: zero-step time events
    cols = np.broadcast_to(np.arange(K), (E, K))
    row = np.arange(E)[:, None] + shift            # each event's row in the packed stream
    planes[row, cols, :3] = vals
    planes[row, cols, 3] = word.view(np.float32)
    e, k = np.nonzero(insert)
    step = (gap[e, k] - gap_field[e, k]).astype(np.float64).view(np.uint32).reshape(-1, 2)   # float64 halves
    planes[row[e, k] - 1, k, 0] = step[:, 0].view(np.float32)
    planes[row[e, k] - 1, k, 1] = step[:, 1].view(np.float32)
    return planes


EV64_T_LIMIT = 1 << 51  # FP64 events: |t| < 2^51 ns keeps the two lowest mantissa bits of t free for the type
EV64_NONE_W = 0x8000000000000003  # FP64 events: w of "no message" (the bits of -0.0 with type 3; include/pekf.h)


def pack_events64(ev, values=None):
    """generate_events-style dict -> the FP64 event plane (E, K, 4) float64 {x, y, z, w}
    (PEKF_EV_F64_EVENTS, include/pekf.h): x, y, z the sample as float64 -- `values` if given, else
    ev["values64"] if present (e.g. wire.parse's doubles), else ev["values"] widened -- and w's bits
    those of the event's absolute time in ns as a float64 with the type in its two lowest bits.  32 B
    per event; times are absolute, so no time events are needed for any gap or clock step.  Type
    EV_OTHER (3) is a message of no sensor type at its time; EV_NONE (4, no message) packs as
    {0, 0, 0, EV64_NONE_W}."""
    types = np.asarray(ev["types"], np.uint64)
    times = np.asarray(ev["times"], np.int64)
    if values is None:
        values = ev["values64"] if "values64" in ev else ev["values"]
    values = np.asarray(values, np.float64)
    if types.size and int(types.max()) > EV_NONE:
        raise ValueError("event types are 0 acc, 1 gyro, 2 mag, 3 a message of no sensor type, 4 no message")
    none = types == EV_NONE
    if times.size and int(np.abs(np.where(none, 0, times)).max()) >= EV64_T_LIMIT:
        raise ValueError("FP64 events need |t| < 2^51 ns")
    E, K = types.shape
    planes = np.empty((E, K, 4), np.float64)
    planes[..., :3] = np.where(none[..., None], 0.0, values)
    w = times.astype(np.float64).view(np.uint64) | np.where(none, 0, types)
    planes[..., 3] = np.where(none, np.uint64(EV64_NONE_W), w).view(np.float64)
    return planes


def has_time_events(planes):
    """Whether an event plane holds time events (word == EV_TIME): the flag the phase-3 kernels need."""
    return bool((np.ascontiguousarray(planes[..., 3]).view(np.uint32) == EV_TIME).any())


def window_bytes(batch, window):
    return int(batch) * int(window) * 40


def c1_timestamps(dt_ns, t0_ns=1_234_567_890_123):
    """Absolute ns timestamps for the single-filter log (config 1): T0 then cumulative sums."""
    t = [float(t0_ns)]
    acc = t0_ns
    for d in np.asarray(dt_ns, dtype=np.int64):
        acc += int(d)
        t.append(float(acc))
    return t


__all__ = ["DEFAULT_SEED", "SynthParams", "Records", "philox4x32", "reference_vectors", "generate",
           "pack_planes", "unpack_planes", "refs_array", "window_bytes", "c1_timestamps",
           "MISSING_BIT", "DT_MASK", "DT_ESCAPE", "pack_events", "pack_events64", "has_time_events", "EV_TIME", "EV_OTHER", "EV_NONE", "EV64_NONE_W"]
