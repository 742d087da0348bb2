"""Host side of the batched engine: device buffers, resident IMU windows, fused runs.

Everything here is plumbing around the C ABI (include/pekf.h); all arithmetic of the
filter runs in the HIP kernels of libpekf.so.
"""
from __future__ import annotations

import ctypes
import os
import types

import numpy as np

from . import synth
from ._lib import (EV_F32_RECORDS, EV_F64_EVENTS, EV_TIME_EVENTS, RUN_MIXED_PRECISION, RUN_STATE_SOA, WIRE_FRAME_ROWS,
                   check, dptr, f64, lib)


# ------------------------------------------------------------------ device plumbing

class DeviceBuffer:
    """A raw hipMalloc allocation owned by Python."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        self._lib = lib   # freed by the library that allocated it
        p = ctypes.c_void_p()
        check(lib.pekf_malloc(ctypes.byref(p), max(1, self.nbytes)))
        self.ptr = p.value

    def upload(self, arr, stream=None):
        a = np.ascontiguousarray(arr)
        assert a.nbytes <= self.nbytes, (a.nbytes, self.nbytes)
        check(lib.pekf_memcpy_h2d(self.ptr, a.ctypes.data, a.nbytes, stream))
        return self

    def download(self, shape, dtype, stream=None, offset=0):
        out = np.empty(shape, dtype)
        assert offset + out.nbytes <= self.nbytes
        check(lib.pekf_memcpy_d2h(out.ctypes.data, self.ptr + offset, out.nbytes, stream))
        return out

    def free(self):
        if getattr(self, "ptr", None):
            self._lib.pekf_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self):
        self._lib = lib
        s = ctypes.c_void_p()
        check(lib.pekf_stream_create(ctypes.byref(s)))
        self.handle = s.value

    def sync(self):
        check(self._lib.pekf_stream_sync(self.handle))

    def __del__(self):
        try:
            if self.handle:
                self._lib.pekf_stream_destroy(self.handle)
        except Exception:
            pass


class Event:
    def __init__(self):
        self._lib = lib
        e = ctypes.c_void_p()
        check(lib.pekf_event_create(ctypes.byref(e)))
        self.handle = e.value

    def record(self, stream=None):
        check(lib.pekf_event_record(self.handle, stream))

    def sync(self):
        check(lib.pekf_event_sync(self.handle))

    def elapsed_ms(self, end):
        ms = ctypes.c_float()
        check(lib.pekf_event_elapsed_ms(ctypes.byref(ms), self.handle, end.handle))
        return ms.value

    def __del__(self):
        try:
            if self.handle:
                self._lib.pekf_event_destroy(self.handle)
        except Exception:
            pass


def set_device(dev):
    check(lib.pekf_set_device(int(dev)))


def device_name(dev=0):
    buf = ctypes.create_string_buffer(128)
    check(lib.pekf_device_name(int(dev), buf, 128))
    return buf.value.decode()


PERCALL_SERVICE, PERCALL_LAUNCH = 0, 1


def percall_mode(mode=None):
    """How n = 1 per-call operators reach the GPU (include/pekf.h): PERCALL_SERVICE (a resident
    kernel answering requests in pinned host memory, the default) or PERCALL_LAUNCH (one launch
    per call).  Sets the mode when given; returns the mode in effect."""
    if mode is not None:
        check(lib.pekf_set_percall_mode(int(mode)))
    m = ctypes.c_int()
    check(lib.pekf_get_percall_mode(ctypes.byref(m)))
    return m.value


# ------------------------------------------------------------------ recorded traces (host ingest)

def read_log_records(path):
    """Parse one server log natively (pekf_log_scan / pekf_log_read) into a 1-filter synth.Records.

    The records are the 40 B stream format: f32 sensor values, u32 ns dt (the drop-in
    ReadFile / logformat path keeps the parsed float64 values instead)."""
    bpath = os.fsencode(path)
    n = ctypes.c_int64()
    check(lib.pekf_log_scan(bpath, ctypes.byref(n)))
    n = n.value
    gyro, acc, mag = (np.empty((n, 1, 3), np.float32) for _ in range(3))
    dtw = np.empty((n, 1), np.uint32)
    dtx = np.empty((n, 1), np.float64)
    acc0, mag0, t0, n_esc = np.empty((1, 3)), np.empty((1, 3)), ctypes.c_double(), ctypes.c_int64()
    check(lib.pekf_log_read_ext(bpath, n, gyro.ctypes.data, acc.ctypes.data, mag.ctypes.data, dtw.ctypes.data,
                                dtx.ctypes.data, ctypes.byref(n_esc), dptr(acc0), dptr(mag0), ctypes.byref(t0)))
    # records whose T - previousT does not fit the dt word (a pause >= 2^31 ns, a negative or fractional
    # difference) carry it in the float64 side plane
    return synth.Records(gyro, acc, mag, dtw, acc0, mag0, dtx if n_esc.value else None)


# ------------------------------------------------------------------ resident IMU window

class IMUWindow:
    """`window` steps x `batch` filters of the 40 B/step input record, resident in HBM.

    Planes (filter-minor, see synth.pack_planes): gd float4, am float4, my float2, plus the
    per-filter reference block refs (batch, 6) float64.  Either uploaded from host records or
    generated on the device with the bit-identical Philox generator (pekf_synth_dev).
    """

    def __init__(self, batch, window):
        self.batch, self.window = int(batch), int(window)
        n = self.batch * self.window
        self.gd = DeviceBuffer(16 * n)
        self.am = DeviceBuffer(16 * n)
        self.my = DeviceBuffer(8 * n)
        self.refs = DeviceBuffer(48 * self.batch)
        self.counts = None  # per-filter valid record counts when filters are ragged (logs, front-end)
        self.dtx = None     # dt side plane [window][batch] float64 when some record's dt is escaped (pekf.h)

    @property
    def nbytes(self):
        return self.gd.nbytes + self.am.nbytes + self.my.nbytes

    @classmethod
    def from_records(cls, rec: synth.Records):
        W, K = rec.dtw.shape
        win = cls(K, W)
        gd, am, my = synth.pack_planes(rec)
        win.gd.upload(gd)
        win.am.upload(am)
        win.my.upload(my)
        win.refs.upload(synth.refs_array(rec.acc0, rec.mag0))
        if rec.dtx is not None:
            win.dtx = DeviceBuffer(8 * W * K).upload(np.ascontiguousarray(rec.dtx, np.float64))
        return win

    @classmethod
    def from_planes(cls, gd, am, my, acc0, mag0, dtx=None):
        W, K = gd.shape[:2]
        win = cls(K, W)
        win.gd.upload(np.ascontiguousarray(gd, np.float32))
        win.am.upload(np.ascontiguousarray(am, np.float32))
        win.my.upload(np.ascontiguousarray(my, np.float32))
        win.refs.upload(synth.refs_array(acc0, mag0))
        if dtx is not None:
            win.dtx = DeviceBuffer(8 * W * K).upload(np.ascontiguousarray(dtx, np.float64))
        return win

    @classmethod
    def from_logs(cls, paths, n_records=None):
        """One filter per server log, parsed natively (pekf_log_read).

        Logs may differ in length: the window holds the longest log's records (n_records caps
        it), shorter logs are zero-padded and win.counts[b] is filter b's own record count,
        which BatchedEKF.run applies so each filter consumes exactly its own records."""
        recs = [read_log_records(p) for p in paths]
        lens = np.array([r.dtw.shape[0] for r in recs], dtype=np.int64)
        n = int(lens.max()) if n_records is None else int(n_records)

        def cat(name):
            out = []
            for r in recs:
                a = getattr(r, name)
                m = min(n, a.shape[0])
                pad = np.zeros((n,) + a.shape[1:], a.dtype)
                pad[:m] = a[:m]
                out.append(pad)
            return np.concatenate(out, axis=1)
        escaped = any(r.dtx is not None for r in recs)
        dtx = None
        if escaped:  # logs without escapes get a zero side plane (never read: their words are not escapes)
            dtx = [r.dtx if r.dtx is not None else np.zeros(r.dtw.shape, np.float64) for r in recs]
            dtx = np.concatenate([np.pad(d[:n], ((0, n - min(n, d.shape[0])), (0, 0))) for d in dtx], axis=1)
        rec = synth.Records(cat("gyro"), cat("acc"), cat("mag"), cat("dtw"),
                            np.concatenate([r.acc0 for r in recs]), np.concatenate([r.mag0 for r in recs]), dtx)
        win = cls.from_records(rec)
        win.counts = np.minimum(lens, n).astype(np.int32)
        return win

    def synthesize(self, seed=synth.DEFAULT_SEED, first_filter=0, missing=False,
                   params=synth.SynthParams(), stream=None):
        sc = np.array(params.scales(), dtype=np.float64)
        check(lib.pekf_synth_dev(self.batch, self.window, int(first_filter), int(seed) & 0xFFFFFFFF,
                                 1 if missing else 0, dptr(sc), float(params.ar_w), self.gd.ptr,
                                 self.am.ptr, self.my.ptr, self.refs.ptr, stream))
        if stream is None:
            check(lib.pekf_device_sync())
        return self

    def wahba_quaternions(self, n_steps=None, step0=0, k_acc=0.5, k_mag=0.5):
        """Pure-Wahba attitude of every record with fixed weights (main_file.py:40): (n_steps, batch, 4)."""
        n_steps = self.window if n_steps is None else int(n_steps)
        out = DeviceBuffer(32 * n_steps * self.batch)
        check(lib.pekf_wahba_stream_dev(self.batch, n_steps, self.window, int(step0), self.am.ptr, self.my.ptr,
                                        self.refs.ptr, float(k_acc), float(k_mag), out.ptr, None))
        check(lib.pekf_device_sync())
        return out.download((n_steps, self.batch, 4), np.float64)

    def gyro_chain(self, q0=None, n_steps=None, step0=0, want_traj=False):
        """Pure-gyro attitude (RK4 of the gyro records alone, KFS/KalmanFilter.cpp:149) from q0 (default
        [1,0,0,0]); returns (q_final (batch,4), traj (n_steps,batch,4) or None)."""
        n_steps = self.window if n_steps is None else int(n_steps)
        q = np.tile([1.0, 0.0, 0.0, 0.0], (self.batch, 1)) if q0 is None else f64(q0, (self.batch, 4))
        qb = DeviceBuffer(32 * self.batch).upload(q)
        tb = DeviceBuffer(32 * n_steps * self.batch) if want_traj else None
        # escaped records (a dt the word cannot hold) take their dt from the window's side plane, as in the filter
        check(lib.pekf_gyro_chain_ext_dev(self.batch, n_steps, self.window, int(step0), self.gd.ptr,
                                          self.dtx.ptr if self.dtx is not None else None, qb.ptr,
                                          tb.ptr if tb is not None else None, None))
        check(lib.pekf_device_sync())
        return (qb.download((self.batch, 4), np.float64),
                tb.download((n_steps, self.batch, 4), np.float64) if want_traj else None)

    def download_filters(self, cols):
        """Pull the records of filter columns `cols` back to the host as synth.Records."""
        cols = np.asarray(cols)
        gd = self.gd.download((self.window, self.batch, 4), np.float32)[:, cols]
        am = self.am.download((self.window, self.batch, 4), np.float32)[:, cols]
        my = self.my.download((self.window, self.batch, 2), np.float32)[:, cols]
        refs = self.refs.download((self.batch, 6), np.float64)[cols]
        dtx = None if self.dtx is None else self.dtx.download((self.window, self.batch), np.float64)[:, cols]
        return synth.unpack_planes(gd, am, my, refs[:, :3], refs[:, 3:], dtx)


class RecordWindow64:
    """`window` steps x `batch` filters of FP64 records (80 B per filter-record, pekf_run_rec64_dev), for
    inputs that are float64 to begin with: recorded logs, parsed into float64 as the reference parses
    them (ReadFile.py:14-21), where IMUWindow's 40 B record would round them to f32.

    Planes [window][batch]: gd double4 {gyro xyz, dt_ns}, am double4 {acc xyz, mag x}, my double2
    {mag yz}; dt is the float64 T - previousT itself (any pause, clock step or fraction).  Every record
    is a full record (no missing-magnetometer flag).  BatchedEKF.run / run_async take it like an
    IMUWindow (FP64 AoS state)."""

    def __init__(self, batch, window):
        self.batch, self.window = int(batch), int(window)
        n = self.batch * self.window
        self.gd = DeviceBuffer(32 * n)
        self.am = DeviceBuffer(32 * n)
        self.my = DeviceBuffer(16 * n)
        self.refs = DeviceBuffer(48 * self.batch)
        self.counts = None  # per-filter valid record counts when filters are ragged (logs)

    @property
    def nbytes(self):
        return self.gd.nbytes + self.am.nbytes + self.my.nbytes

    @classmethod
    def from_arrays(cls, gyro, dt_ns, acc, mag, acc0, mag0):
        """gyro / acc / mag (W, K, 3), dt_ns (W, K) float64 (the reference's T - previousT); acc0 / mag0
        (K, 3) the reference pairs (KalmanFilter(T0, mag_0, acc_0))."""
        gyro, acc, mag = (np.asarray(a, np.float64) for a in (gyro, acc, mag))
        W, K = gyro.shape[:2]
        dt = np.asarray(dt_ns, np.float64).reshape(W, K)
        win = cls(K, W)
        win.gd.upload(np.ascontiguousarray(np.concatenate([gyro, dt[..., None]], axis=2)))
        win.am.upload(np.ascontiguousarray(np.concatenate([acc, mag[..., :1]], axis=2)))
        win.my.upload(np.ascontiguousarray(mag[..., 1:]))
        win.refs.upload(synth.refs_array(np.asarray(acc0, np.float64).reshape(K, 3),
                                         np.asarray(mag0, np.float64).reshape(K, 3)))
        return win

    @classmethod
    def from_logs(cls, paths, n_records=None):
        """One filter per server log, parsed natively into float64 (pekf_log_read64); ragged logs as
        IMUWindow.from_logs (zero-padded, win.counts = each filter's own record count)."""
        cols = []
        for p in paths:
            bpath = os.fsencode(p)
            n = ctypes.c_int64()
            check(lib.pekf_log_scan(bpath, ctypes.byref(n)))
            g, a, m = (np.empty((n.value, 3)) for _ in range(3))
            dt = np.empty(n.value)
            a0, m0, t0 = np.empty(3), np.empty(3), ctypes.c_double()
            check(lib.pekf_log_read64(bpath, n.value, g.ctypes.data, a.ctypes.data, m.ctypes.data, dt.ctypes.data,
                                      dptr(a0), dptr(m0), ctypes.byref(t0)))
            cols.append((g, dt, a, m, a0, m0))
        lens = np.array([c[1].shape[0] for c in cols], np.int64)
        W = int(lens.max()) if n_records is None else int(n_records)

        def stack(i, shape):
            out = np.zeros((W, len(cols)) + shape)
            for k, c in enumerate(cols):
                m = min(W, c[i].shape[0])
                out[:m, k] = c[i][:m]
            return out
        win = cls.from_arrays(stack(0, (3,)), stack(1, ()), stack(2, (3,)), stack(3, (3,)),
                              np.stack([c[4] for c in cols]), np.stack([c[5] for c in cols]))
        win.counts = np.minimum(lens, W).astype(np.int32)
        return win

    def download_filters(self, cols):
        """The records of filter columns `cols` as float64 arrays: (gyro (W, n, 3), dt_ns (W, n), acc (W, n, 3),
        mag (W, n, 3), refs (n, 6))."""
        cols = np.asarray(cols)
        gd = self.gd.download((self.window, self.batch, 4), np.float64)[:, cols]
        am = self.am.download((self.window, self.batch, 4), np.float64)[:, cols]
        my = self.my.download((self.window, self.batch, 2), np.float64)[:, cols]
        refs = self.refs.download((self.batch, 6), np.float64)[cols]
        return gd[..., :3], gd[..., 3], am[..., :3], np.concatenate([am[..., 3:4], my], axis=-1), refs

    def wahba_quaternions(self, n_steps=None, step0=0, k_acc=0.5, k_mag=0.5):
        """Pure-Wahba attitude of every record with fixed weights (main_file.py:40): (n_steps, batch, 4)."""
        n_steps = self.window if n_steps is None else int(n_steps)
        out = DeviceBuffer(32 * n_steps * self.batch)
        check(lib.pekf_wahba_stream_rec64_dev(self.batch, n_steps, self.window, int(step0), self.am.ptr, self.my.ptr,
                                              self.refs.ptr, float(k_acc), float(k_mag), out.ptr, None))
        check(lib.pekf_device_sync())
        return out.download((n_steps, self.batch, 4), np.float64)

    def gyro_chain(self, q0=None, n_steps=None, step0=0, want_traj=False):
        """Pure-gyro attitude (RK4 of the gyro records alone, KFS/KalmanFilter.cpp:149) from q0 (default
        [1,0,0,0]); returns (q_final (batch,4), traj (n_steps,batch,4) or None)."""
        n_steps = self.window if n_steps is None else int(n_steps)
        q = np.tile([1.0, 0.0, 0.0, 0.0], (self.batch, 1)) if q0 is None else f64(q0, (self.batch, 4))
        qb = DeviceBuffer(32 * self.batch).upload(q)
        tb = DeviceBuffer(32 * n_steps * self.batch) if want_traj else None
        check(lib.pekf_gyro_chain_rec64_dev(self.batch, n_steps, self.window, int(step0), self.gd.ptr, qb.ptr,
                                            tb.ptr if tb is not None else None, None))
        check(lib.pekf_device_sync())
        return (qb.download((self.batch, 4), np.float64),
                tb.download((n_steps, self.batch, 4), np.float64) if want_traj else None)


# ------------------------------------------------------------------ server front-end (raw events)

EVENT_FORMS = ("f32", "f64")


def server_event_values(ev):
    """The sample values the server computes with: ev["values64"] when the events came as wire text
    (wire.events_from_wire: the server's own std::stod parse), else the doubles it would parse from
    the phone's Float.toString of ev["values"] (wire.server_values)."""
    from . import wire
    return np.asarray(ev["values64"], np.float64) if "values64" in ev else wire.server_values(ev["values"])


def _event_planes(ev, events="f32"):
    """(device event planes, n_events, flags).  events="f32": synth.pack_events (16 B, the float32
    samples; time events inserted for gaps the 30-bit field cannot hold), flags = PEKF_EV_TIME_EVENTS when
    the planes hold any.  events="f64": synth.pack_events64 of the server's values (32 B,
    server_event_values), flags = PEKF_EV_F64_EVENTS."""
    if events not in EVENT_FORMS:
        raise ValueError("events must be 'f32' or 'f64'")
    if events == "f64":
        planes = synth.pack_events64(ev, server_event_values(ev))
        return DeviceBuffer(planes.nbytes).upload(planes), planes.shape[0], EV_F64_EVENTS
    planes = synth.pack_events(ev)
    return (DeviceBuffer(planes.nbytes).upload(planes), planes.shape[0],
            EV_TIME_EVENTS if synth.has_time_events(planes) else 0)


def run_frontend(ev, alpha=0.1, r_max=None, events="f32"):
    """Raw phone events (synth.generate_events layout) -> (window of records, counts (K,) int32).

    Runs pekf_frontend_ext_dev.  Every record needs a gyro, an accelerometer and a
    magnetometer event, so r_max defaults to n_events // 3 + 1.  Raises if a filter overflows r_max.
    events="f32": float32 samples -> an IMUWindow of 40 B records; event gaps of any size go through
    time events, and records whose dt does not fit the dt word through the window's dt side plane
    (win.dtx, kept only if some record needed it).  events="f64": the server's own sample values
    (server_event_values) -> a RecordWindow64 of FP64 records, every field FP64 (pekf_run_rec64_dev's
    input), any dt."""
    K = np.asarray(ev["types"]).shape[1]
    E0 = np.asarray(ev["types"]).shape[0]
    evb, E, flags = _event_planes(ev, events)
    r_max = E0 // 3 + 1 if r_max is None else int(r_max)
    init = DeviceBuffer(48 * K).upload(np.concatenate([ev["init_acc"], ev["init_mag"]], axis=1).astype(np.float64))
    tib = DeviceBuffer(8 * K).upload(np.ascontiguousarray(ev["t_init"], np.int64))
    cnt = DeviceBuffer(4 * K)
    errb = DeviceBuffer(4)
    if events == "f64":
        win = RecordWindow64(K, max(1, r_max))
        errb.upload(np.zeros(1, np.int32))
        check(lib.pekf_frontend_ext_dev(K, E, evb.ptr, init.ptr, tib.ptr, float(alpha), r_max, win.gd.ptr,
                                        win.am.ptr, win.my.ptr, None, cnt.ptr, win.refs.ptr, flags, errb.ptr, None))
        check(lib.pekf_device_sync())
        if int(errb.download((1,), np.int32)[0]) & 2:
            raise ValueError("more than r_max=%d records for some filter" % r_max)
        win.counts = cnt.download((K,), np.int32)
        return win, win.counts
    win = IMUWindow(K, max(1, r_max))
    dtx = None
    while True:
        # without a side plane first; only if some record's dt does not fit the dt word (err bit 1: a
        # pause of 2^31 ns or more) run again with one (8 B per record slot, kept in win.dtx)
        errb.upload(np.zeros(1, np.int32))
        check(lib.pekf_frontend_ext_dev(K, E, evb.ptr, init.ptr, tib.ptr, float(alpha), r_max, win.gd.ptr,
                                        win.am.ptr, win.my.ptr, dtx.ptr if dtx is not None else None, cnt.ptr,
                                        win.refs.ptr, flags, errb.ptr, None))
        check(lib.pekf_device_sync())
        err = int(errb.download((1,), np.int32)[0])
        if err & 1 and dtx is None:
            dtx = DeviceBuffer(8 * K * max(1, r_max))
            continue
        break
    if err & 2:
        raise ValueError("more than r_max=%d records for some filter" % r_max)
    if err & 4:
        win.dtx = dtx
    win.counts = cnt.download((K,), np.int32)
    return win, win.counts


def frontend_init(ev, n_avg=100, stats=True, events="f32"):
    """Phase-2 events (synth.generate_events layout; ev["t_init"] = the time before the first one) ->
    dict(init (K, 6) raw {acc, mag} means, t_init (K,) int64, ready (K,) bool, gyro_mean (K, 3),
    var_acc / var_mag / var_gyro (K, 3)) by pekf_frontend_init_ext_dev: the inputs run_frontend needs
    for phase 3 (KFS/Parser.cpp:36-58,84-140, KFS/InitialValues.cpp).  stats=False: init / t_init /
    ready only (the kernel then skips its second pass, the variances).  events: as run_frontend ("f64":
    the statistics of the server's own sample values)."""
    K = np.asarray(ev["types"]).shape[1]
    evb, E, flags = _event_planes(ev, events)   # phase 2 always honours time events
    tsb = DeviceBuffer(8 * K).upload(np.ascontiguousarray(ev["t_init"], np.int64))
    ib, tib, rb = DeviceBuffer(48 * K), DeviceBuffer(8 * K), DeviceBuffer(4 * K)
    sb = DeviceBuffer(96 * K) if stats else None
    check(lib.pekf_frontend_init_ext_dev(K, E, evb.ptr, tsb.ptr, int(n_avg), ib.ptr, tib.ptr,
                                         sb.ptr if stats else None, rb.ptr, flags & EV_F64_EVENTS, None))
    check(lib.pekf_device_sync())
    out = dict(init=ib.download((K, 6), np.float64), t_init=tib.download((K,), np.int64),
               ready=rb.download((K,), np.int32).astype(bool))
    if stats:
        st = sb.download((K, 12), np.float64)
        out.update(gyro_mean=st[:, 0:3], var_acc=st[:, 3:6], var_mag=st[:, 6:9], var_gyro=st[:, 9:12])
    return out


def _record_flags(records, events="f32"):
    """pekf_live_ext_dev's record precision: "f64" (the low-pass acc / mag as the server's filter gets them,
    KFS/KalmanFilter.cpp:279-303) or "f32" (the 40 B stream record, as the split pipeline's).  FP64 events
    always make FP64 records."""
    if records not in ("f64", "f32"):
        raise ValueError("records must be 'f64' or 'f32'")
    if events == "f64" and records != "f64":
        raise ValueError("FP64 events make FP64 records (records='f64')")
    return EV_F32_RECORDS if records == "f32" else 0


def run_session(phase2, phase3, filters, n_avg=100, alpha=0.1, records="f64", events="f32"):
    """A whole client session of the server on the device (KFS/Parser.cpp:28-72): phase-2 events ->
    initial means and start time (pekf_frontend_init_dev) -> phase-3 events -> records -> the filters'
    state (pekf_live_dev), the phase-2 results handed over in device memory.  phase3's times continue
    phase2's (its first gap is taken from phase2's last event, the time phase 3 starts from).
    filters: a BatchedEKF (FP64, AoS) whose state is advanced; records and events as
    BatchedEKF.run_events.
    Returns dict(ready (K,) bool -- a filter
    that never finished phase 2 has NaN references, applies no record and keeps its state --, counts
    (K,) records applied, refs (K, 6))."""
    K = filters.batch
    assert np.asarray(phase2["types"]).shape[1] == K and np.asarray(phase2["types"]).shape[0] > 0
    assert np.asarray(phase3["types"]).shape[1] == K
    t_last = np.asarray(phase2["times"], np.int64)[-1]
    ev2, E2, flags2 = _event_planes(phase2, events)
    ev3, E3, flags3 = _event_planes(dict(phase3, t_init=t_last), events)
    tsb = DeviceBuffer(8 * K).upload(np.ascontiguousarray(phase2["t_init"], np.int64))
    ib, tib, rb = DeviceBuffer(48 * K), DeviceBuffer(8 * K), DeviceBuffer(4 * K)
    check(lib.pekf_frontend_init_ext_dev(K, E2, ev2.ptr, tsb.ptr, int(n_avg), ib.ptr, tib.ptr, None, rb.ptr,
                                         flags2 & EV_F64_EVENTS, None))
    cnt, refs = DeviceBuffer(4 * K), DeviceBuffer(48 * K)
    filters.run_events_async(ev3, E3, ib, tib, cnt, refs, alpha, flags=flags3 | _record_flags(records, events))
    check(lib.pekf_device_sync())
    return dict(ready=rb.download((K,), np.int32).astype(bool), counts=cnt.download((K,), np.int32),
                refs=refs.download((K, 6), np.float64))


def wire_events(frames, stream=None, frame_rows=False):
    """The clients' 100-byte wire frames -> FP64 event planes on the device (pekf_wire_events_ext_dev).

    frames: [n_frames][batch][100] uint8 (wire.frames) as a host array or a (DeviceBuffer, n_frames,
    batch) triple.  Returns dict(ev2, ev3 DeviceBuffers [n_frames][batch] double4, E2 / E3 the rows a
    consumer needs -- the most messages any phone has in phase 2 / 3, or with frame_rows n_frames --,
    n2 / n3 (batch,) int32 messages per phase, first_t2 DeviceBuffer (batch,) int64 (phase 2's t_start);
    with frame_rows, ev2's first E2 rows and ev3's E3 rows from row ev3_from hold every message).
    frame_rows (PEKF_WIRE_FRAME_ROWS): row f of each plane is frame f's message of that phase or the
    no-message event (for phones whose rows would drift apart; the consumers skip those rows).  Raises
    if a phone's frame is not in the client's form (wire.parse on the host reads any form std::stod
    does)."""
    if isinstance(frames, tuple):
        fb, F, K = frames
    else:
        fr = np.ascontiguousarray(frames, np.uint8)
        if fr.ndim != 3 or fr.shape[2] != 100:
            raise ValueError("frames must be [n_frames][batch][100] bytes")
        F, K = fr.shape[:2]
        fb = DeviceBuffer(max(fr.nbytes, 4)).upload(fr)
    F, K = int(F), int(K)
    ev2, ev3 = DeviceBuffer(32 * max(F, 1) * K), DeviceBuffer(32 * max(F, 1) * K)
    t2b, n2b, n3b, badb = DeviceBuffer(8 * K), DeviceBuffer(4 * K), DeviceBuffer(4 * K), DeviceBuffer(4 * K)
    errb = DeviceBuffer(4).upload(np.zeros(1, np.int32))
    bounds = DeviceBuffer(8)
    check(lib.pekf_wire_events_ext_dev(K, F, fb.ptr, F, F, ev2.ptr, ev3.ptr, t2b.ptr, n2b.ptr, n3b.ptr, badb.ptr,
                                       errb.ptr, bounds.ptr if frame_rows else None,
                                       WIRE_FRAME_ROWS if frame_rows else 0, stream))
    check(lib.pekf_device_sync() if stream is None else lib.pekf_stream_sync(stream))
    n2, n3 = n2b.download((K,), np.int32), n3b.download((K,), np.int32)
    if int(errb.download((1,), np.int32)[0]) & 1:
        bad = badb.download((K,), np.int32)
        k = int(np.argmax(bad >= 0))
        raise ValueError("phone %d, frame %d: not in the client's message form (wire.parse reads it)" % (k, bad[k]))
    if frame_rows:  # the rows that hold messages of any phone: ev2's first E2, ev3's from row F - E3
        E2, E3 = (int(v) for v in bounds.download((2,), np.int32))
    else:
        E2, E3 = int(n2.max(initial=0)), int(n3.max(initial=0))
    return dict(ev2=ev2, ev3=ev3, E2=E2, E3=E3, ev3_from=F - E3 if frame_rows else 0, n2=n2, n3=n3,
                first_t2=t2b, frames=fb)


def run_wire_session(frames, filters, n_avg=100, alpha=0.1, stream=None, frame_rows=True):
    """A whole client session from the clients' wire frames, on the device end to end (KFS/Server.cpp's
    recv'd frames -> Parser.cpp:28-72): pekf_wire_events_ext_dev (the server's parse into FP64 event
    planes), pekf_frontend_init_ext_dev (phase 2) and pekf_live_ext_dev (phase 3 + the filter) on the
    server's own values, no host parse.  filters: a BatchedEKF (FP64, AoS).  Returns run_session's dict,
    the same with or without frame_rows.  frame_rows (default): planes with a row per frame index (see
    wire_events), whose stores stay coalesced when the phones' phase-1 / phase-2 parts differ in length
    and whose frames a small batch splits over several waves; phase 2 and phase 3 read only the rows that
    hold messages (65,536 phones: 5.0 ms against 6.0 compacted with aligned rows, 5.0 against 8.0 ms with
    rows 64 apart)."""
    w = wire_events(frames, stream, frame_rows)
    K = filters.batch
    ib, tib, rb = DeviceBuffer(48 * K), DeviceBuffer(8 * K), DeviceBuffer(4 * K)
    check(lib.pekf_frontend_init_ext_dev(K, w["E2"], w["ev2"].ptr, w["first_t2"].ptr, int(n_avg), ib.ptr, tib.ptr,
                                         None, rb.ptr, EV_F64_EVENTS, stream))
    cnt, refs = DeviceBuffer(4 * K), DeviceBuffer(48 * K)
    ev3 = w["ev3"]
    if w["ev3_from"]:  # (frame rows) the leading rows no phone has a phase-3 message in
        ev3 = types.SimpleNamespace(ptr=ev3.ptr + 32 * K * w["ev3_from"])
    filters.run_events_async(ev3, w["E3"], ib, tib, cnt, refs, alpha, stream, flags=EV_F64_EVENTS)
    check(lib.pekf_device_sync() if stream is None else lib.pekf_stream_sync(stream))
    return dict(ready=rb.download((K,), np.int32).astype(bool), counts=cnt.download((K,), np.int32),
                refs=refs.download((K, 6), np.float64))


# ------------------------------------------------------------------ the batched filter

class BatchedEKF:
    """B independent filters of the reference model, state resident on the device.

    Equivalent, filter by filter, to the reference's main_file.py:19-47 driver:
    KalmanFilter(T0, mag_0, acc_0) with setQ(q), setR(r), P = I, X = [1,0,0,0], then
    Prediction + Correction for every record.  `run` advances all filters n_steps records.
    """

    def __init__(self, batch, q=1.0, r=0.1, precision="f64", layout="aos"):
        """precision: "f64" (default, as the reference) or "mixed" (covariance path in f32).
        layout: "aos" (X[B][4], P[B][4][4]) or "soa" (X[4][B], P[10][B]: coalesced state access,
        for launches that cover few records, e.g. online serving)."""
        if precision not in ("f64", "mixed"):
            raise ValueError("precision must be 'f64' or 'mixed'")
        if layout not in ("aos", "soa"):
            raise ValueError("layout must be 'aos' or 'soa'")
        self.batch = int(batch)
        self.q, self.r = float(q), float(r)
        self.layout = layout
        self.flags = (RUN_MIXED_PRECISION if precision == "mixed" else 0) | (RUN_STATE_SOA if layout == "soa" else 0)
        self.X = DeviceBuffer(32 * self.batch)
        self.P = DeviceBuffer((80 if layout == "soa" else 128) * self.batch)
        self.reset()

    def _to_layout(self, Xa, Pa, to_soa, stream=None):
        check(lib.pekf_state_layout_dev(self.batch, Xa.ptr, Pa.ptr, self.X.ptr, self.P.ptr, int(to_soa), stream))

    def reset(self, stream=None):
        if self.layout == "soa":
            Xa, Pa = DeviceBuffer(32 * self.batch), DeviceBuffer(128 * self.batch)
            check(lib.pekf_reset_state_dev(self.batch, Xa.ptr, Pa.ptr, stream))
            self._to_layout(Xa, Pa, True, stream)
        else:
            check(lib.pekf_reset_state_dev(self.batch, self.X.ptr, self.P.ptr, stream))
        check(lib.pekf_device_sync() if stream is None else lib.pekf_stream_sync(stream))

    def set_state(self, X, P):
        """X (B, 4), P (B, 4, 4) in the reference's row-major layout, whatever self.layout is."""
        X, P = f64(X, (self.batch, 4)), f64(P, (self.batch, 4, 4))
        if self.layout == "soa":
            Xa, Pa = DeviceBuffer(X.nbytes).upload(X), DeviceBuffer(P.nbytes).upload(P)
            self._to_layout(Xa, Pa, True)
            check(lib.pekf_device_sync())
        else:
            self.X.upload(X)
            self.P.upload(P)

    def get_state(self):
        """(X (B, 4), P (B, 4, 4)) in the reference's row-major layout."""
        if self.layout == "soa":
            Xa, Pa = DeviceBuffer(32 * self.batch), DeviceBuffer(128 * self.batch)
            self._to_layout(Xa, Pa, False)
            check(lib.pekf_device_sync())
            return Xa.download((self.batch, 4), np.float64), Pa.download((self.batch, 4, 4), np.float64)
        return (self.X.download((self.batch, 4), np.float64),
                self.P.download((self.batch, 4, 4), np.float64))

    def run_async(self, win: IMUWindow, n_steps, step0=0, stream=None, traj=None, counts=None):
        """Enqueue one fused launch; traj: optional DeviceBuffer of n_steps*batch*32 bytes;
        counts: optional DeviceBuffer of batch int32 (filter b applies its first counts[b] records).
        A window with a dt side plane (escaped records) runs pekf_run_ext_dev with it; a RecordWindow64
        (FP64 records) runs pekf_run_rec64_dev."""
        assert win.batch == self.batch
        tr, cn = traj.ptr if traj is not None else None, counts.ptr if counts is not None else None
        if isinstance(win, RecordWindow64):
            if self.layout != "aos" or self.flags & RUN_MIXED_PRECISION:
                raise ValueError("FP64-record windows run the FP64 filter on AoS state")
            check(lib.pekf_run_rec64_dev(self.batch, int(n_steps), win.window, int(step0), win.gd.ptr, win.am.ptr,
                                         win.my.ptr, win.refs.ptr, self.X.ptr, self.P.ptr, self.q, self.r, tr, cn,
                                         stream))
        elif win.dtx is None:
            check(lib.pekf_run_dev(self.batch, int(n_steps), win.window, int(step0), win.gd.ptr, win.am.ptr,
                                   win.my.ptr, win.refs.ptr, self.X.ptr, self.P.ptr, self.q, self.r, tr, cn,
                                   self.flags, stream))
        else:
            check(lib.pekf_run_ext_dev(self.batch, int(n_steps), win.window, int(step0), win.gd.ptr, win.am.ptr,
                                       win.my.ptr, win.dtx.ptr, win.refs.ptr, self.X.ptr, self.P.ptr, self.q,
                                       self.r, tr, cn, self.flags, stream))

    def run(self, win: IMUWindow, n_steps=None, step0=0, want_traj=False, counts=None):
        """Advance every filter n_steps records (default: the whole window) from row step0.

        counts: per-filter record counts for this launch (array of batch ints or a DeviceBuffer);
        default win.counts (ragged logs / front-end output) shifted by step0, so each filter
        applies exactly its own records while sharing one launch."""
        n_steps = win.window if n_steps is None else int(n_steps)
        tb = DeviceBuffer(32 * n_steps * self.batch) if want_traj else None
        if counts is None and win.counts is not None:
            counts = np.clip(np.asarray(win.counts, np.int64) - int(step0), 0, n_steps)
        if counts is not None and not isinstance(counts, DeviceBuffer):
            c = np.ascontiguousarray(counts, dtype=np.int32).reshape(self.batch)
            counts = DeviceBuffer(c.nbytes).upload(c)
        self.run_async(win, n_steps, step0, None, tb, counts)
        check(lib.pekf_device_sync())
        if want_traj:
            return tb.download((n_steps, self.batch, 4), np.float64)
        return None

    def run_events_async(self, ev_planes, n_events, init, t_init, counts, refs, alpha=0.1, stream=None, flags=0):
        """Enqueue pekf_live_ext_dev: device event planes [n_events][batch][4] f32 (synth.pack_events), init
        (batch, 6), t_init (batch,) int64; counts (batch,) int32 and refs (batch, 6) outputs -- DeviceBuffers;
        flags: EV_TIME_EVENTS if the planes hold time events, EV_F32_RECORDS for f32 records."""
        if self.layout != "aos" or self.flags & RUN_MIXED_PRECISION:
            raise ValueError("the fused front-end + filter kernel runs the FP64 filter on AoS state")
        check(lib.pekf_live_ext_dev(self.batch, int(n_events), ev_planes.ptr, init.ptr, t_init.ptr, float(alpha),
                                    self.X.ptr, self.P.ptr, self.q, self.r, counts.ptr, refs.ptr, int(flags), None,
                                    stream))

    def run_events(self, ev, alpha=0.1, records="f64", events="f32"):
        """Raw phone events (synth.generate_events layout) -> front-end -> filter, fused in one launch
        (pekf_live_ext_dev).  Returns (counts (batch,) int32 records applied, refs (batch, 6)
        the filters' acc0 / mag0).  Any event gap and any record dt is applied (time events, escapes).
        records: "f64" (default) feeds the filter the FP64 low-pass acc / mag, as the server does
        (KFS/KalmanFilter.cpp:279-303); "f32" rounds them to the 40 B stream record first, which makes the
        result equal run_frontend + run bit for bit.
        events: "f32" the float32 samples (16 B events); "f64" the server's own values (32 B events,
        server_event_values: what std::stod parses from the phone's text), every record field FP64 --
        equal to run_frontend(events="f64") + run bit for bit."""
        assert np.asarray(ev["types"]).shape[1] == self.batch
        evb, E, flags = _event_planes(ev, events)
        init = DeviceBuffer(48 * self.batch).upload(
            np.concatenate([ev["init_acc"], ev["init_mag"]], axis=1).astype(np.float64))
        tib = DeviceBuffer(8 * self.batch).upload(np.ascontiguousarray(ev["t_init"], np.int64))
        cnt, refs = DeviceBuffer(4 * self.batch), DeviceBuffer(48 * self.batch)
        self.run_events_async(evb, E, init, tib, cnt, refs, alpha, flags=flags | _record_flags(records, events))
        check(lib.pekf_device_sync())
        return cnt.download((self.batch,), np.int32), refs.download((self.batch, 6), np.float64)


class FilterHandle:
    """B KalmanFilter objects behind one native handle (pekf_filter_*).

    The handle owns what the reference object owns (ExtendedKalmanFilter.py:6-15): the Wahba
    reference (acc0, mag0), Q = q I, R = r I and previousT, plus the state X, P, which stays in
    device memory.  `update` is one main_file.py:42-45 iteration for every filter from FP64
    host arrays (online serving); `run` advances the same state through a resident stream window.
    """

    def __init__(self, acc0, mag0, q=1.0, r=0.1, t0_ns=None, precision="f64", layout="aos"):
        acc0 = np.ascontiguousarray(acc0, np.float64).reshape(-1, 3)
        mag0 = np.ascontiguousarray(mag0, np.float64).reshape(-1, 3)
        self.batch = acc0.shape[0]
        assert mag0.shape[0] == self.batch
        flags = (RUN_MIXED_PRECISION if precision == "mixed" else 0) | (RUN_STATE_SOA if layout == "soa" else 0)
        t0 = None if t0_ns is None else np.ascontiguousarray(t0_ns, np.int64).reshape(self.batch)
        h = ctypes.c_void_p()
        check(lib.pekf_filter_create(self.batch, acc0.ctypes.data, mag0.ctypes.data, float(q), float(r),
                                     t0.ctypes.data if t0 is not None else None, flags, ctypes.byref(h)))
        self.h = h.value

    def update(self, gyro, t_ns, acc, mag, missing=None, want_x=True):
        """One record per filter: Prediction(gyro, t_ns) + Correction(mag, acc). Returns X (B, 4)."""
        B = self.batch
        g, a, m = (np.ascontiguousarray(v, np.float64).reshape(B, 3) for v in (gyro, acc, mag))
        t = np.ascontiguousarray(t_ns, np.int64).reshape(B)
        miss = None if missing is None else np.ascontiguousarray(missing, np.uint8).reshape(B)
        X = np.empty((B, 4)) if want_x else None
        check(lib.pekf_filter_update(self.h, g.ctypes.data, t.ctypes.data, a.ctypes.data, m.ctypes.data,
                                     miss.ctypes.data if miss is not None else None,
                                     X.ctypes.data if X is not None else None))
        return X

    def run(self, win: IMUWindow, n_steps=None, step0=0, want_traj=False, counts=None):
        """pekf_filter_run over a resident window (the window's refs are not used: the handle's are)."""
        n_steps = win.window if n_steps is None else int(n_steps)
        assert win.batch == self.batch
        tb = DeviceBuffer(32 * n_steps * self.batch) if want_traj else None
        if counts is None and win.counts is not None:
            counts = np.clip(np.asarray(win.counts, np.int64) - int(step0), 0, n_steps)
        cb = None
        if counts is not None:
            c = np.ascontiguousarray(counts, dtype=np.int32).reshape(self.batch)
            cb = DeviceBuffer(c.nbytes).upload(c)
        check(lib.pekf_filter_run_ext(self.h, n_steps, win.window, int(step0), win.gd.ptr, win.am.ptr, win.my.ptr,
                                      win.dtx.ptr if win.dtx is not None else None,
                                      tb.ptr if tb is not None else None, cb.ptr if cb is not None else None, None))
        check(lib.pekf_device_sync())
        return tb.download((n_steps, self.batch, 4), np.float64) if want_traj else None

    def set_state(self, X=None, P=None):
        Xa = None if X is None else f64(X, (self.batch, 4))
        Pa = None if P is None else f64(P, (self.batch, 4, 4))
        check(lib.pekf_filter_set_state(self.h, Xa.ctypes.data if Xa is not None else None,
                                        Pa.ctypes.data if Pa is not None else None))

    def get_state(self):
        X, P = np.empty((self.batch, 4)), np.empty((self.batch, 4, 4))
        check(lib.pekf_filter_get_state(self.h, X.ctypes.data, P.ctypes.data))
        return X, P

    def set_time(self, t_ns):
        t = np.ascontiguousarray(t_ns, np.int64).reshape(self.batch)
        check(lib.pekf_filter_set_time(self.h, t.ctypes.data))

    def get_time(self):
        """previousT of every filter (B,) int64 ns (KalmanFilter.previousT)."""
        t = np.empty(self.batch, np.int64)
        check(lib.pekf_filter_get_time(self.h, t.ctypes.data))
        return t

    def close(self):
        if getattr(self, "h", None):
            lib.pekf_filter_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ batched per-call operators
# NumPy-level wrappers over the host-pointer entry points (one GPU thread per item).

def _in(a, shape):
    """Read-only C-contiguous float64 view of an input (copied only if it is not one already):
    the host-pointer entry points never write their inputs."""
    return np.ascontiguousarray(a, dtype=np.float64).reshape(shape)


def _n(a, k):
    return np.size(a) // k


def _p(a):
    return a.ctypes.data


def rk4(q0, dt_ns, w):
    n = _n(q0, 4)
    q0, dt, w = _in(q0, (n, 4)), _in(dt_ns, (n,)), _in(w, (n, 3))
    out = np.empty((n, 4))
    check(lib.pekf_rk4(n, _p(q0), _p(dt), _p(w), _p(out)))
    return out


def norm(a):
    """Row norms of a (n, len) array, sequential sum of squares (UtilityFunctions.py:16-21)."""
    a = np.atleast_2d(np.ascontiguousarray(a, dtype=np.float64))
    n, k = a.shape
    out = np.empty(n)
    check(lib.pekf_norm(n, k, _p(a), _p(out)))
    return out


def jacobian_a(w):
    n = _n(w, 3)
    w = _in(w, (n, 3))
    out = np.empty((n, 4, 4))
    check(lib.pekf_jacobian_a(n, _p(w), _p(out)))
    return out


def jacobian_b(q):
    n = _n(q, 4)
    q = _in(q, (n, 4))
    out = np.empty((n, 4, 3))
    check(lib.pekf_jacobian_b(n, _p(q), _p(out)))
    return out


def comparator(q1, q2):
    n = _n(q1, 4)
    a, b = _in(q1, (n, 4)), _in(q2, (n, 4))
    out = np.empty((n, 4))
    check(lib.pekf_comparator(n, _p(a), _p(b), _p(out)))
    return out


def predict(gyro, dt_ns, X, P, Q, R):
    n = _n(X, 4)
    args = (_in(gyro, (n, 3)), _in(dt_ns, (n,)), _in(X, (n, 4)), _in(P, (n, 4, 4)),
            _in(Q, (n, 3, 3)), _in(R, (n, 4, 4)))
    z, Pm, K = np.empty((n, 4)), np.empty((n, 4, 4)), np.empty((n, 4, 4))
    check(lib.pekf_predict(n, *[_p(a) for a in args], _p(z), _p(Pm), _p(K)))
    return z, Pm, K


def correct(mag, acc, z, P, K, acc0, mag0):
    n = _n(z, 4)
    args = (_in(mag, (n, 3)), _in(acc, (n, 3)), _in(z, (n, 4)), _in(P, (n, 4, 4)), _in(K, (n, 4, 4)),
            _in(acc0, (n, 3)), _in(mag0, (n, 3)))
    X, Po = np.empty((n, 4)), np.empty((n, 4, 4))
    check(lib.pekf_correct(n, *[_p(a) for a in args], _p(X), _p(Po)))
    return X, Po


def _wahba(fn, k, acc0, mag0, acc, mag, k_acc, k_mag):
    n = _n(acc, 3)
    args = (_in(acc0, (n, 3)), _in(mag0, (n, 3)), _in(acc, (n, 3)), _in(mag, (n, 3)),
            _in(k_acc, (n,)), _in(k_mag, (n,)))
    out = np.empty((n,) + k)
    check(fn(n, *[_p(a) for a in args], _p(out)))
    return out


def wahba_rotation(acc0, mag0, acc, mag, k_acc, k_mag):
    return _wahba(lib.pekf_wahba_rotation, (3, 3), acc0, mag0, acc, mag, k_acc, k_mag)


def wahba_quaternion(acc0, mag0, acc, mag, k_acc, k_mag):
    return _wahba(lib.pekf_wahba_quaternion, (4,), acc0, mag0, acc, mag, k_acc, k_mag)


def quat_to_rpy(q):
    """UtilityFunctions.Quart2RPY for each row of q (n,4): roll, pitch, yaw in degrees."""
    n = _n(q, 4)
    q = _in(q, (n, 4))
    out = np.empty((n, 3))
    check(lib.pekf_quat_to_rpy(n, _p(q), _p(out)))
    return out


def rotmat_to_quat(M):
    n = _n(M, 9)
    M = _in(M, (n, 3, 3))
    out = np.empty((n, 4))
    check(lib.pekf_rotmat_to_quat(n, _p(M), _p(out)))
    return out
