"""The phone -> server link: the sample values the server computes with.

The Android client sends every sample as text -- ``Float.toString`` of each value, in
``"#<phase>,<type>:<x>,<y>,<z>,t:<ns>"`` padded with spaces to 99 characters
(ASC/MessageSender.java:217-233, ConvertSensorMsg) -- and the server parses the values with
``std::stod`` (KFS/Parser.cpp:12-26).  The server's filter therefore starts from the doubles nearest
the printed decimals, not from the floats the phone measured (``"0.1"`` is 0.1, not
0.100000001490116...).  The FP64 event planes (``PEKF_EV_F64_EVENTS``, include/pekf.h) carry exactly
those doubles; this module produces them, natively (libpekf's host functions, csrc/pekf_wire.cpp):

* :func:`parse` -- the server's own parse of wire text (``pekf_wire_parse``);
* :func:`server_values` -- for samples known only as float32, the double the server would parse from
  ``Float.toString(f)`` (``pekf_f32_wire_values``);
* :func:`message` / :func:`events_text` -- the client's text for given samples (what the phone sends,
  JDK 19+ ``Float.toString`` formatting), for feeding recorded or synthetic streams through the same
  parse;
* :func:`events_from_wire` -- per-filter wire streams -> the event dict the engine takes.
"""
from __future__ import annotations

import ctypes
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import synth
from ._lib import check, lib


def server_values(values):
    """float32 samples (any shape) -> float64: std::stod(Float.toString(f)) for each (large arrays in
    chunks on a thread pool: the conversion runs in libpekf with the GIL released)."""
    f = np.ascontiguousarray(values, np.float32)
    out = np.empty(f.shape, np.float64)
    fr, orv = f.reshape(-1), out.reshape(-1)
    chunk = 1 << 20
    starts = range(0, fr.size, chunk)

    def run(s):
        n = min(chunk, fr.size - s)
        check(lib.pekf_f32_wire_values(n, fr[s:].ctypes.data, orv[s:].ctypes.data))
    workers = max(1, min(len(starts), os.cpu_count() or 1, 32))
    if workers > 1:
        with ThreadPoolExecutor(workers) as pool:
            list(pool.map(run, starts))
    else:
        for s in starts:
            run(s)
    return out


def parse(text):
    """Wire text (str or bytes, one message per line) -> dict(phase (n,) uint8, types (n,) uint8,
    values (n, 3) float64, times (n,) int64), as the server's Parser reads it."""
    b = text.encode() if isinstance(text, str) else bytes(text)
    # one pass: a counted message is '#' and more than 30 characters, so there are at most len / 32 + 1
    cap = len(b) // 32 + 1
    ph, ty = np.empty(cap, np.uint8), np.empty(cap, np.uint8)
    xyz, t = np.empty((cap, 3), np.float64), np.empty(cap, np.int64)
    n = ctypes.c_int64()
    check(lib.pekf_wire_parse(b, len(b), cap, ph.ctypes.data, ty.ctypes.data, xyz.ctypes.data, t.ctypes.data,
                              ctypes.byref(n)))
    n = n.value
    return dict(phase=ph[:n].copy(), types=ty[:n].copy(), values=xyz[:n].copy(), times=t[:n].copy())


def java_float_string(f):
    """Float.toString(f) as JDK 19+ prints it: the shortest decimal that rounds to f, the closest among
    those (one or two digits when one suffices), as "ddd.ddd" for 1e-3 <= |f| < 1e7, else "d.dddE[-]n"."""
    f = np.float32(f)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if np.signbit(f) else "0.0"
    sci = np.format_float_scientific(f, unique=True, trim="-")       # shortest digits, e.g. "1.2345e-05"
    mant, exp = sci.split("e")
    if len(mant.lstrip("-").replace(".", "")) == 1:                   # one digit: the closest of one or two
        mant, exp = ("%.1e" % float(f)).split("e")
    neg = mant.startswith("-")
    digits = mant.lstrip("-").replace(".", "").rstrip("0") or "0"
    e = int(exp)
    a = abs(float(f))
    if 1e-3 <= a < 1e7:
        if e >= 0:
            ip = digits[:e + 1].ljust(e + 1, "0")
            fp = digits[e + 1:] or "0"
        else:
            ip, fp = "0", "0" * (-e - 1) + digits
        s = ip + "." + fp
    else:
        s = digits[0] + "." + (digits[1:] or "0") + "E" + str(e)
    return ("-" if neg else "") + s


def message(phase, sensor_type, xyz, t_ns):
    """One client message (ConvertSensorMsg, MessageSender.java:217-233): "#p,t:x,y,z,t:ns" padded with
    spaces to 99 characters; println adds the newline."""
    s = "#%d,%d:" % (int(phase), int(sensor_type))
    for v in np.asarray(xyz, np.float32).reshape(3):
        s += java_float_string(v) + ","
    s += "t:%d" % int(t_ns)
    return s.ljust(99) + "\n"


def events_text(types, values, times, phase=3):
    """One filter's stream of float32 samples -> the text the phone sends (one message per event)."""
    return "".join(message(phase, ty, v, t) for ty, v, t in zip(np.asarray(types), np.asarray(values, np.float32),
                                                               np.asarray(times)))


def events_from_wire(texts, init_acc, init_mag, t_init, phase=3):
    """Per-filter wire texts -> the engine's event dict (types (E, K), values64 (E, K, 3) the server's
    doubles, times (E, K), init_acc / init_mag (K, 3), t_init (K,)).  Messages of other phases are
    dropped; a message whose sensor type is not 0 / 1 / 2 keeps its time as type synth.EV_OTHER (3): no
    sensor takes its sample (KFS/Parser.cpp:148-219), but in phase 2 it is a message like any other
    (:36-62); streams of different lengths are padded with synth.EV_NONE (4): no message at all."""
    texts = list(texts)
    # one text per thread: the parse runs in libpekf with the GIL released (ctypes)
    workers = max(1, min(len(texts), os.cpu_count() or 1, 32))
    if workers > 1:
        with ThreadPoolExecutor(workers) as pool:
            ps = list(pool.map(parse, texts))
    else:
        ps = [parse(t) for t in texts]
    ps = [{k: v[p["phase"] == phase] for k, v in p.items()} for p in ps]
    E, K = max((len(p["types"]) for p in ps), default=0), len(ps)
    types = np.full((E, K), synth.EV_NONE, np.uint32)
    vals = np.zeros((E, K, 3), np.float64)
    times = np.zeros((E, K), np.int64)
    for k, p in enumerate(ps):
        n = len(p["types"])
        types[:n, k] = np.where(p["types"] <= 2, p["types"], synth.EV_OTHER)
        vals[:n, k] = p["values"]
        times[:n, k] = p["times"]
        times[n:, k] = p["times"][-1] if n else int(np.asarray(t_init).reshape(-1)[k])
    with np.errstate(over="ignore"):  # a double beyond the float range is +-inf as a float
        vals32 = vals.astype(np.float32)
    return dict(types=types, values64=vals, values=vals32, times=times,
                init_acc=np.asarray(init_acc, np.float64).reshape(K, 3),
                init_mag=np.asarray(init_mag, np.float64).reshape(K, 3),
                t_init=np.asarray(t_init, np.int64).reshape(K))


FRAME = 100  # bytes per message, as the client sends it and the server receives it (Server.cpp:35,84)


def frames(texts, n_frames=None):
    """Per-phone wire texts -> the [n_frames][K][100] uint8 frame array of engine.wire_events: each text cut
    into the server's 100-byte recv frames (its length must be a multiple of 100, as the client's messages
    are); shorter streams are padded with blank frames (no message)."""
    bs = [t.encode() if isinstance(t, str) else bytes(t) for t in texts]
    for k, b in enumerate(bs):
        if len(b) % FRAME:
            raise ValueError("text %d is %d bytes, not whole %d-byte frames" % (k, len(b), FRAME))
    F = max((len(b) // FRAME for b in bs), default=0) if n_frames is None else int(n_frames)
    out = np.full((F, len(bs), FRAME), ord(" "), np.uint8)
    for k, b in enumerate(bs):
        a = np.frombuffer(b, np.uint8).reshape(-1, FRAME)[:F]
        out[:a.shape[0], k] = a
    return out


__all__ = ["server_values", "parse", "java_float_string", "message", "events_text", "events_from_wire", "frames",
           "FRAME"]
