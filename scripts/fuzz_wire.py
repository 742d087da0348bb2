#!/usr/bin/env python3
"""Randomised check of the device wire parser (pekf_wire_events_dev) against the host parse
(pekf_wire_parse, itself checked against Python's float() in tests/test_wire.py), on the GPU box.

Each case: 64-300 phones, each a stream of client frames -- random float32 samples of every class printed
as Float.toString prints them (plain and computerized forms, subnormals, NaN, Infinity), random phases
(1, 2, 3, others), sensor types (0-2 and others), blank and non-'#' frames -- and, with some probability per
frame, a corruption: a number replaced by a random decimal (1-25 digits, exponents to +-120, signs,
leading zeros), by a form strtod reads but the client never prints (blanks, hex, inf, trailing text), a
deleted character, or a random byte other than '\n'.  (The server takes each 100-byte recv as one message,
KFS/Server.cpp:84-98, as the device does; the host parse splits its text at newlines -- the two agree on
every frame without an inner newline, and a newline in the Type field would be a message to the one and
two lines to the other.)  Per phone the device must either parse every frame exactly as the
host does (the same phase-2 / phase-3 events bit for bit, counts and first phase-2 time), or report the
phone's first frame it does not take; that frame must be one of the corrupted ones, and the frames
before it must match the host's.

usage: python3 scripts/fuzz_wire.py [--cases N] [--seed S] [--corrupt P] [--rows]   (exit status 1 on any difference)
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from poseestimationkf_amd import engine, synth, wire  # noqa: E402
from poseestimationkf_amd._lib import check, lib  # noqa: E402


def rand_decimal(rng):
    nd = int(rng.integers(1, 26))
    digits = "".join(str(d) for d in rng.integers(0, 10, nd))
    point = int(rng.integers(0, nd + 1))
    s = "0" * int(rng.integers(0, 3)) + digits[:point] + ("." + digits[point:] if rng.random() < 0.7 else "")
    if rng.random() < 0.5:
        s += rng.choice(["e", "E"]) + rng.choice(["", "+", "-"]) + str(int(rng.integers(0, 121)))
    return rng.choice(["", "-", "+"]) + s


ODD = [" 1.5", "\t2", "0x1p-3", "inf", "-inf", "nan", "1.5abc", "1e", "1e+", ".", "-", "1..2", "++1", "1,5"]


def phone_text(rng, n, corrupt_rate=0.05):
    with np.errstate(over="ignore"):  # beyond the float range: +-inf, printed "Infinity"
        vals = (rng.standard_normal((n, 3)) * 10.0 ** rng.integers(-45, 39, (n, 3))).astype(np.float32)
    for special in (np.nan, np.inf, -np.inf, np.float32(1.4e-45), np.float32(-0.0)):
        vals[rng.random(vals.shape) < 0.01] = special
    t = int(rng.integers(0, 10 ** 13)) + np.cumsum(rng.integers(0, 4_000_000, n))
    frames, corrupt = [], []
    for i in range(n):
        u = rng.random()
        if u < 0.02:
            frames.append(" " * 99 + "\n")
            corrupt.append(False)
            continue
        phase = int(rng.choice([1, 2, 3, 3, 3, 2, 4]))
        ty = str(rng.choice(["0", "1", "2", "0", "1", "2", "7", "x"]))
        toks = [wire.java_float_string(v) for v in vals[i]]
        bad = False
        if rng.random() < corrupt_rate:
            k = int(rng.integers(0, 3))
            toks[k] = rand_decimal(rng) if rng.random() < 0.7 else str(rng.choice(ODD))
            bad = True
        s = "#%d,%s:%s,%s,%s,t:%d" % (phase, ty, toks[0], toks[1], toks[2], t[i])
        if rng.random() < corrupt_rate / 5:
            j = int(rng.integers(1, len(s)))
            s = s[:j] + s[j + 1:]
            bad = True
        if rng.random() < corrupt_rate / 10:
            j = int(rng.integers(0, len(s)))
            c = int(rng.integers(1, 126))
            s = s[:j] + chr(c + (c >= 10)) + s[j + 1:]  # not '\n': see the module docstring
            bad = True
        if len(s) > 99:
            s = s[:99]
            bad = True
        frames.append(s.ljust(99) + "\n")
        corrupt.append(bad)
    return frames, corrupt


def host_events(frames, upto, phase):
    """The host parse of frames [0, upto) of one phone: its phase-`phase` FP64 events, or None if the host
    rejects one of them (std::stod / std::stoll would throw: the device must not have taken it)."""
    text = "".join(frames[:upto])
    try:
        p = wire.parse(text)
    except Exception:
        return None
    sel = p["phase"] == phase
    ev = dict(types=np.where(p["types"][sel] <= 2, p["types"][sel], synth.EV_OTHER)[:, None],
              times=p["times"][sel][:, None], values64=p["values"][sel][:, None, :])
    return synth.pack_events64(ev)[:, 0] if sel.any() else np.zeros((0, 4))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--corrupt", type=float, default=0.05, help="per-frame probability of a replaced number")
    ap.add_argument("--rows", action="store_true", help="PEKF_WIRE_FRAME_ROWS planes (compacted here to compare)")
    a = ap.parse_args(argv)
    rng = np.random.default_rng(a.seed)
    n_frames = n_bad_phones = differ = 0
    for case in range(a.cases):
        K = int(rng.integers(64, 301))
        texts, corr = [], []
        for _ in range(K):
            fr, c = phone_text(rng, int(rng.integers(1, 120)), a.corrupt)
            texts.append(fr)
            corr.append(c)
        F = max(len(t) for t in texts)
        frames = wire.frames(["".join(t) for t in texts], F)
        n_frames += sum(len(t) for t in texts)
        fb = engine.DeviceBuffer(frames.nbytes).upload(frames)
        ev2, ev3 = engine.DeviceBuffer(32 * F * K), engine.DeviceBuffer(32 * F * K)
        t2b, n2b, n3b, badb = (engine.DeviceBuffer(8 * K), engine.DeviceBuffer(4 * K), engine.DeviceBuffer(4 * K),
                               engine.DeviceBuffer(4 * K))
        errb = engine.DeviceBuffer(4).upload(np.zeros(1, np.int32))
        check(lib.pekf_wire_events_ext_dev(K, F, fb.ptr, F, F, ev2.ptr, ev3.ptr, t2b.ptr, n2b.ptr, n3b.ptr,
                                           badb.ptr, errb.ptr, None, 1 if a.rows else 0, None))
        check(lib.pekf_device_sync())
        d2, d3 = ev2.download((F, K, 4), np.float64), ev3.download((F, K, 4), np.float64)
        n2, n3 = n2b.download((K,), np.int32), n3b.download((K,), np.int32)
        t2, bad = t2b.download((K,), np.int64), badb.download((K,), np.int32)
        for k in range(K):
            upto = len(texts[k]) if bad[k] < 0 else int(bad[k])
            if bad[k] >= 0:
                n_bad_phones += 1
                if not corr[k][bad[k]]:
                    print("case %d phone %d: frame %d refused but not corrupted: %r" % (case, k, bad[k],
                                                                                      texts[k][bad[k]]))
                    differ += 1
                    continue
            for phase, dev, n in ((2, d2, n2), (3, d3, n3)):
                h = host_events(texts[k], upto, phase)
                if h is None:
                    print("case %d phone %d: the device took a frame the host parse rejects" % (case, k))
                    differ += 1
                    break
                if a.rows:  # a row per frame index: the rows that are not the no-message event, in order
                    col = dev[:, k]
                    got = col[col[:, 3:4].view(np.uint64)[:, 0] != np.uint64(synth.EV64_NONE_W)]
                    if got.shape[0] != h.shape[0]:
                        print("case %d phone %d phase %d: %d rows, the host %d" % (case, k, phase, got.shape[0],
                                                                                 h.shape[0]))
                        differ += 1
                        continue
                else:
                    got = dev[:h.shape[0], k]
                ok = n[k] == h.shape[0] and np.array_equal(got.view(np.uint64), h.view(np.uint64))
                if phase == 2 and h.shape[0]:
                    first = (h[0:1, 3].view(np.uint64) & ~np.uint64(3)).view(np.float64)[0]
                    ok = ok and t2[k] == int(first)
                if not ok:
                    print("case %d phone %d phase %d: device differs from the host parse" % (case, k, phase))
                    differ += 1
        if (case + 1) % 5 == 0 or case + 1 == a.cases:
            print("%d cases, %d frames, %d phones stopped at a frame the device does not take, %d differ"
                  % (case + 1, n_frames, n_bad_phones, differ), flush=True)
    print("done: %d cases, %d frames, %d differ" % (a.cases, n_frames, differ))
    return 1 if differ else 0


if __name__ == "__main__":
    sys.exit(main())
