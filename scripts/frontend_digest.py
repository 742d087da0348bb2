#!/usr/bin/env python3
"""The front-end kernels' outputs on fixed generated streams, saved to an .npz, to compare two builds of
libpekf.so bit for bit (select the build with PEKF_LIB=...): a change to pekf_phase3.hpp that only moves
values differently (register layout, masked moves instead of selects) must leave every output unchanged.

Outputs: k_frontend's records (f32 events -> 40 B records, with time events and escaped dts; FP64 events
-> FP64 records), each plane masked to the filter's own record count; k_live's final state, counts and
reference pairs for every event / record form (FP64 records, f32 records, FP64 events, time events).

usage: python3 scripts/frontend_digest.py <out.npz>
       python3 scripts/frontend_digest.py --compare <a.npz> <b.npz>    (exit status 1 on any difference)
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def _streams():
    from poseestimationkf_amd import synth
    K, E = 16384, 600
    plain = synth.generate_events(np.arange(K), E, seed=91)
    # a second set with pauses the 30-bit gap field cannot hold (time events) and record dts past 2^31 ns
    # (escaped), on every 7th filter
    paused = synth.generate_events(np.arange(K), E, seed=92)
    t = np.asarray(paused["times"], np.int64).copy()
    jump = np.zeros_like(t)
    jump[E // 3:, ::7] = 3 << 30
    jump[2 * E // 3:, ::7] += 5 << 31
    paused = dict(paused, times=t + jump)
    return {"plain": plain, "paused": paused}


def _masked(planes, counts):
    W = planes.shape[0]
    keep = np.arange(W)[:, None] < np.asarray(counts)[None, :]
    return np.where(keep.reshape(keep.shape + (1,) * (planes.ndim - 2)), planes, 0)


def digest(path):
    from poseestimationkf_amd import engine
    out = {}
    for name, ev in _streams().items():
        K = np.asarray(ev["types"]).shape[1]
        win, cnt = engine.run_frontend(ev)
        out[name + "/fe_counts"] = cnt
        for pl, shape in (("gd", 4), ("am", 4), ("my", 2)):
            out[name + "/fe_" + pl] = _masked(getattr(win, pl).download((win.window, K, shape), np.float32), cnt)
        if win.dtx is not None:
            out[name + "/fe_dtx"] = _masked(win.dtx.download((win.window, K), np.float64), cnt)
        f = engine.BatchedEKF(K)
        f.run(win)
        out[name + "/split_X"], out[name + "/split_P"] = f.get_state()
        w64, c64 = engine.run_frontend(ev, events="f64")
        out[name + "/fe64_counts"] = c64
        for pl, shape in (("gd", 4), ("am", 4), ("my", 2)):
            out[name + "/fe64_" + pl] = _masked(getattr(w64, pl).download((w64.window, K, shape), np.float64), c64)
        for records, events in (("f64", "f32"), ("f32", "f32"), ("f64", "f64")):
            f = engine.BatchedEKF(K)
            c, refs = f.run_events(ev, records=records, events=events)
            key = "%s/live_r%s_e%s_" % (name, records, events)
            out[key + "counts"], out[key + "refs"] = c, refs
            out[key + "X"], out[key + "P"] = f.get_state()
    np.savez(path, **out)
    print("wrote %s: %d arrays" % (path, len(out)))


def compare(a_path, b_path):
    a, b = np.load(a_path), np.load(b_path)
    bad = 0
    for k in sorted(set(a.files) | set(b.files)):
        if k not in a.files or k not in b.files:
            print("%s: only in one file" % k)
            bad += 1
            continue
        x, y = a[k], b[k]
        same = x.shape == y.shape and x.dtype == y.dtype and x.tobytes() == y.tobytes()
        n = 0 if same else int(np.sum(x.view(np.uint8).reshape(x.shape[0], -1) !=
                                      y.view(np.uint8).reshape(y.shape[0], -1)))
        print("%s: %s" % (k, "bit-identical" if same else "DIFFERS (%d bytes)" % n))
        bad += not same
    print("%d of %d arrays differ" % (bad, len(set(a.files) | set(b.files))))
    return 1 if bad else 0


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    digest(sys.argv[1])
