#!/usr/bin/env python3
"""The front-end kernel alone (the bench_aux.py workload: 16K generated event streams tiled x64 ->
1,048,576 filters x 1,024 events), for rocprofv3 PMC passes that should see only k_frontend; with
--live the fused front-end + filter kernel (pekf_live_dev) on the same events instead, with --init
phase 2 (pekf_frontend_init_dev, the means / variances of the first 100 samples; --init-means: the
means alone, no stats, as engine.run_session calls it).

usage: python3 scripts/frontend_probe.py [reps] [--live [--f64 | --f32] | --init | --init-means] [--ev64]
(--live: the records' acc / mag in FP64, the default, or as f32 stream records with --f32; --ev64: FP64
events -- the server's stod values, PEKF_EV_F64_EVENTS -- instead of f32 ones.  PEKF_EV64_CACHE names an
.npz that keeps the generated streams between runs.)
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poseestimationkf_amd import engine, synth, wire  # noqa: E402
from poseestimationkf_amd._lib import EV_F32_RECORDS, EV_F64_EVENTS, check, lib  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    live = "--live" in sys.argv
    rec_flags = EV_F32_RECORDS if "--f32" in sys.argv else 0
    means_only = "--init-means" in sys.argv
    phase2 = "--init" in sys.argv or means_only
    reps = int(args[0]) if args else 3
    st = engine.Stream()
    s = st.handle
    ev64 = "--ev64" in sys.argv
    ev_flags = EV_F64_EVENTS if ev64 else 0
    if ev64:
        rec_flags = 0
    K0, E, tile = 16384, 1024, 64
    cache = os.environ.get("PEKF_EV64_CACHE")
    if cache and os.path.exists(cache):
        with np.load(cache) as z:
            ev = {k: z[k] for k in z.files}
    else:
        ev = synth.generate_events(np.arange(K0), E, seed=11)
        if cache:
            np.savez(cache, **ev)
    packed = synth.pack_events64(ev, wire.server_values(ev["values"])) if ev64 else synth.pack_events(ev)
    planes = np.ascontiguousarray(np.tile(packed, (1, tile, 1)))
    del packed
    K = K0 * tile
    init = np.tile(np.concatenate([ev["init_acc"], ev["init_mag"]], axis=1), (tile, 1))
    tinit = np.tile(ev["t_init"], tile)
    evb = engine.DeviceBuffer(planes.nbytes).upload(planes)
    ib = engine.DeviceBuffer(init.nbytes).upload(init)
    tb = engine.DeviceBuffer(tinit.nbytes).upload(tinit.astype(np.int64))
    r_max = E // 3 + 1
    win = (engine.RecordWindow64 if ev64 else engine.IMUWindow)(K, 1 if live else r_max)
    cnt = engine.DeviceBuffer(4 * K)
    err = engine.DeviceBuffer(4).upload(np.zeros(1, np.int32))
    e0, e1 = engine.Event(), engine.Event()
    times = []
    f = engine.BatchedEKF(K) if live else None
    if phase2:
        ob, tob, rb = engine.DeviceBuffer(48 * K), engine.DeviceBuffer(8 * K), engine.DeviceBuffer(4 * K)
        sb = engine.DeviceBuffer(96 * K)
    for _ in range(reps):
        e0.record(s)
        if phase2:
            check(lib.pekf_frontend_init_ext_dev(K, E, evb.ptr, tb.ptr, 100, ob.ptr, tob.ptr,
                                                 None if means_only else sb.ptr, rb.ptr, ev_flags, s))
        elif live:
            f.run_events_async(evb, E, ib, tb, cnt, win.refs, 0.1, s, flags=rec_flags | ev_flags)
        else:
            check(lib.pekf_frontend_ext_dev(K, E, evb.ptr, ib.ptr, tb.ptr, 0.1, r_max, win.gd.ptr, win.am.ptr,
                                            win.my.ptr, None, cnt.ptr, win.refs.ptr, ev_flags, err.ptr, s))
        e1.record(s)
        e1.sync()
        times.append(e0.elapsed_ms(e1))
    if phase2:
        ready = int(rb.download((K,), np.int32).sum())
        src = ob.download((K, 6), np.float64) if means_only else sb.download((K, 12), np.float64)
        digest = float(np.nansum(src)) + float(tob.download((K,), np.int64).astype(np.float64).sum())
        print("frontend_probe %s: %d filters x %d events, %d ready, %s digest %.17g, ms %s"
              % ("--init-means" if means_only else "--init", K, E, ready, "means" if means_only else "stats",
                 digest, ["%.3f" % t for t in times]))
        return
    recs = int(cnt.download((K,), np.int32).sum())
    digest = ""
    if live:
        X, _ = f.get_state()
        digest = " X digest %.17g" % float(np.sum(X * np.arange(1, 5)))
    print("frontend_probe%s: %d filters x %d events, %d records,%s ms %s"
          % (" --live" + (" --f32" if rec_flags else " (f64 records)") if live else "", K, E, recs, digest,
             ["%.3f" % t for t in times]))


if __name__ == "__main__":
    main()
