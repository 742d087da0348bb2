#!/usr/bin/env python3
"""FP64 events (PEKF_EV_F64_EVENTS) against f32 events on the same streams: 16,384 generated phone
streams x 1,024 events tiled x64 = 1,048,576 filters (the shape of scripts/bench_aux.py's front-end
lines).  One JSON object on stdout; kernel times are HIP events on the launch stream (median of 3).

  live_f32       k_live, f32 events, FP64 records (round 5's default)
  live_ev64      k_live, FP64 events (the server's stod values), all-FP64 records
  frontend_f32   k_frontend, f32 events -> 40 B records
  frontend_ev64  k_frontend, FP64 events -> 80 B FP64 records
  run64_after    k_run64 over frontend_ev64's records (the FP64 split pipeline's second half)
  init_f32 / init_ev64   k_frontend_init, means only

PEKF_LIB selects the library (A/B of build variants); PEKF_EV64_ONLY=live skips the split pipeline."""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poseestimationkf_amd import engine, synth, wire  # noqa: E402
from poseestimationkf_amd._lib import EV_F64_EVENTS, check, lib  # noqa: E402

HBM = 8000.0


def log(m):
    print("[ev64] " + m, file=sys.stderr, flush=True)


def timed(fn, stream, reps=3):
    e0, e1 = engine.Event(), engine.Event()
    fn()
    check(lib.pekf_stream_sync(stream))
    out = []
    for _ in range(reps):
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.sync()
        out.append(e0.elapsed_ms(e1))
    return float(np.median(out))


def main():
    st = engine.Stream()
    s = st.handle
    K0, E, tile = int(os.environ.get("PEKF_EV64_K0", 16384)), 1024, 64
    cache = os.environ.get("PEKF_EV64_CACHE")   # the generated streams, shared by the runs of an A/B
    if cache and os.path.exists(cache):
        with np.load(cache) as z:
            ev = {k: z[k] for k in z.files}
    else:
        log("generating %d x %d events" % (K0, E))
        ev = synth.generate_events(np.arange(K0), E, seed=11)
        if cache:
            np.savez(cache, **ev)
    K = K0 * tile
    init = np.tile(np.concatenate([ev["init_acc"], ev["init_mag"]], axis=1), (tile, 1))
    tinit = np.tile(ev["t_init"], tile).astype(np.int64)
    ib = engine.DeviceBuffer(init.nbytes).upload(init)
    tb = engine.DeviceBuffer(tinit.nbytes).upload(tinit)
    res = {"filters": K, "events_per_filter": E}

    def upload(planes):
        big = np.ascontiguousarray(np.tile(planes, (1, tile, 1)))
        return engine.DeviceBuffer(big.nbytes).upload(big)

    ev32 = upload(synth.pack_events(ev))
    ev64 = upload(synth.pack_events64(ev, wire.server_values(ev["values"])))
    cnt, refs = engine.DeviceBuffer(4 * K), engine.DeviceBuffer(48 * K)

    counts = {}
    for name, evb, flags in (("live_f32", ev32, 0), ("live_ev64", ev64, EV_F64_EVENTS)):
        f = engine.BatchedEKF(K)
        ms = timed(lambda: f.run_events_async(evb, E, ib, tb, cnt, refs, 0.1, s, flags=flags), s)
        counts[name] = cnt.download((K,), np.int32)
        byts = K * E * (32 if flags else 16) + K * (160 + 160 + 48 + 48 + 8 + 4)
        res[name] = {"kernel_ms": ms, "events_per_s": K * E / (ms * 1e-3), "records": int(counts[name].sum()),
                     "bytes": byts, "gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
        log("%s: %.3f ms" % (name, ms))
        del f
    assert np.array_equal(counts["live_f32"], counts["live_ev64"])
    res["live_ev64_vs_f32"] = res["live_ev64"]["kernel_ms"] / res["live_f32"]["kernel_ms"]
    log("live: FP64 events / f32 events = %.4f" % res["live_ev64_vs_f32"])
    if os.environ.get("PEKF_EV64_ONLY") == "live":
        print(json.dumps(res))
        return

    recs = int(counts["live_f32"].sum())
    r_max = E // 3 + 1
    err = engine.DeviceBuffer(4).upload(np.zeros(1, np.int32))
    win = engine.IMUWindow(K, r_max)
    ms = timed(lambda: check(lib.pekf_frontend_ext_dev(K, E, ev32.ptr, ib.ptr, tb.ptr, 0.1, r_max, win.gd.ptr,
                                                       win.am.ptr, win.my.ptr, None, cnt.ptr, win.refs.ptr, 0,
                                                       err.ptr, s)), s)
    byts = K * E * 16 + recs * 40
    res["frontend_f32"] = {"kernel_ms": ms, "bytes": byts, "gbs": byts / (ms * 1e-3) / 1e9,
                           "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
    log("frontend_f32: %.3f ms" % ms)
    del win
    w64 = engine.RecordWindow64(K, r_max)
    ms = timed(lambda: check(lib.pekf_frontend_ext_dev(K, E, ev64.ptr, ib.ptr, tb.ptr, 0.1, r_max, w64.gd.ptr,
                                                       w64.am.ptr, w64.my.ptr, None, cnt.ptr, w64.refs.ptr,
                                                       EV_F64_EVENTS, err.ptr, s)), s)
    assert np.array_equal(cnt.download((K,), np.int32), counts["live_f32"])
    byts = K * E * 32 + recs * 80
    res["frontend_ev64"] = {"kernel_ms": ms, "bytes": byts, "gbs": byts / (ms * 1e-3) / 1e9,
                            "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
    log("frontend_ev64: %.3f ms" % ms)
    f = engine.BatchedEKF(K)
    n_rec = int(counts["live_f32"].max())
    ms = timed(lambda: check(lib.pekf_run_rec64_dev(K, n_rec, r_max, 0, w64.gd.ptr, w64.am.ptr, w64.my.ptr,
                                                    w64.refs.ptr, f.X.ptr, f.P.ptr, 1.0, 0.1, None, cnt.ptr, s)), s)
    res["run64_after"] = {"kernel_ms": ms, "records": recs}
    res["split_ev64_ms"] = res["frontend_ev64"]["kernel_ms"] + ms
    log("run64 over those records: %.3f ms" % ms)
    del f, w64
    ib2, tb2, rb2 = (engine.DeviceBuffer(k * K) for k in (48, 8, 4))
    for name, evb, flags in (("init_f32", ev32, 0), ("init_ev64", ev64, EV_F64_EVENTS)):
        ms = timed(lambda: check(lib.pekf_frontend_init_ext_dev(K, E, evb.ptr, tb.ptr, 100, ib2.ptr, tb2.ptr, None,
                                                                rb2.ptr, flags, s)), s)
        byts = K * E * (32 if flags else 16)
        res[name] = {"kernel_ms": ms, "gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
        log("%s: %.3f ms" % (name, ms))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
