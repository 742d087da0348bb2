#!/usr/bin/env python3
"""The wire on the device at scale: pekf_wire_events_dev on 262,144 phones x 1,024 frames (26.8 GB of
client text, 1,024 generated phones' phase-3 streams tiled x256), then the device session
(engine.run_wire_session: frames -> FP64 events -> phase 2 -> k_live) on a smaller set.  Prints one JSON
line: kernel ms (HIP events, median of reps), frames/s, GB/s of frames read + events written.

usage: python3 scripts/wire_probe.py [reps] [--session] [--tile T (phones = 1,024 T; default 256)] [--drift D] [--phones K (at most 1,024 T)] [--rows] [--no-check]
"""
from __future__ import annotations

import json
import os
import sys
import time
import types

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from poseestimationkf_amd import engine, synth, wire  # noqa: E402
from poseestimationkf_amd._lib import check, lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5
    tile = int(sys.argv[sys.argv.index("--tile") + 1]) if "--tile" in sys.argv else 256
    K0, E = 1024, 1024
    t0 = time.time()
    ev = synth.generate_events(np.arange(K0), E, seed=5)
    texts = [wire.events_text(ev["types"][:, k], ev["values"][:, k], ev["times"][:, k]) for k in range(K0)]
    drift = int(sys.argv[sys.argv.index("--drift") + 1]) if "--drift" in sys.argv else 0
    if drift:  # up to `drift` blank frames at random places in each phone's stream: its rows drift apart
        rng = np.random.default_rng(6)
        for k in range(K0):
            rows = [texts[k][i:i + 100] for i in range(0, len(texts[k]), 100)]
            for _ in range(int(rng.integers(0, drift + 1))):
                rows.insert(int(rng.integers(0, len(rows) + 1)), " " * 99 + "\n")
            texts[k] = "".join(rows)
    fr0 = wire.frames(texts)                                   # [F][K0][100]
    fr = np.ascontiguousarray(np.tile(fr0, (1, tile, 1)))       # [E][K0 * tile][100]
    if "--phones" in sys.argv:  # any batch (e.g. one whose row pitch, 32 B x phones, is no power of two)
        fr = np.ascontiguousarray(fr[:, :int(sys.argv[sys.argv.index("--phones") + 1])])
    gen_s = time.time() - t0
    F, K = fr.shape[:2]
    fb = engine.DeviceBuffer(fr.nbytes).upload(fr)
    del fr
    rows = "--rows" in sys.argv  # PEKF_WIRE_FRAME_ROWS: a row per frame index in both planes
    ev2 = engine.DeviceBuffer(32 * F * K if rows else 32)
    ev3 = engine.DeviceBuffer(32 * (F if rows else E) * K)  # E phase-3 messages per phone
    t2b, n2b, n3b, badb = (engine.DeviceBuffer(8 * K), engine.DeviceBuffer(4 * K), engine.DeviceBuffer(4 * K),
                           engine.DeviceBuffer(4 * K))
    errb = engine.DeviceBuffer(4).upload(np.zeros(1, np.int32))
    st = engine.Stream()
    e0, e1 = engine.Event(), engine.Event()
    ms = []
    for _ in range(reps):
        e0.record(st.handle)
        check(lib.pekf_wire_events_ext_dev(K, F, fb.ptr, F if rows else 0, F if rows else E, ev2.ptr, ev3.ptr,
                                           t2b.ptr, n2b.ptr, n3b.ptr, badb.ptr, errb.ptr, None, 1 if rows else 0,
                                           st.handle))
        e1.record(st.handle)
        e1.sync()
        ms.append(e0.elapsed_ms(e1))
    check_out = "--no-check" not in sys.argv  # (timing-only builds of experiments)
    assert not check_out or int(errb.download((1,), np.int32)[0]) == 0
    n3 = n3b.download((K,), np.int32) if check_out else np.full(K, E)
    assert np.all(n3 == E)
    # spot check against the host parse: phone 0 and a tiled copy of it
    got = ev3.download((F if rows else E, K, 4), np.float64)[:, [0, K0 * 7]]
    if rows:  # the rows that are not the no-message event (one phone's and its copy's: the same frames)
        keep = got[:, 0, 3:4].view(np.uint64)[:, 0] != np.uint64(synth.EV64_NONE_W)
        got = got[keep]
    want = synth.pack_events64(wire.events_from_wire(texts[:1], np.zeros((1, 3)), np.zeros((1, 3)), [0]))
    assert not check_out or np.array_equal(got[:, 0].view(np.uint64), want[:, 0].view(np.uint64))
    assert not check_out or np.array_equal(got[:, 1].view(np.uint64), want[:, 0].view(np.uint64))
    med = float(np.median(ms[1:] if len(ms) > 1 else ms))
    frames = F * K
    byts = frames * 100 + (2 * F if rows else E) * K * 32
    print(json.dumps(dict(kernel="k_wire_events", phones=K, frames_per_phone=F, drift=drift, frame_rows=rows,
                          kernel_ms=med, ms=ms,
                          frames_per_s=frames / med * 1e3, gbs=byts / med / 1e6, hbm_frac=byts / med / 1e6 / 8000,
                          bytes_per_frame="100 read + 32 written per message", text_gen_s=gen_s)))


def session(reps):
    """frames -> FP64 events -> phase 2 -> phase 3 + filter on the device (engine.run_wire_session's
    launches, each timed): 65,536 phones x (700 phase-2 + 1,024 phase-3 frames), 1,024 generated phones
    tiled x64."""
    K0, tile, E2, E3 = 1024, 64, 700, 1024
    ph2 = synth.generate_events(np.arange(K0), E2, seed=71)
    ph3 = synth.generate_events(np.arange(K0), E3, seed=72)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    # --drift D: phase-2 parts of E2 - (0..D) messages, so that the phones' phase-3 rows drift apart
    drift = int(sys.argv[sys.argv.index("--drift") + 1]) if "--drift" in sys.argv else 0
    n2k = E2 - np.random.default_rng(8).integers(0, drift + 1, K0)
    texts = [wire.events_text(ph2["types"][:n2k[k], k], ph2["values"][:n2k[k], k], ph2["times"][:n2k[k], k],
                              phase=2) +
             wire.events_text(ph3["types"][:, k], ph3["values"][:, k], ph3["times"][:, k], phase=3)
             for k in range(K0)]
    rows_mode = "--rows" in sys.argv
    fr = np.ascontiguousarray(np.tile(wire.frames(texts), (1, tile, 1)))
    F, K = fr.shape[:2]
    fb = engine.DeviceBuffer(fr.nbytes).upload(fr)
    del fr
    from poseestimationkf_amd._lib import EV_F64_EVENTS
    ev2, ev3 = engine.DeviceBuffer(32 * F * K), engine.DeviceBuffer(32 * F * K)
    t2b, n2b, n3b = engine.DeviceBuffer(8 * K), engine.DeviceBuffer(4 * K), engine.DeviceBuffer(4 * K)
    errb = engine.DeviceBuffer(4).upload(np.zeros(1, np.int32))
    ib, tib, rb = engine.DeviceBuffer(48 * K), engine.DeviceBuffer(8 * K), engine.DeviceBuffer(4 * K)
    cnt, refs = engine.DeviceBuffer(4 * K), engine.DeviceBuffer(48 * K)
    f = engine.BatchedEKF(K)
    bounds = engine.DeviceBuffer(8)
    st = engine.Stream()
    ev = [engine.Event() for _ in range(5)]
    rows = []
    for _ in range(reps):
        f.reset()
        ev[0].record(st.handle)
        check(lib.pekf_wire_events_ext_dev(K, F, fb.ptr, F, F, ev2.ptr, ev3.ptr, t2b.ptr, n2b.ptr, n3b.ptr, None,
                                           errb.ptr, bounds.ptr if rows_mode else None, 1 if rows_mode else 0,
                                           st.handle))
        ev[1].record(st.handle)
        if rows_mode:  # (engine.run_wire_session reads the bounds the same way: one small copy, not timed)
            r2, r3 = (int(v) for v in bounds.download((2,), np.int32, st.handle))
        ev[4].record(st.handle)
        check(lib.pekf_frontend_init_ext_dev(K, r2 if rows_mode else E2, ev2.ptr, t2b.ptr, 100, ib.ptr, tib.ptr, None,
                                             rb.ptr, EV_F64_EVENTS, st.handle))
        ev[2].record(st.handle)
        ev3v = types.SimpleNamespace(ptr=ev3.ptr + 32 * K * (F - r3)) if rows_mode else ev3
        f.run_events_async(ev3v, r3 if rows_mode else E3, ib, tib, cnt, refs, 0.1, st.handle, flags=EV_F64_EVENTS)
        ev[3].record(st.handle)
        ev[3].sync()
        rows.append([ev[0].elapsed_ms(ev[1]), ev[4].elapsed_ms(ev[2]), ev[2].elapsed_ms(ev[3])])
    assert int(errb.download((1,), np.int32)[0]) == 0
    assert np.array_equal(n2b.download((K,), np.int32), np.tile(n2k, tile)) and np.all(n3b.download((K,), np.int32) == E3)
    assert rb.download((K,), np.int32).all()
    med = np.median(np.array(rows[1:] if len(rows) > 1 else rows), axis=0)
    print(json.dumps(dict(kernel="wire session", phones=K, frames_per_phone=F, drift=drift, frame_rows=rows_mode,
                          wire_ms=float(med[0]),
                          phase2_ms=float(med[1]), live_ms=float(med[2]), total_ms=float(med.sum()),
                          messages_per_s=K * F / float(med.sum()) * 1e3,
                          records=int(cnt.download((K,), np.int32).sum()))))


if __name__ == "__main__":
    if "--session" in sys.argv:
        session(int(sys.argv[1]) if sys.argv[1:2] and sys.argv[1].isdigit() else 5)
    else:
        main()
