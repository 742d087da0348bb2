#!/usr/bin/env python3
"""The FP64-record launch (pekf_run_rec64_dev) against the 40 B-record launch (pekf_run_dev) on the same
values at scale: 1,048,576 filters x 10,000 records over a 128-record resident window (10.7 GB of FP64
records, 5.4 GB of 40 B records: both far beyond the Infinity Cache).  The window is generated on the
device (Philox), widened to FP64 on the host, and both launches are timed with HIP events in ABAB order;
the final states must be bit-identical.

usage: python3 scripts/rec64_probe.py [--batch B] [--records N] [--window W] [--rounds R]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poseestimationkf_amd import engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--records", type=int, default=10000)
    ap.add_argument("--window", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    K, W = a.batch, a.window
    w32 = engine.IMUWindow(K, W).synthesize(seed=synth.DEFAULT_SEED)
    w64 = engine.RecordWindow64(K, W)
    for r0 in range(0, W, 16):   # widen 16 rows at a time (host memory)
        r1 = min(W, r0 + 16)
        n = (r1 - r0) * K
        gd = np.empty((r1 - r0, K, 4), np.float32)
        am = np.empty((r1 - r0, K, 4), np.float32)
        my = np.empty((r1 - r0, K, 2), np.float32)
        engine.check(engine.lib.pekf_memcpy_d2h(gd.ctypes.data, w32.gd.ptr + 16 * r0 * K, 16 * n, None))
        engine.check(engine.lib.pekf_memcpy_d2h(am.ctypes.data, w32.am.ptr + 16 * r0 * K, 16 * n, None))
        engine.check(engine.lib.pekf_memcpy_d2h(my.ctypes.data, w32.my.ptr + 8 * r0 * K, 8 * n, None))
        g64 = gd.astype(np.float64)
        g64[..., 3] = (gd[..., 3].view(np.uint32) & np.uint32(synth.DT_MASK)).astype(np.float64)
        for dst, src in ((w64.gd.ptr + 32 * r0 * K, g64), (w64.am.ptr + 32 * r0 * K, am.astype(np.float64)),
                         (w64.my.ptr + 16 * r0 * K, my.astype(np.float64))):
            src = np.ascontiguousarray(src)
            engine.check(engine.lib.pekf_memcpy_h2d(dst, src.ctypes.data, src.nbytes, None))
    engine.check(engine.lib.pekf_memcpy_d2d(w64.refs.ptr, w32.refs.ptr, 48 * K, None))
    engine.check(engine.lib.pekf_device_sync())
    st = engine.Stream()
    s = st.handle
    e0, e1 = engine.Event(), engine.Event()
    f = {"f32": engine.BatchedEKF(K), "f64": engine.BatchedEKF(K)}
    t = {"f32": [], "f64": []}
    for rnd in range(a.rounds + 1):
        for name, win in (("f32", w32), ("f64", w64)):
            f[name].reset(s)
            e0.record(s)
            f[name].run_async(win, a.records, 0, s)
            e1.record(s)
            e1.sync()
            if rnd:
                t[name].append(e0.elapsed_ms(e1))
    X32, P32 = f["f32"].get_state()
    X64, P64 = f["f64"].get_state()
    same = np.array_equal(X32, X64) and np.array_equal(P32, P64)
    for name, bpr in (("f32", 40), ("f64", 80)):
        ms = float(np.median(t[name]))
        print("%s records: %d filters x %d records: %.3f ms median (%s), %.3g steps/s, %.0f GB/s of records"
              % (name, K, a.records, ms, ", ".join("%.2f" % v for v in t[name]), K * a.records / ms * 1e3,
                 K * a.records * bpr / ms / 1e6))
    print("final states bit-identical: %s" % same)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
