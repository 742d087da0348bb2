#!/usr/bin/env python3
"""Online serving alone (the bench_aux.py workload): 1,048,576 filters advanced by ONE record per
launch (pekf_run_dev, n_steps = 1) with AoS and SoA state, kernel time by HIP events; for A/B of
builds with PEKF_LIB=...

usage: python3 scripts/online_probe.py [reps]
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poseestimationkf_amd import engine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    st = engine.Stream()
    s = st.handle
    B = 1 << 20
    win = engine.IMUWindow(B, 8).synthesize(stream=s)
    e0, e1 = engine.Event(), engine.Event()
    out = []
    for layout in ("aos", "soa"):
        f = engine.BatchedEKF(B, layout=layout)
        for k in range(3):
            f.run_async(win, 1, k % 8, s)
        e0.record(s)
        for k in range(reps):
            f.run_async(win, 1, k % 8, s)
        e1.record(s)
        e1.sync()
        out.append("%s %.4f ms" % (layout, e0.elapsed_ms(e1) / reps))
        del f
    print("online_probe: 1M filters x 1 record per launch: " + ", ".join(out))


if __name__ == "__main__":
    main()
