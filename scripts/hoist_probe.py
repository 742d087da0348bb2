#!/usr/bin/env python3
"""In-process ABBA of k_run's HOIST schedule: PEKF_RUN_HOIST is read at every launch, so one process
alternates 0 / 1 over the same resident window (config 2: 65,536 filters x 10,000 records over a
1,024-record window; --batch for others) and prints each schedule's HIP-event kernel ms.

usage: python3 scripts/hoist_probe.py [--batch B] [--rounds R]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poseestimationkf_amd import engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--records", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    st = engine.Stream()
    s = st.handle
    win = engine.IMUWindow(a.batch, 1024).synthesize(seed=20261015, stream=s)
    f = engine.BatchedEKF(a.batch)
    e0, e1 = engine.Event(), engine.Event()

    def once(h):
        os.environ["PEKF_RUN_HOIST"] = h
        e0.record(s)
        f.run_async(win, a.records, 0, s)
        e1.record(s)
        e1.sync()
        return e0.elapsed_ms(e1)

    for h in "0101":
        once(h)   # warm-up
    t = {"0": [], "1": []}
    for _ in range(a.rounds):
        for h in "0110":
            t[h].append(once(h))
    for h in "01":
        v = np.array(t[h])
        print("batch %d hoist=%s: mean %.4f ms, median %.4f, min %.4f (n=%d)" % (a.batch, h, v.mean(), np.median(v),
                                                                            v.min(), v.size))
    m0, m1 = np.median(t["0"]), np.median(t["1"])
    print("batch %d: hoist/default = %.4f" % (a.batch, m1 / m0))


if __name__ == "__main__":
    main()
