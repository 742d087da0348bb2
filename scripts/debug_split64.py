#!/usr/bin/env python3
"""Debug: FP64-event k_live against the FP64 split pipeline (k_frontend FP64 records -> k_run64)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poseestimationkf_amd import engine, synth  # noqa: E402


def main():
    for K, E, seed in ((64, 37, 42), (512, 200, 43), (1000, 1500, 41)):
        ev = synth.generate_events(np.arange(K), E, seed=seed)
        f = engine.BatchedEKF(K)
        c1, r1 = f.run_events(ev, records="f64", events="f64")
        X1, P1 = f.get_state()
        win, c2 = engine.run_frontend(ev, events="f64")
        g = engine.BatchedEKF(K)
        g.run(win, n_steps=max(2, int(c2.max())))
        X2, P2 = g.get_state()
        # the same through f32 events: k_live R64 (FP64 records) vs itself re-run (determinism)
        d = np.abs(X1 - X2).max(axis=1)
        print("K=%d E=%d: counts equal %s, refs equal %s, X max diff %.3e, filters differing %d, P max diff %.3e"
              % (K, E, np.array_equal(c1, c2), np.array_equal(r1, win.refs.download((K, 6), np.float64)),
                 d.max(), int((d > 0).sum()), np.abs(P1 - P2).max()), flush=True)
        bad = np.nonzero(d > 0)[0][:5]
        print("   first differing filters", bad.tolist(), "their counts", c1[bad].tolist(), flush=True)


if __name__ == "__main__":
    main()
