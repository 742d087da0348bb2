#!/usr/bin/env python3
"""Debug: FP64 events across long / negative gaps -- which path departs from the oracle chain?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poseestimationkf_amd import engine, synth, wire  # noqa: E402
from oracle import ekf_numpy, frontend_numpy as fe  # noqa: E402
from tests.test_frontend import _events  # noqa: E402


def oracle(ev, k, refs, X0, P0, server):
    vals = wire.server_values(ev["values"][:, k]) if server else ev["values"][:, k].astype(np.float64)
    g, dt, a, m = fe.run_frontend(ev["types"][:, k], vals, ev["times"][:, k], ev["init_acc"][k], ev["init_mag"][k],
                                  ev["t_init"][k])
    X, _, _ = ekf_numpy.run_filter(g, dt.astype(np.float64), a, m, refs[k, :3], refs[k, 3:], X0=X0, P0=P0,
                                   record=False)
    return X


def main():
    K = 64
    g = (1 << 31) + 12345
    specs = {
        "full": [(synth.EV_GYRO, 1000), (synth.EV_ACC, g), (synth.EV_MAG, 10), (synth.EV_GYRO, -5_000_000),
                 (synth.EV_ACC, 700), (synth.EV_MAG, 0), (synth.EV_GYRO, 3 * g), (synth.EV_ACC, 10),
                 (synth.EV_MAG, 10)] * 4,
        "short_gaps_negative": [(synth.EV_GYRO, 1000), (synth.EV_ACC, 2000), (synth.EV_MAG, 10),
                                (synth.EV_GYRO, -5_000), (synth.EV_ACC, 700), (synth.EV_MAG, 0)] * 4,
        "long_gaps_only": [(synth.EV_GYRO, 1000), (synth.EV_ACC, g), (synth.EV_MAG, 10)] * 6,
        "medium": [(synth.EV_GYRO, 1_000_000), (synth.EV_ACC, 2_000_000), (synth.EV_MAG, 1_000_000)] * 12,
    }
    rng = np.random.default_rng(44)
    X0 = rng.standard_normal((K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.tile(np.eye(4) * 0.4, (K, 1, 1))
    for name, spec in specs.items():
        ev = _events(K, spec)
        out = {}
        for tag, kw in (("live_ev64", dict(records="f64", events="f64")), ("live_f32ev_r64", dict(records="f64")),
                        ("live_f32ev_r32", dict(records="f32"))):
            f = engine.BatchedEKF(K)
            f.set_state(X0, P0)
            c, refs = f.run_events(ev, **kw)
            out[tag] = (f.get_state()[0], c, refs)
        win, c = engine.run_frontend(ev, events="f64")
        f = engine.BatchedEKF(K)
        f.set_state(X0, P0)
        f.run(win, n_steps=max(2, int(c.max())))
        out["split_ev64"] = (f.get_state()[0], c, win.refs.download((K, 6), np.float64))
        refs = out["live_ev64"][2]
        for tag, (X, c, r) in out.items():
            e_s = max(float(np.abs(X[k] - oracle(ev, k, refs, X0[k], P0[k], True)).max()) for k in range(0, K, 7))
            e_f = max(float(np.abs(X[k] - oracle(ev, k, refs, X0[k], P0[k], False)).max()) for k in range(0, K, 7))
            print("%-20s %-16s counts %s  vs server-value chain %.3e  vs f32-value chain %.3e"
                  % (name, tag, np.unique(c), e_s, e_f), flush=True)


if __name__ == "__main__":
    main()
