#!/usr/bin/env python3
"""When should the fused front-end + filter kernel (csrc/pekf_live.hip) run a filter step?

A wave of 64 filters walks its event streams in blocks of RING events; lanes complete records at
different events.  Each lane queues up to Q records; at a block's end the wave runs filter steps (one
queued record for every lane that has one) while some lane could overflow within the next block
(queue > Q - RING/3), then one more if at least QUORUM lanes have a record queued; after the last
event it drains.  This simulates that policy on synth.generate_events streams (the record timing
depends only on the event types) and prints, per setting, the filter steps per wave and the fraction
of lanes busy in them (records / (steps x 64)) -- the filter's SIMD efficiency.

    python scripts/live_queue_sim.py [--filters 2048] [--events 1024]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poseestimationkf_amd import synth  # noqa: E402


def completions(types):
    """(E, K) bool: event e completes a record of filter k (Parser.cpp:148-219's state machine)."""
    E, K = types.shape
    gs, a1, m1 = (np.zeros(K, bool) for _ in range(3))
    out = np.zeros((E, K), bool)
    for e in range(E):
        t = types[e]
        isA, isM, isG = t == synth.EV_ACC, t == synth.EV_MAG, t == synth.EV_GYRO
        a1s = (isA & gs) | (a1 & ~(isG & gs))
        m1s = (isM & gs) | (m1 & ~(isG & gs))
        done = a1s & m1s
        out[e] = done
        gs, a1, m1 = (gs | isG) & ~done, a1s & ~done, m1s & ~done
    return out


def simulate(done, ring, q, quorum):
    E, K = done.shape
    push = ring // 3
    steps = recs = 0
    for w in range(K // 64):
        d = done[:, 64 * w:64 * w + 64]
        n = np.zeros(64, int)
        for e0 in range(0, E, ring):
            n += d[e0:e0 + ring].sum(0)
            assert n.max() <= q
            last = e0 + ring >= E
            while (n > 0).any():
                if not (last or (n > q - push).any() or (n > 0).sum() >= quorum):
                    break
                steps += 1
                recs += int((n > 0).sum())
                n = np.maximum(n - 1, 0)
    waves = K // 64
    return steps / waves, recs / (steps * 64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=2048)
    ap.add_argument("--events", type=int, default=1024)
    a = ap.parse_args()
    ev = synth.generate_events(np.arange(a.filters), a.events, seed=3)
    done = completions(ev["types"])
    print("records per filter: %.1f over %d events" % (done.sum(0).mean(), a.events))
    print("ring queue quorum  steps/wave  lanes busy")
    for ring in (3, 6, 9):
        for q in range(ring // 3, ring // 3 + 4):
            for quorum in (1, 32, 48, 56):
                s, eff = simulate(done, ring, q, quorum)
                print("%4d %5d %6d  %10.1f  %10.3f" % (ring, q, quorum, s, eff))


if __name__ == "__main__":
    main()
