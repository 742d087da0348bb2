#!/usr/bin/env python3
"""How far apart are the record rows of a wave's 64 lanes?  k_frontend stores each lane's r-th record
in row r of the [record][filter] window, so the store instructions of a wave coalesce only as far as
its lanes sit on the same row.  Per wave of the probe's event streams (synth.generate_events, seed
11, as scripts/frontend_probe.py), this prints the spread (max - min record count) over the events and
the distribution of |r - median| across lanes and events, using scripts/live_queue_sim.py's model of
the Parser state machine's record completions.

    python scripts/record_drift.py [--filters 2048] [--events 1024]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from poseestimationkf_amd import synth  # noqa: E402
from live_queue_sim import completions  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=2048)
    ap.add_argument("--events", type=int, default=1024)
    a = ap.parse_args()
    ev = synth.generate_events(np.arange(a.filters), a.events, seed=11)
    cum = np.cumsum(completions(ev["types"]), 0)
    print("records per filter: %.1f over %d events" % (cum[-1].mean(), a.events))
    spread, dev = [], []
    for w in range(a.filters // 64):
        c = cum[:, 64 * w:64 * w + 64]
        spread.append(c.max(1) - c.min(1))
        dev.append(np.abs(c - np.median(c, 1)[:, None]).ravel())
    spread, dev = np.concatenate(spread), np.concatenate(dev)
    print("rows between a wave's first and last lane: mean %.1f, max %d" % (spread.mean(), spread.max()))
    print("|row - wave median| p50 / p90 / p99: %.1f / %.1f / %.1f" % tuple(np.percentile(dev, [50, 90, 99])))


if __name__ == "__main__":
    main()
