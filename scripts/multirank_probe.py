#!/usr/bin/env python3
"""Probe: can RCCL put two ranks of one communicator on the same GPU (ncclCommInitAll with devices
[0, 0])?  If it can, the one-process N-GPU path (MultiDeviceEKF, grouped gather) runs at N = 2 on a
one-GPU box.  Prints what happened."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from poseestimationkf_amd import engine, shard, synth  # noqa: E402
from poseestimationkf_amd._lib import PekfError  # noqa: E402

engine.set_device(0)
try:
    m = shard.MultiDeviceEKF([0, 0], 4096, 32).synthesize(seed=synth.DEFAULT_SEED)
except PekfError as e:
    print("probe: two ranks on one device refused: %s" % e, flush=True)
    sys.exit(0)
m.run_async(64, 0)
m.gather_async()
m.sync()
got = m.gathered()
m.close()
from oracle import oracle_c  # noqa: E402  (test infrastructure: the checker)
cols = np.array([0, 1, 4095, 4096, 4097, 8191])
Xo, _, _ = oracle_c.run(synth.generate(cols, 32), n_steps=64)
print("probe: two ranks on one device ran; gathered %s, max |dq| vs oracle %.3e" % (got.shape, np.abs(got[cols] - Xo).max()),
      flush=True)
