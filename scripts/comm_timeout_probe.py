#!/usr/bin/env python3
"""Probe of the RCCL init deadline (include/pekf.h pekf_comm_init_timeout): rank 0 of a 2-rank
communicator whose rank 1 never comes; prints the time the call returns and its error."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poseestimationkf_amd import engine, shard  # noqa: E402
from poseestimationkf_amd._lib import PekfError  # noqa: E402

engine.set_device(0)
uid = shard.Communicator.unique_id()
t0 = time.monotonic()
print("probe: init start (PEKF_COMM_TIMEOUT_S=%s)" % os.environ.get("PEKF_COMM_TIMEOUT_S"), flush=True)
try:
    shard.Communicator(uid, 2, 0)
    print("probe: init returned ok?!", flush=True)
except PekfError as e:
    print("probe: init raised after %.1f s: %s" % (time.monotonic() - t0, e), flush=True)
