"""Golden vectors for the front-end's low-pass stage, from the REFERENCE's own Test.py (run in the
survey container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_lpf_golden.py

`Python Kalman Filter/Test.py:1-35` reads a log with ReadFile.getData() and low-passes the Acc_1 /
Mag_1 samples with alpha = 0.1 from a zero state -- the same recurrence the C++ server applies in
its front-end (KFS/KalmanFilter.cpp:16-18,21-24,279-303), which oracle/frontend_numpy.py restates.
Test.py is run unchanged (matplotlib on the Agg backend, only its hard-coded log path redirected
to the config-1 log); its module globals after the run hold the filtered arrays.  Stored: the raw
samples (inputs) and Test.py's outputs.  No reference source is stored.

Output: tests/golden/lpf_testpy.npz
"""
from __future__ import annotations

import builtins
import gzip
import os
import runpy
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# where the fixtures are written (tests/test_golden_regen.py regenerates them into a scratch directory)
OUT = os.environ.get("PEKF_GOLDEN_OUT") or HERE
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_DIR = "/root/reference/Python Kalman Filter"
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

from poseestimationkf_amd import logformat  # noqa: E402


def main():
    with gzip.open(os.path.join(HERE, "c1_log.txt.gz"), "rt") as fh:
        text = fh.read()
    tmp = os.path.join("/tmp", "pekf_lpf_log.txt")
    with open(tmp, "w") as fh:
        fh.write(text)
    raw = logformat.read_log(tmp)
    acc_raw = np.asarray(raw.acc_1, np.float64)
    mag_raw = np.asarray(raw.mag_1, np.float64)
    real_open = builtins.open

    def redirect(path, *args, **kw):
        if path == logformat.REFERENCE_LOG_PATH:
            path = tmp
        return real_open(path, *args, **kw)

    os.environ["MPLBACKEND"] = "Agg"
    sys.path.insert(0, REF_DIR)
    builtins.open = redirect
    try:
        g = runpy.run_path(os.path.join(REF_DIR, "Test.py"), run_name="__main__")["g"]
    finally:
        builtins.open = real_open
    np.savez_compressed(os.path.join(OUT, "lpf_testpy.npz"), acc_raw=acc_raw, mag_raw=mag_raw,
                        acc_lpf=np.asarray(g.acc_1, np.float64), mag_lpf=np.asarray(g.mag_1, np.float64),
                        alpha=np.array([0.1]))
    print("lpf_testpy.npz", os.path.getsize(os.path.join(OUT, "lpf_testpy.npz")))


if __name__ == "__main__":
    main()
