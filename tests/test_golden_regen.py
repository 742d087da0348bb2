"""The oracle's pin stays honest as the code evolves: the golden fixtures are regenerated from the
REFERENCE itself (tests/golden/make_golden.py, make_gaps_golden.py, make_lpf_golden.py import its
modules and run main_file.py / Test.py unchanged) into a scratch directory and compared with the
committed ones, array for array.  The fixtures depend on this repo's synth.generate (Philox streams)
and logformat.write_log, so a change to either that moved an input would show here, not as a silent
drift between the oracle's pin and the reference.

Runs only where /root/reference exists (the build container); it is absent on the GPU box, where the
committed fixtures are all the tests read."""
import gzip
import os
import subprocess
import sys

import numpy as np
import pytest

from .conftest import GOLDEN

REF_DIR = "/root/reference/Python Kalman Filter"

pytestmark = pytest.mark.skipif(not os.path.isdir(REF_DIR), reason="the reference is not present here")


def _regenerate(script, out):
    env = dict(os.environ, PEKF_GOLDEN_OUT=str(out), PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg")
    r = subprocess.run([sys.executable, os.path.join(GOLDEN, script)], cwd=str(out), env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


def _same_npz(name, out):
    with np.load(os.path.join(GOLDEN, name)) as a, np.load(os.path.join(out, name)) as b:
        assert sorted(a.files) == sorted(b.files), name
        for k in a.files:
            assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, (name, k)
            assert np.array_equal(a[k], b[k], equal_nan=True), (name, k)


def test_make_golden_regenerates_the_committed_fixtures(tmp_path):
    _regenerate("make_golden.py", tmp_path)
    for name in ("kat.npz", "traj.npz", "edge.npz", "side.npz"):
        _same_npz(name, tmp_path)
    with gzip.open(os.path.join(GOLDEN, "c1_log.txt.gz"), "rb") as a, \
            gzip.open(os.path.join(tmp_path, "c1_log.txt.gz"), "rb") as b:
        assert a.read() == b.read()
    xa, xb = np.load(os.path.join(GOLDEN, "c1_xk.npy")), np.load(os.path.join(tmp_path, "c1_xk.npy"))
    assert xa.dtype == xb.dtype and np.array_equal(xa, xb)


def test_make_gaps_and_lpf_golden_regenerate_the_committed_fixtures(tmp_path):
    _regenerate("make_gaps_golden.py", tmp_path)
    _same_npz("gaps.npz", tmp_path)
    _regenerate("make_lpf_golden.py", tmp_path)
    _same_npz("lpf_testpy.npz", tmp_path)


def test_regeneration_leaves_the_reference_untouched():
    """No bytecode or output was written under /root/reference (the scripts set dont_write_bytecode)."""
    for dirpath, dirnames, filenames in os.walk(REF_DIR):
        assert "__pycache__" not in dirnames, dirpath
