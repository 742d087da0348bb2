"""Randomised launch shapes against the C oracle (scripts/fuzz_gpu.py): batches of 1-300 filters,
windows of 1-48 rows wrapped, runs cut into one-record and multi-record launches, per-launch counts,
trajectories, AoS / SoA state, FP64 / mixed precision, the batched engine and the native handle,
random initial states, escaped dts and missing magnetometer samples.  The sweep is seeded, so a
failure names a reproducible case; the GPU box runs longer sweeps of the same script
(profiles/r3/fuzz/).  scripts/fuzz_live.py does the same for the fused front-end + filter kernel, which
must equal the split pipeline bit for bit (and its records the front-end restatement's), and
scripts/fuzz_percall.py the per-call operators item by item against the NumPy restatement."""
from __future__ import annotations

import importlib.util
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fuzz(name="fuzz_gpu"):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "scripts", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_fuzz_cases_cover_the_launch_shapes(oracle_c):
    """CPU: the case generator reaches every launch shape, and the expectation for a single full
    launch is the oracle's whole-window run."""
    fz = _fuzz()
    rng = np.random.default_rng(3)
    seen = set()
    for _ in range(60):
        c = fz.draw_case(rng)
        for _, L, counts, want in c["launches"]:
            seen.add(("one" if L == 1 else "multi", counts is not None, want))
        seen.add((c["layout"], c["precision"], c["handle"], c["rec"].dtx is not None))
        if len(c["launches"]) == 1 and c["launches"][0][2] is None and c["K"] <= 40:
            s, L, _, _ = c["launches"][0]
            X, P, _ = fz.expected(c)
            Xo, Po, _ = oracle_c.run(c["rec"], n_steps=L, step0=s, q=c["q"], r=c["r"], X=c["X0"], P=c["P0"])
            assert np.array_equal(X, Xo) and np.array_equal(P, Po)
    for shape in ("one", "multi"):
        for cn in (False, True):
            for tr in (False, True):
                assert (shape, cn, tr) in seen
    assert any(k[0] == "soa" for k in seen if len(k) == 4) and any(k[1] == "mixed" for k in seen if len(k) == 4)
    assert any(k[2] is True for k in seen if len(k) == 4) and any(k[3] is True for k in seen if len(k) == 4)


@pytest.mark.gpu
def test_random_launch_shapes_vs_oracle(oracle_c):
    assert _fuzz().main(["--cases", "40", "--seed", "7"]) == 0


@pytest.mark.gpu
def test_random_event_streams_live_equals_split():
    assert _fuzz("fuzz_live").main(["--cases", "20", "--seed", "7"]) == 0


@pytest.mark.gpu
def test_random_percall_items_vs_numpy_restatement(oracle_c):
    assert _fuzz("fuzz_percall").main(["--cases", "3", "--seed", "7"]) == 0
