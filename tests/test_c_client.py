"""The C ABI from a C++ caller (examples/c_client.cpp): the filter handle without Python.

The test writes one input file, runs the compiled client on the GPU (loaded as a shared library:
no process is started from the GPU-initialised test process) and runs the same sequence through
engine.FilterHandle; both go through the same entry points, so the results must agree bit for
bit.  The client builds (executable and library forms) are checked on CPU.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from poseestimationkf_amd import synth

from .conftest import ROOT

CLIENT_SRC = os.path.join(ROOT, "examples", "c_client.cpp")
WIRE_SRC = os.path.join(ROOT, "examples", "wire_client.cpp")
PREBUILT = os.path.join(ROOT, "examples", "build", "libc_client.so")
WIRE_PREBUILT = os.path.join(ROOT, "examples", "build", "libwire_client.so")


def _build(tmp_path, library, src=CLIENT_SRC):
    name = os.path.splitext(os.path.basename(src))[0]
    out = str(tmp_path / (("lib%s.so" % name) if library else name))
    pkg = os.path.join(ROOT, "poseestimationkf_amd")
    extra = ["-shared", "-fPIC", "-DPEKF_EXAMPLE_LIBRARY"] if library else []
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", *extra, src,
                           "-I" + os.path.join(ROOT, "include"), "-L" + pkg, "-lpekf", "-Wl,-rpath," + pkg, "-o", out])
    return out


@pytest.mark.parametrize("library", [False, True])
@pytest.mark.parametrize("src", [CLIENT_SRC, WIRE_SRC])
def test_c_client_builds(tmp_path, library, src):
    assert os.path.exists(_build(tmp_path, library, src))


@pytest.mark.gpu
def test_c_client_matches_python_engine(tmp_path):
    from poseestimationkf_amd import engine
    B, N, W = 7, 30, 12
    rec = synth.generate(np.arange(B), N + W, seed=23, missing=True)
    rng = np.random.default_rng(1)
    gyro = rec.gyro[:N].astype(np.float64) + rng.normal(scale=1e-9, size=(N, B, 3))   # FP64 records
    acc = rec.acc[:N].astype(np.float64)
    mag = rec.mag[:N].astype(np.float64)
    t = np.cumsum((rec.dtw[:N] & 0x7FFFFFFF).astype(np.int64), axis=0)
    tail = synth.Records(rec.gyro[N:], rec.acc[N:], rec.mag[N:], rec.dtw[N:], rec.acc0, rec.mag0)
    gd, am, my = synth.pack_planes(tail)
    path = tmp_path / "inputs.bin"
    with open(path, "wb") as fh:
        fh.write(np.array([B, N, W], np.int64).tobytes())
        fh.write(np.ascontiguousarray(rec.acc0, np.float64).tobytes())
        fh.write(np.ascontiguousarray(rec.mag0, np.float64).tobytes())
        for i in range(N):
            for a in (gyro[i], acc[i], mag[i]):
                fh.write(np.ascontiguousarray(a, np.float64).tobytes())
            fh.write(np.ascontiguousarray(t[i], np.int64).tobytes())
        for a in (gd, am, my):
            fh.write(np.ascontiguousarray(a, np.float32).tobytes())
    client = ctypes.CDLL(PREBUILT)  # built by csrc/Makefile with the library: no compiler run here
    client.pekf_example_run.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    res = tmp_path / "outputs.txt"
    assert client.pekf_example_run(os.fsencode(path), os.fsencode(res)) == 0
    vals = np.array([[float(v) for v in line.split()] for line in res.read_text().strip().splitlines()])
    assert vals.shape == (2 * B, 4)

    h = engine.FilterHandle(rec.acc0, rec.mag0, q=1.0, r=0.1, layout="soa")
    for i in range(N):
        X1 = h.update(gyro[i], t[i], acc[i], mag[i])
    win = engine.IMUWindow.from_planes(gd, am, my, rec.acc0, rec.mag0)
    h.run(win, n_steps=W)
    X2, _ = h.get_state()
    assert np.array_equal(vals[:B], X1) and np.array_equal(vals[B:], X2)


@pytest.mark.gpu
def test_wire_client_matches_python_session(tmp_path):
    """examples/wire_client.cpp: K phones' wire text (phase-2 then phase-3 messages, as the Android
    client sends them) -> pekf_wire_parse on the host, or the 100-byte frames -> pekf_wire_events_dev on
    the GPU -> FP64 event planes -> pekf_frontend_init_ext_dev -> pekf_live_ext_dev, all from C++; both
    parses give the same result, and the same texts through wire.events_from_wire and
    engine.run_session(events="f64") give the same counts and quaternions, bit for bit."""
    from poseestimationkf_amd import engine, wire
    K = 24
    ph2 = synth.generate_events(np.arange(K), 700, seed=51)
    ph3 = synth.generate_events(np.arange(K), 400, seed=52)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    paths = []
    for k in range(K):
        n3 = 400 - 7 * (k % 4)                                   # ragged phase-3 streams
        t3 = wire.events_text(ph3["types"][:n3, k], ph3["values"][:n3, k], ph3["times"][:n3, k], phase=3)
        if k % 5 == 1:                                           # a sensor type the server matches no sensor for
            cut = 100 * 200
            t3 = t3[:cut] + wire.message(3, 7, [1.5, -2.0, 3.25], ph3["times"][199, k]) + t3[cut:]
        text = wire.events_text(ph2["types"][:, k], ph2["values"][:, k], ph2["times"][:, k], phase=2) + t3
        p = tmp_path / ("phone%d.txt" % k)
        p.write_text(text)
        paths.append(str(p))
    client = ctypes.CDLL(WIRE_PREBUILT)  # built by csrc/Makefile with the library
    client.pekf_wire_example_run_mode.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    outs = []
    for device in (0, 1):  # the host parse (pekf_wire_parse), then the device parse (pekf_wire_events_dev)
        res = tmp_path / ("out%d.txt" % device)
        assert client.pekf_wire_example_run_mode("\n".join(paths).encode(), os.fsencode(res), device) == 0
        outs.append(np.array([[float(v) for v in line.split()] for line in res.read_text().strip().splitlines()]))
    got = outs[0]
    assert got.shape == (K, 5) and np.array_equal(outs[1], got)

    texts = [open(p).read() for p in paths]
    t0 = ph2["times"][0]
    e2 = wire.events_from_wire(texts, np.zeros((K, 3)), np.zeros((K, 3)), t0, phase=2)
    e3 = wire.events_from_wire(texts, np.zeros((K, 3)), np.zeros((K, 3)), t0, phase=3)
    f = engine.BatchedEKF(K)
    out = engine.run_session(e2, e3, f, events="f64")
    X, _ = f.get_state()
    assert out["ready"].all() and out["counts"].min() > 0
    assert np.array_equal(got[:, 0].astype(np.int64), out["counts"])
    assert np.array_equal(got[:, 1:], X)
