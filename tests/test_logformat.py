"""The server's text log: Python reader (drop-in ReadFile semantics) and the
native ingest (pekf_log_scan / pekf_log_read, host code: runs without a GPU)."""
import gzip
import io
import os

import numpy as np
import pytest

from poseestimationkf_amd import logformat, synth

from .conftest import GOLDEN


@pytest.fixture(scope="module")
def c1_log(tmp_path_factory):
    p = tmp_path_factory.mktemp("log") / "KalmanFilter.txt"
    with gzip.open(os.path.join(GOLDEN, "c1_log.txt.gz"), "rt") as fh:
        p.write_text(fh.read())
    return str(p)


def test_reader_tag_precedence():
    lines = ["mag_0 : 0.5,0,-0.8\n", "acc_0 : 0,0,1\n", "q_gyro : 1.0, 0.0, 0.0, 0.0\n",
             "X_k : 1.0, 0.0, 0.0, 0.0\n", "Wahba_quart : 1.0, 0.0, 0.0, 0.0\n",
             "gyro : 0.1,0.2,0.3\n", "T : 100\n", "T : 200\n", "q_gyro : 1,0,0,0\n",
             "Mag_1 : 0.5,0.01,-0.8\n", "Acc_1 : 0.01,0.02,0.99\n"]
    d = logformat.parse_lines(lines)
    assert d.gyro == [[0.1, 0.2, 0.3]]                 # q_gyro lines are not gyro (ReadFile.py:36-39)
    assert d.quart_gyro == [[1.0, 0, 0, 0], [1, 0, 0, 0]]
    assert d.timestamp == [[100.0], [200.0]]
    assert d.quart_xk == [[1.0, 0, 0, 0]] and d.quart_wahba == [[1.0, 0, 0, 0]]
    g, dt, a, m, a0, m0 = logformat.log_to_arrays(d)
    assert dt.tolist() == [100.0] and a0.tolist() == [0, 0, 1]


def test_writer_reader_roundtrip_at_percent_f():
    rec = synth.generate(np.arange(1), 20)
    g, d, a, m = rec.filter(0)
    ts = synth.c1_timestamps(d.astype(np.int64))
    buf = io.StringIO()
    logformat.write_log(buf, ts, g, a, m, rec.acc0[0], rec.mag0[0])
    got = logformat.log_to_arrays(logformat.parse_lines(io.StringIO(buf.getvalue()).readlines()))
    assert np.array_equal(got[1], d)                   # integer ns timestamps survive exactly
    assert np.abs(got[0] - g).max() <= 5e-7            # std::to_string keeps 6 decimals
    assert np.abs(got[2] - a).max() <= 5e-7


def test_native_ingest_matches_python_reader(c1_log):
    from poseestimationkf_amd import engine
    rec = engine.read_log_records(c1_log)
    g, dt, a, m, a0, m0 = logformat.log_to_arrays(logformat.read_log(c1_log))
    assert rec.dtw.shape == (1550, 1)
    assert np.array_equal(rec.dt_ns[:, 0], dt)
    assert np.array_equal(rec.gyro[:, 0], g.astype(np.float32))
    assert np.array_equal(rec.acc[:, 0], a.astype(np.float32))
    assert np.array_equal(rec.mag[:, 0], m.astype(np.float32))
    assert np.array_equal(rec.acc0[0], a0) and np.array_equal(rec.mag0[0], m0)


def test_native_ingest_errors_are_reported(tmp_path):
    from poseestimationkf_amd import _lib, engine
    bad = tmp_path / "bad.txt"
    bad.write_text("mag_0 : 1,0,0\nacc_0 : 0,0,1\ngyro : 0,0,0\nT : 0\nT : 0.5\nMag_1 : 1,0,0\nAcc_1 : 0,0,1\n")
    # the plain reader refuses a dt the dt word cannot hold; read_log_records takes it via the side plane
    f3, u1 = np.empty(3, np.float32), np.empty(1, np.uint32)
    a0, m0 = np.empty(3), np.empty(3)
    st = _lib.lib.pekf_log_read(os.fsencode(str(bad)), 1, f3.ctypes.data, f3.ctypes.data, f3.ctypes.data,
                                u1.ctypes.data, _lib.dptr(a0), _lib.dptr(m0), None)
    assert st == _lib.PEKF_ERR_INVALID and "not an integer" in _lib.last_error()
    rec = engine.read_log_records(str(bad))
    assert rec.dtw[0, 0] == synth.DT_ESCAPE and rec.dt_ns[0, 0] == 0.5
    with pytest.raises(_lib.PekfError, match="cannot open"):
        engine.read_log_records(str(tmp_path / "missing.txt"))
    short = tmp_path / "short.txt"
    short.write_text("mag_0 : 1,0,0\nacc_0 : 0,0,1\nMag_1 : 1,0,0\nAcc_1 : 0,0,1\n")
    with pytest.raises(_lib.PekfError, match="Acc_1 records"):
        engine.read_log_records(str(short))


def test_native_ingest_escapes_long_negative_and_fractional_gaps(tmp_path):
    """Any float64 T - previousT the reference accepts (ExtendedKalmanFilter.py:62): a 5 s pause, a
    clock stepping back, a fractional ns difference and the escape value itself go to the dt side
    plane; the other records keep their dt in the word, and dt_ns equals the Python reader's."""
    from poseestimationkf_amd import engine
    rec = synth.generate(np.arange(1), 8)
    g, d, a, m = rec.filter(0)
    d = d.copy()
    d[2] = 5e9                 # a pause past 2^31 ns
    d[4] = -3e6                # a negative gap
    d[5] = float(0x7FFFFFFF)   # exactly the escape value: must be escaped too
    ts = [1_000_000_000_000.0]
    for v in d:
        ts.append(ts[-1] + v)
    path = tmp_path / "gaps.txt"
    with open(path, "w") as fh:
        logformat.write_log(fh, ts, g, a, m, rec.acc0[0], rec.mag0[0])
    lines = path.read_text().splitlines(keepends=True)
    last_t = max(i for i, l in enumerate(lines) if l.startswith("T : "))
    lines[last_t] = lines[last_t].rstrip("\n") + ".5\n"   # a fractional last gap (float64 timestamps)
    path.write_text("".join(lines))
    got = engine.read_log_records(str(path))
    _, dt_py, *_ = logformat.log_to_arrays(logformat.read_log(str(path)))
    assert np.array_equal(got.dt_ns[:, 0], dt_py)
    esc = got.dtw[:, 0] & synth.DT_MASK
    assert np.nonzero(esc == synth.DT_ESCAPE)[0].tolist() == [2, 4, 5, 7]
    assert got.dtx is not None and got.dtx[2, 0] == 5e9 and got.dtx[4, 0] == -3e6


def test_native_ingest_takes_lines_of_any_length(tmp_path):
    """A line is a line however long (Python's line iteration, ReadFile.py:27): a 3,000-value side
    channel and a sample padded with 6,000 blanks parse as the Python reader parses them."""
    from poseestimationkf_amd import engine
    rec = synth.generate(np.arange(1), 6)
    g, d, a, m = rec.filter(0)
    ts = synth.c1_timestamps(d.astype(np.int64))
    path = tmp_path / "long.txt"
    with open(path, "w") as fh:
        logformat.write_log(fh, ts, g, a, m, rec.acc0[0], rec.mag0[0])
    lines = path.read_text().splitlines(keepends=True)
    x = next(i for i, l in enumerate(lines) if l.startswith("X_k"))
    lines[x] = "X_k : " + ", ".join(["1.0"] * 3000) + "\n"
    gi = next(i for i, l in enumerate(lines) if l.startswith("gyro"))
    lines[gi] = "gyro : " + " " * 6000 + "0.25, -0.5, 0.125\n"
    path.write_text("".join(lines))
    got = engine.read_log_records(str(path))
    gp, dt_py, ap, mp, _, _ = logformat.log_to_arrays(logformat.read_log(str(path)))
    assert got.dtw.shape == (6, 1) and np.array_equal(got.dt_ns[:, 0], dt_py)
    assert np.array_equal(got.gyro[:, 0], gp.astype(np.float32)) and got.gyro[0, 0].tolist() == [0.25, -0.5, 0.125]


def _read64(path):
    import ctypes

    from poseestimationkf_amd import _lib
    bpath = os.fsencode(path)
    n = ctypes.c_int64()
    _lib.check(_lib.lib.pekf_log_scan(bpath, ctypes.byref(n)))
    g, a, m = (np.empty((n.value, 3)) for _ in range(3))
    dt, a0, m0, t0 = np.empty(n.value), np.empty(3), np.empty(3), ctypes.c_double()
    _lib.check(_lib.lib.pekf_log_read64(bpath, n.value, g.ctypes.data, a.ctypes.data, m.ctypes.data, dt.ctypes.data,
                                        _lib.dptr(a0), _lib.dptr(m0), ctypes.byref(t0)))
    return g, dt, a, m, a0, m0, t0.value


def test_native_ingest_float64_matches_python_reader(c1_log, tmp_path):
    """pekf_log_read64 (the FP64 records of pekf_run_rec64_dev): the log's values exactly as the Python
    reader (ReadFile.py:14-21's float64) parses them, dt = T[i+1] - T[i] as the reference forms it --
    on config 1's log and on a log with pauses and a clock stepping back."""
    g, dt, a, m, a0, m0, _ = _read64(c1_log)
    want = logformat.log_to_arrays(logformat.read_log(c1_log))
    for got, w in zip((g, dt, a, m, a0, m0), want):
        assert np.array_equal(got, w)
    rng = np.random.default_rng(4)
    n = 40
    ts = 1e15 + np.cumsum(rng.choice([1e7, 3.5e9, -2e6, 1234.0], size=n + 1))
    path = tmp_path / "odd.txt"
    logformat.write_log(str(path), ts, rng.normal(size=(n, 3)), rng.normal(size=(n, 3)) + [0, 0, 9.8],
                        rng.normal(size=(n, 3)) * 30, [0.1, 0.2, 9.8], [20.0, 1.0, -40.0])
    got = _read64(str(path))
    want = logformat.log_to_arrays(logformat.read_log(str(path)))
    for x, w in zip(got[:6], want):
        assert np.array_equal(x, w)
    assert (got[1] < 0).any() and got[1].max() > 2 ** 31   # (the writer's "T : %d" keeps integer ns)


def test_native_emit_matches_python_writer(tmp_path):
    """pekf_log_write (C++) writes write_log's bytes -- the server's WriteTextFile lines, std::to_string's
    "%f" -- for values of every size and sign, with and without the side channels, and the native reader
    reads the result back at that precision."""
    from poseestimationkf_amd._lib import PekfError
    rng = np.random.default_rng(3)
    n = 300
    scale = 10.0 ** rng.integers(-9, 11, size=(n, 3))
    g, a, m = (rng.standard_normal((n, 3)) * scale for _ in range(3))
    g[0] = [0.0, -0.0, -1e-9]
    a[1] = [np.inf, -np.inf, 123456789.123456789]
    t = 1_700_000_000_000_000_000 + np.cumsum(rng.integers(-5, 20_000_000, n + 1))
    a0, m0 = np.array([0.1, -0.2, 9.8]), np.array([20.5, -1e-7, -40.0])
    sides = [rng.standard_normal((n, 4)) for _ in range(3)]
    for kw in ({}, dict(zip(("q_gyro", "x_k", "wahba"), sides))):
        py, cc = tmp_path / "py.txt", tmp_path / "c.txt"
        logformat.write_log(str(py), t, g, a, m, a0, m0, **kw)
        logformat.write_log_native(str(cc), t, g, a, m, a0, m0, **kw)
        assert cc.read_bytes() == py.read_bytes()
    # the native float64 reader gets the printed values back ("inf" included, as float() reads it)
    import ctypes
    from poseestimationkf_amd._lib import check, lib
    cnt = ctypes.c_int64()
    check(lib.pekf_log_scan(os.fsencode(str(cc)), ctypes.byref(cnt)))
    assert cnt.value == n
    out = [np.empty((n, 3)) for _ in range(3)]
    dt, ra0, rm0 = np.empty(n), np.empty(3), np.empty(3)
    check(lib.pekf_log_read64(os.fsencode(str(cc)), n, out[0].ctypes.data, out[1].ctypes.data, out[2].ctypes.data,
                              dt.ctypes.data, ra0.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                              rm0.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), None))
    printed = lambda x: np.vectorize(lambda v: float("%f" % v))(x)  # noqa: E731
    for got, want in zip(out, (g, a, m)):
        assert np.array_equal(got, printed(want))
    assert np.array_equal(ra0, printed(a0)) and np.array_equal(rm0, printed(m0))
    # T parsed as float64 (ReadFile.py:20,41), so ns times past 2^53 round as the reference's own reader rounds them
    assert np.array_equal(dt, np.diff(t.astype(np.float64)))
    with pytest.raises(PekfError, match="cannot open"):
        logformat.write_log_native(str(tmp_path / "no" / "such" / "dir.txt"), t[:2], g[:1], a[:1], m[:1], a0, m0)
    logformat.write_log_native(str(cc), t[:1], g[:0], a[:0], m[:0], a0, m0)   # no record: the header only
    assert cc.read_text().count("\n") == 5
