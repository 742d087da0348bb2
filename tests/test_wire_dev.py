"""The wire on the device (csrc/pekf_wire_dev.hip, engine.wire_events / run_wire_session): the clients'
100-byte frames parsed into the FP64 event planes by the GPU, checked against the host parse of the same
text (pekf_wire_parse: the server's std::stod / std::stoll, itself checked against Python in
tests/test_wire.py) bit for bit, and the whole device session against engine.run_session on the host's
events."""
import numpy as np
import pytest

from poseestimationkf_amd import synth, wire


def _frame(tokens, t, phase=3, ty=0):
    s = "#%d,%s:%s,%s,%s,t:%s" % (phase, ty, tokens[0], tokens[1], tokens[2], t)
    assert len(s) <= 99
    return s.ljust(99) + "\n"


def test_frames_layout():
    a = wire.message(3, 0, [1, 2, 3], 5) + wire.message(2, 1, [4, 5, 6], 7)
    b = wire.message(3, 2, [7, 8, 9], 9)
    fr = wire.frames([a, b])
    assert fr.shape == (2, 2, 100) and fr.dtype == np.uint8
    assert bytes(fr[1, 0]) == a[100:].encode() and bytes(fr[0, 1]) == b.encode()
    assert np.all(fr[1, 1] == ord(" "))                      # padding: a blank frame, no message
    with pytest.raises(ValueError, match="whole 100-byte frames"):
        wire.frames([a[:-1]])


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _host_planes(texts, phase, E):
    ev = wire.events_from_wire(texts, np.zeros((len(texts), 3)), np.zeros((len(texts), 3)),
                               np.zeros(len(texts), np.int64), phase=phase)
    p = synth.pack_events64(ev)
    out = np.empty((E, len(texts), 4))
    out[...] = np.uint64(synth.EV64_NONE_W).view(np.float64)
    out[..., :3] = 0.0
    n = min(E, p.shape[0])
    out[:n] = p[:n]
    return out


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint64), np.ascontiguousarray(b).view(np.uint64))


@pytest.mark.gpu
def test_wire_events_equal_the_host_parse(eng):
    """Phase-2 and phase-3 messages of ragged streams with phase-1 messages, blank and non-'#' frames,
    sensor types no sensor takes and every kind of float the client prints (Float.toString: plain and
    computerized forms, 1.4E-45 .. 3.4028235E38, NaN, Infinity): the device planes equal the host's,
    bit for bit, and so do the counts and phase 2's first time."""
    rng = np.random.default_rng(21)
    K = 150
    texts = []
    for k in range(K):
        n2, n3 = int(rng.integers(0, 60)), int(rng.integers(0, 90))
        vals = rng.standard_normal((n2 + n3, 3)) * 10.0 ** rng.integers(-40, 38, (n2 + n3, 3))
        vals = vals.astype(np.float32)
        vals[rng.random(vals.shape) < 0.01] = np.nan
        vals[rng.random(vals.shape) < 0.01] = np.inf
        vals[rng.random(vals.shape) < 0.01] = -np.inf
        vals[rng.random(vals.shape) < 0.01] = np.float32(1.4e-45)
        t = 10 ** 12 + np.cumsum(rng.integers(0, 3_000_000, n2 + n3))
        types = rng.integers(0, 3, n2 + n3).astype(str).astype(object)
        types[rng.random(n2 + n3) < 0.03] = "7"
        msgs = [wire.message(2 if i < n2 else 3, types[i], vals[i], t[i]) for i in range(n2 + n3)]
        if k % 5 == 0:
            msgs.insert(int(rng.integers(0, len(msgs) + 1)), wire.message(1, 2, [1, 2, 3], 42))
        if k % 7 == 0:
            msgs.insert(int(rng.integers(0, len(msgs) + 1)), " " * 99 + "\n")
        if k % 11 == 0:
            msgs.insert(int(rng.integers(0, len(msgs) + 1)), "x" * 99 + "\n")
        texts.append("".join(msgs))
    fr = wire.frames(texts)
    w = eng.wire_events(fr)
    F = fr.shape[0]
    host2, host3 = _host_planes(texts, 2, F), _host_planes(texts, 3, F)
    assert _same(w["ev2"].download((F, K, 4), np.float64), host2)
    assert _same(w["ev3"].download((F, K, 4), np.float64), host3)
    for k, tx in enumerate(texts):
        p = wire.parse(tx)
        assert w["n2"][k] == (p["phase"] == 2).sum() and w["n3"][k] == (p["phase"] == 3).sum()
        t2 = p["times"][p["phase"] == 2]
        assert w["first_t2"].download((K,), np.int64)[k] == (t2[0] if t2.size else 0)
    assert w["E3"] == int(w["n3"].max())


@pytest.mark.gpu
def test_wire_events_number_forms(eng):
    """Decimals the client never prints but the device parser takes: up to 19 significant digits, exponents
    to +-80 -- one IEEE operation where that is exact, the big-integer path elsewhere (also near halfway
    points) --, signs, leading zeros: strtod's value (the host parse's) bit for bit."""
    rng = np.random.default_rng(22)
    toks = []
    for _ in range(4000):
        nd = int(rng.integers(1, 20))
        digits = "".join(str(d) for d in rng.integers(0, 10, nd))
        point = int(rng.integers(0, nd + 1))
        mant = digits[:point] + ("." + digits[point:] if point < nd or rng.random() < 0.3 else "")
        if not mant.strip("."):
            mant = "0"
        e = int(rng.integers(-60, 60))
        toks.append(rng.choice(["", "-", "+"]) + mant + ("e%d" % e if rng.random() < 0.8 else ""))
    # halfway cases between adjacent doubles, written out in full, and their neighbours
    for v in rng.standard_normal(300) * 10.0 ** rng.integers(-30, 30, 300):
        a = np.float64(v)
        b = np.nextafter(a, np.inf)
        mid = (np.longdouble(a) + np.longdouble(b)) / 2
        toks.append(np.format_float_scientific(mid, precision=18, unique=False))
    toks += ["1.4E-45", "3.4028235E38", "9007199254740993", "1e22", "1e23", "0e80", "-0.0", "1e-80", "9e80"]
    rows = []
    for i in range(0, len(toks) - 2, 3):
        rows.append(_frame(toks[i:i + 3], i))
    K = 64
    texts = ["".join(rows[k::K]) for k in range(K)]
    fr = wire.frames(texts)
    w = eng.wire_events(fr)
    F = fr.shape[0]
    assert _same(w["ev3"].download((F, K, 4), np.float64), _host_planes(texts, 3, F))


def _fast_form(rng):
    """A number of the device's fast form: [-]D{1,8}.D+(E[-]D{1,2})? with at most 15 digits."""
    nI = int(rng.integers(1, 9))
    nF = int(rng.integers(1, 16 - nI))
    s = ("-" if rng.random() < 0.5 else "") + "".join(str(d) for d in rng.integers(0, 10, nI)) + "." + \
        "".join(str(d) for d in rng.integers(0, 10, nF))
    if rng.random() < 0.5:
        s += "E" + ("-" if rng.random() < 0.5 else "") + str(int(rng.integers(0, 23 if rng.random() < 0.5 else 60)))
    return s


# at the edges of the fast form and just past them (wire_frame takes those): width, digit counts, exponents
_EDGE_NUMBERS = ["12345678.5", "123456789.5", "12345678.1234567", "12345678.12345678", "1.23456789012345",
                 "1.234567890123456", "0.00000000000001", "0.000000000000001", "-1234567.123456",
                 "-1234567.1234567", "1.5E22", "1.5E-21", "1.5E-23", "9.9E-22", "1.5E79", "1.5E+5", "1.5e5",
                 "1.5E005", "+1.5", "1.", ".5", "5", "-0.0", "0.0E-99", "1.4E-45", "3.4028235E38", "NaN",
                 "-Infinity", "00000001.5", "1.5E-0"]
_EDGE_TIMES = ["0", "7", "12345678", "123456789", "2251799813685247", "0000000000000005", "00000000000000005",
               "-5", "-0"]


@pytest.mark.gpu
def test_wire_events_fast_form_edges(eng):
    """The device parses the client's own form without character loops and hands every other frame to the
    general parser -- per lane, in the same waves, a phone going on from its first such frame with the
    general parser.  Fast-form numbers and times at their limits, the forms just past them, and frames
    whose Type field is empty or longer, interleaved at random over 64 phones: every plane, count and
    first phase-2 time equals the host parse bit for bit."""
    rng = np.random.default_rng(23)
    K = 64
    texts = []
    for k in range(K):
        rows = []
        for i in range(int(rng.integers(20, 60))):
            u = rng.random()
            toks = [_fast_form(rng) if rng.random() < 0.7 else str(rng.choice(_EDGE_NUMBERS)) for _ in range(3)]
            if u < 0.85 or k % 4 == 0:      # some phones stay in the fast form throughout
                toks = [_fast_form(rng) for _ in range(3)]
            t = str(int(rng.integers(0, 10 ** int(rng.integers(1, 16))))) if rng.random() < 0.8 \
                else str(rng.choice(_EDGE_TIMES))
            ty = str(rng.choice(["0", "1", "2", "7", "12", ""])) if rng.random() < 0.2 else str(rng.integers(0, 3))
            rows.append(_frame(toks, t, phase=int(rng.choice([2, 3, 3, 1])), ty=ty))
        texts.append("".join(rows))
    fr = wire.frames(texts)
    w = eng.wire_events(fr)
    F = fr.shape[0]
    assert _same(w["ev2"].download((F, K, 4), np.float64), _host_planes(texts, 2, F))
    assert _same(w["ev3"].download((F, K, 4), np.float64), _host_planes(texts, 3, F))
    t2 = w["first_t2"].download((K,), np.int64)
    for k, tx in enumerate(texts):
        p = wire.parse(tx)
        assert w["n2"][k] == (p["phase"] == 2).sum() and w["n3"][k] == (p["phase"] == 3).sum()
        assert t2[k] == (p["times"][p["phase"] == 2][0] if (p["phase"] == 2).any() else 0)


@pytest.mark.gpu
@pytest.mark.parametrize("tok,t", [(" 1.5", "5"), ("0x1p3", "5"), ("1.5abc", "5"), ("12345678901234567890", "5"),
                                   ("1e81", "5"), ("inf", "5"), ("-NaN", "5"), ("1.5", "+5"), ("1.5", " 5"),
                                   ("1.5", "99999999999999999999"), ("1.5", "")])
def test_wire_events_report_other_forms(eng, tok, t):
    """A frame the client would never send -- a number in a form strtod reads but Float.toString never
    prints, or text std::stod / std::stoll throws on -- stops its phone and is reported (the host parse
    takes the forms strtod reads)."""
    good = _frame(["1.0", "2.0", "3.0"], 7)
    texts = [good * 3, good + _frame([tok, "2.0", "3.0"], t) + good]
    with pytest.raises(ValueError, match="phone 1, frame 1"):
        eng.wire_events(wire.frames(texts))


@pytest.mark.gpu
@pytest.mark.parametrize("K,F", [(1, 1), (65, 1), (65, 2), (64, 3), (129, 5)])
def test_wire_events_ring_edges(eng, K, F):
    """The two-slot LDS ring at its ends -- one or two frame indices, a last block of one phone --, with
    phase-2 and phase-3 messages, blank frames and, on some phones, a frame for the general parser in the
    middle: the planes, counts and first phase-2 times equal the host parse's."""
    rng = np.random.default_rng(K * 10 + F)
    texts = []
    for k in range(K):
        rows = []
        for i in range(F):
            u = rng.random()
            if u < 0.15:
                rows.append(" " * 99 + "\n")
            else:
                toks = [_fast_form(rng) for _ in range(3)]
                if k % 3 == 1 and i == F // 2:
                    toks[1] = "+1.5e3"                      # not the fast form: the general parser takes it
                rows.append(_frame(toks, int(rng.integers(0, 10 ** 12)), phase=int(rng.choice([2, 3])),
                                   ty=int(rng.integers(0, 3))))
        texts.append("".join(rows))
    fr = wire.frames(texts)
    w = eng.wire_events(fr)
    assert _same(w["ev2"].download((F, K, 4), np.float64), _host_planes(texts, 2, F))
    assert _same(w["ev3"].download((F, K, 4), np.float64), _host_planes(texts, 3, F))
    t2 = w["first_t2"].download((K,), np.int64)
    for k, tx in enumerate(texts):
        p = wire.parse(tx)
        assert w["n2"][k] == (p["phase"] == 2).sum() and w["n3"][k] == (p["phase"] == 3).sum()
        assert t2[k] == (p["times"][p["phase"] == 2][0] if (p["phase"] == 2).any() else 0)


def _compact(planes, K):
    """[F][K] frame-row planes -> each phone's rows that are not the no-message event, in order."""
    w = np.ascontiguousarray(planes[..., 3]).view(np.uint64)
    return [planes[w[:, k] != np.uint64(synth.EV64_NONE_W), k] for k in range(K)]


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [None, "3", "7"])
def test_wire_events_frame_rows(eng, chunks, monkeypatch):
    """PEKF_WIRE_FRAME_ROWS: row f of each plane is frame f's message of that phase or the no-message
    event; without those rows each phone's planes are the compacted planes bit for bit, with the same
    counts and first phase-2 times, on streams whose rows drift apart (phase-2 parts of different
    lengths, blank and phase-1 frames) and with a refused frame (its phone's rows from there on are
    no-message events) -- also with the frames split into chunks parsed by separate waves
    (PEKF_WIRE_CHUNKS; automatic where the grid is small)."""
    if chunks:
        monkeypatch.setenv("PEKF_WIRE_CHUNKS", chunks)
    rng = np.random.default_rng(31)
    K = 150
    texts = []
    for k in range(K):
        rows = []
        for ph, n in ((2, int(rng.integers(0, 40))), (3, int(rng.integers(0, 60)))):
            for i in range(n):
                if rng.random() < 0.1:
                    rows.append(" " * 99 + "\n" if rng.random() < 0.5 else wire.message(1, 2, [1, 2, 3], 42))
                rows.append(_frame([_fast_form(rng) for _ in range(3)], int(rng.integers(0, 10 ** 12)), phase=ph,
                                   ty=str(rng.choice(["0", "1", "2", "7"]))))
        texts.append("".join(rows))
    fr = wire.frames(texts)
    F = fr.shape[0]
    a = eng.wire_events(fr)
    r = eng.wire_events(fr, frame_rows=True)
    assert 0 < r["E2"] <= F and 0 < r["E3"] <= F and r["ev3_from"] == F - r["E3"]
    rows2 = r["ev2"].download((F, K, 4), np.float64)[r["E2"]:]
    rows3 = r["ev3"].download((F, K, 4), np.float64)[:r["ev3_from"]]
    for rest in (rows2, rows3):  # the rows outside the bounds hold no message of any phone
        assert np.all(np.ascontiguousarray(rest[..., 3]).view(np.uint64) == np.uint64(synth.EV64_NONE_W))
    assert np.array_equal(a["n2"], r["n2"]) and np.array_equal(a["n3"], r["n3"])
    assert _same(a["first_t2"].download((K,), np.int64), r["first_t2"].download((K,), np.int64))
    for plane, n in (("ev2", "n2"), ("ev3", "n3")):
        comp = a[plane].download((F, K, 4), np.float64)
        rows = r[plane].download((F, K, 4), np.float64)
        for k, got in enumerate(_compact(rows, K)):
            assert got.shape[0] == a[n][k] and _same(got, comp[:a[n][k], k])
    # a refused frame: its phone's rows from there on are no-message events
    bad_texts = [texts[0], _frame(["1.0", "2.0", "3.0"], 5, phase=3) + _frame(["1.5abc", "2.0", "3.0"], 6) +
                 _frame(["1.0", "2.0", "3.0"], 7, phase=3) * 5]
    fb = wire.frames(bad_texts)
    with pytest.raises(ValueError, match="phone 1, frame 1"):
        eng.wire_events(fb, frame_rows=True)
    # the refused phone's counts and rows, read past the error
    from poseestimationkf_amd._lib import check, lib
    Fb, Kb = fb.shape[:2]
    bufs = [eng.DeviceBuffer(n) for n in (fb.nbytes, 32 * Fb * Kb, 32 * Fb * Kb, 8 * Kb, 4 * Kb, 4 * Kb, 4 * Kb, 4)]
    bufs[0].upload(fb)
    bufs[7].upload(np.zeros(1, np.int32))
    check(lib.pekf_wire_events_ext_dev(Kb, Fb, bufs[0].ptr, Fb, Fb, bufs[1].ptr, bufs[2].ptr, bufs[3].ptr,
                                       bufs[4].ptr, bufs[5].ptr, bufs[6].ptr, bufs[7].ptr, None, 1, None))
    check(lib.pekf_device_sync())
    assert bufs[6].download((Kb,), np.int32).tolist() == [-1, 1]
    assert bufs[5].download((Kb,), np.int32)[1] == 1                  # the message before the refused frame
    e3 = bufs[2].download((Fb, Kb, 4), np.float64)[:, 1]
    w = np.ascontiguousarray(e3[:, 3]).view(np.uint64)
    assert w[0] != np.uint64(synth.EV64_NONE_W) and np.all(w[1:] == np.uint64(synth.EV64_NONE_W))


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [None, "5"])
def test_wire_session_frame_rows(eng, chunks, monkeypatch):
    """run_wire_session with frame-row planes (phase 2 and phase 3 skipping the no-message rows) equals
    the compacted session bit for bit -- ready, counts, refs, X, P -- on phones whose phase-2 parts differ
    in length, so that their phase-3 rows drift apart; also with the frames in chunks parsed by separate
    waves."""
    if chunks:
        monkeypatch.setenv("PEKF_WIRE_CHUNKS", chunks)
    K = 96
    ph2 = synth.generate_events(np.arange(K), 700, seed=63)
    ph3 = synth.generate_events(np.arange(K), 500, seed=64)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    texts = []
    for k in range(K):
        n2, n3 = 640 + 4 * (k % 13), 500 - 9 * (k % 5)
        texts.append(wire.events_text(ph2["types"][:n2, k], ph2["values"][:n2, k], ph2["times"][:n2, k], phase=2) +
                     wire.events_text(ph3["types"][:n3, k], ph3["values"][:n3, k], ph3["times"][:n3, k], phase=3))
    fr = wire.frames(texts)
    fa, fb = eng.BatchedEKF(K), eng.BatchedEKF(K)
    oa = eng.run_wire_session(fr, fa, frame_rows=False)
    ob = eng.run_wire_session(fr, fb, frame_rows=True)
    assert oa["ready"].sum() > K // 2 and oa["counts"][oa["ready"]].min() > 0
    for key in ("ready", "counts", "refs"):
        assert np.array_equal(oa[key], ob[key], equal_nan=key == "refs"), key
    for x, y in zip(fa.get_state(), fb.get_state()):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_wire_events_frame_is_the_message(eng):
    """The server takes each 100-byte recv as one message (KFS/Server.cpp:84-98), and so does the device: a
    newline inside a frame does not split it, and a Type field of '\\n' is a message of a type no sensor
    takes (the host's line parse, made for the client's own text, would read two lines there)."""
    good = _frame(["1.0", "2.0", "3.0"], 7, phase=2)
    odd = "#2,\n:1.5,-2.5,3.5E-3,t:9".ljust(99) + "\n"
    w = eng.wire_events(wire.frames([good + odd]))
    assert w["n2"][0] == 2
    ev = w["ev2"].download((2, 1, 4), np.float64)[1, 0]
    assert ev[:3].tolist() == [1.5, -2.5, 3.5e-3]
    bits = int(ev[3:4].view(np.uint64)[0])
    assert bits & 3 == synth.EV_OTHER and np.uint64(bits & ~3).view(np.float64) == 9.0


@pytest.mark.gpu
def test_wire_session_equals_the_host_session(eng):
    """The whole session from wire frames on the device (run_wire_session) equals run_session on the host's
    parse of the same text (wire.events_from_wire, events="f64") bit for bit: ready, counts, refs, X, P."""
    K = 96
    ph2 = synth.generate_events(np.arange(K), 700, seed=61)
    ph3 = synth.generate_events(np.arange(K), 500, seed=62)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    texts = []
    for k in range(K):
        n3 = 500 - 9 * (k % 5)
        texts.append(wire.events_text(ph2["types"][:, k], ph2["values"][:, k], ph2["times"][:, k], phase=2) +
                     wire.events_text(ph3["types"][:n3, k], ph3["values"][:n3, k], ph3["times"][:n3, k], phase=3))
    f_dev = eng.BatchedEKF(K)
    out_dev = eng.run_wire_session(wire.frames(texts), f_dev)
    t0 = ph2["times"][0]
    e2 = wire.events_from_wire(texts, np.zeros((K, 3)), np.zeros((K, 3)), t0, phase=2)
    e3 = wire.events_from_wire(texts, np.zeros((K, 3)), np.zeros((K, 3)), t0, phase=3)
    f_host = eng.BatchedEKF(K)
    out_host = eng.run_session(e2, e3, f_host, events="f64")
    assert out_dev["ready"].all() and out_dev["counts"].min() > 0
    for key in ("ready", "counts", "refs"):
        assert np.array_equal(out_dev[key], out_host[key]), key
    for a, b in zip(f_dev.get_state(), f_host.get_state()):
        assert np.array_equal(a, b)
