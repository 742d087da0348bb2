"""The phone -> server link (poseestimationkf_amd/wire.py, csrc/pekf_wire.cpp): the
sample values the server computes with.

The client sends Float.toString(f) of each sample (ASC/MessageSender.java:217-233) and the server
parses it with std::stod (KFS/Parser.cpp:12-26).  Checked here on the CPU (host functions of
libpekf, no device):
* pekf_f32_wire_values against a Python restatement (Python's shortest float formatting + float()),
  over every kind of float32: random bit patterns, subnormals, powers of ten, typical sensor readings;
* pekf_wire_parse against Python's own parse of the same text, for messages the client formats, the
  server's skip rules ('#' test, the 30-character test) and malformed messages;
* the FP64 event plane's layout (synth.pack_events64) and the f32 events' distance from the server's
  values through the oracle chain (front-end restatement -> NumPy filter), which is what the f32 event
  plane costs in parity (asserted in tests/test_live.py on the GPU)."""
import numpy as np
import pytest

from oracle import frontend_numpy as fe
from poseestimationkf_amd import synth, wire


def _py_server_value(f):
    return float(wire.java_float_string(f))


def _same_bits(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.array_equal(a.view(np.uint64), b.view(np.uint64)) or np.array_equal(a, b, equal_nan=True)


def test_server_values_of_every_kind_of_float():
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2 ** 32, size=20000, dtype=np.uint64).astype(np.uint32)
    f = bits.view(np.float32)
    f = f[np.isfinite(f)]
    extra = np.array([0.1, 0.2, 0.3, 1.0, 9.81, -9.81, 45.0, 1e-3, 9.999e-4, 1e7, 9999999.0, 1.4e-45, 7e-45, 3.4e38,
                      1.17549435e-38, 1e-30, 0.5, 2.0 ** -24, 123456.78, -0.0, 0.0, 16777216.0, 16777217.0],
                     np.float32)
    sensors = (rng.standard_normal(20000) * np.array([0.02, 9.81, 45.0])[rng.integers(0, 3, 20000)]).astype(np.float32)
    for arr in (f, extra, sensors):
        got = wire.server_values(arr)
        want = np.array([_py_server_value(x) for x in arr])
        assert _same_bits(got, want)
        assert np.array_equal(got.astype(np.float32), arr)          # every printed decimal reads back to f
    # in general the server's double is NOT the float: most sensor readings differ from (double)f
    got = wire.server_values(sensors)
    assert np.mean(got != sensors.astype(np.float64)) > 0.9
    assert wire.server_values(np.float32(0.1))[()] == 0.1          # "0.1", not 0.100000001490116
    nan_inf = wire.server_values(np.array([np.nan, np.inf, -np.inf], np.float32))
    assert np.isnan(nan_inf[0]) and nan_inf[1] == np.inf and nan_inf[2] == -np.inf


def test_java_float_string_format():
    """JDK 19+ Float.toString: plain form in [1e-3, 1e7), computerized scientific outside; at least one
    digit after the point; one-digit shortest decimals print the closest of one or two digits."""
    cases = {1.0: "1.0", 0.1: "0.1", 100.0: "100.0", 1e7: "1.0E7", 1e-3: "0.001", 9.999e-4: "9.999E-4",
             -2.5e-5: "-2.5E-5", 123456.78: "123456.78", 1.4e-45: "1.4E-45", 3.4028235e38: "3.4028235E38",
             9.81: "9.81", 1e10: "1.0E10"}
    for v, s in cases.items():
        assert wire.java_float_string(np.float32(v)) == s, (v, wire.java_float_string(np.float32(v)))


def test_wire_parse_is_the_servers_parse():
    rng = np.random.default_rng(8)
    n = 400
    types = rng.integers(0, 3, n)
    vals = (rng.standard_normal((n, 3)) * 20).astype(np.float32)
    vals[::37] *= np.float32(1e-6)
    times = 10 ** 12 + np.cumsum(rng.integers(1, 4_000_000, n))
    text = wire.events_text(types, vals, times)
    assert all(len(line) == 99 for line in text.splitlines())       # the 99-character frames
    got = wire.parse(text)
    assert np.array_equal(got["phase"], np.full(n, 3)) and np.array_equal(got["types"], types)
    assert np.array_equal(got["times"], times)
    want = np.array([[float(tok) for tok in line[5:].split(",")[:3]] for line in text.splitlines()])
    assert _same_bits(got["values"], want)
    assert _same_bits(got["values"], wire.server_values(vals))      # the packer's values are the parse's
    # the server's skip rules: no '#' (Parser::run), 30 characters or fewer after it (ProcessString)
    short = "#3,0:1.0,2.0,3.0,t:5\n"
    assert len(short) - 1 <= 30
    mixed = "noise line\n" + short + wire.message(2, 1, [1, 2, 3], 77) + "\n"
    p = wire.parse(mixed)
    assert p["phase"].tolist() == [2] and p["times"].tolist() == [77]
    # a message std::stod / std::stoll would throw on is an error naming its line
    from poseestimationkf_amd._lib import PekfError
    with pytest.raises(PekfError, match="wire message 2"):
        wire.parse(wire.message(3, 0, [1, 2, 3], 5) + "#3,0:abc,2.0,3.0,t:5" + " " * 40 + "\n")


def test_events_from_wire_pads_ragged_streams():
    ev = synth.generate_events(np.arange(3), 50, seed=4)
    texts = [wire.events_text(ev["types"][:40 + 5 * k, k], ev["values"][:40 + 5 * k, k], ev["times"][:40 + 5 * k, k])
             for k in range(3)]
    got = wire.events_from_wire(texts, ev["init_acc"], ev["init_mag"], ev["t_init"])
    assert got["types"].shape == (50, 3)
    assert np.all(got["types"][40:, 0] == synth.EV_NONE) and np.all(got["types"][:, 2] <= 2)
    # a message of a sensor type no sensor takes keeps its time, as a message (EV_OTHER)
    odd = wire.events_from_wire([wire.message(3, 7, [1, 2, 3], 5) + texts[0]], ev["init_acc"][:1],
                                ev["init_mag"][:1], ev["t_init"][:1])
    assert odd["types"][0, 0] == synth.EV_OTHER and odd["times"][0, 0] == 5
    assert np.array_equal(odd["types"][1:41, 0], got["types"][:40, 0])
    assert _same_bits(got["values64"][:50, 2], wire.server_values(ev["values"][:, 2]))
    # padding is no message: the restatements skip it, in phase 3 and in phase 2
    k = 0
    o = fe.run_frontend(got["types"][:, k], got["values64"][:, k], got["times"][:, k], ev["init_acc"][k],
                        ev["init_mag"][k], ev["t_init"][k])
    o40 = fe.run_frontend(got["types"][:40, k], got["values64"][:40, k], got["times"][:40, k], ev["init_acc"][k],
                          ev["init_mag"][k], ev["t_init"][k])
    assert all(np.array_equal(a, b) for a, b in zip(o, o40))
    i = fe.initial_values(got["types"][:, k], got["values64"][:, k], got["times"][:, k], n_avg=2)
    i40 = fe.initial_values(got["types"][:40, k], got["values64"][:40, k], got["times"][:40, k], n_avg=2)
    assert i["ready"] and i == i40


def test_pack_events64_layout():
    ev = synth.generate_events(np.arange(5), 30, seed=3)
    v64 = wire.server_values(ev["values"])
    p = synth.pack_events64(ev, v64)
    assert p.shape == (30, 5, 4) and p.dtype == np.float64
    assert _same_bits(p[..., :3], v64)
    w = p[..., 3].view(np.uint64)
    assert np.array_equal(w & np.uint64(3), ev["types"].astype(np.uint64))
    assert np.array_equal((w & ~np.uint64(3)).view(np.float64), ev["times"].astype(np.float64))
    with pytest.raises(ValueError, match="2\\^51"):
        synth.pack_events64(dict(ev, times=ev["times"] + (1 << 51)), v64)


def test_f32_events_vs_the_servers_values_through_the_oracle_chain():
    """What the 16 B f32 event plane costs: the same streams through the front-end restatement and the
    NumPy filter, once from (double)f and once from the server's stod values.  Records differ by ~1e-7
    and the final quaternions by ~1e-8 (7.5e-9 measured in round 5's review on 12 filters x 400
    events): inside the north_star's 1e-5, far outside FP64 rounding -- hence the FP64 event plane."""
    from oracle import ekf_numpy
    K, E = 6, 400
    ev = synth.generate_events(np.arange(K), E, seed=25)
    v64 = wire.server_values(ev["values"])
    worst_rec = worst_x = 0.0
    for k in range(K):
        args = (ev["types"][:, k],)
        tail = (ev["times"][:, k], ev["init_acc"][k], ev["init_mag"][k], ev["t_init"][k])
        r32 = fe.run_frontend(*args, ev["values"][:, k].astype(np.float64), *tail)
        r64 = fe.run_frontend(*args, v64[:, k], *tail)
        assert np.array_equal(r32[1], r64[1])                    # same records, same dts
        worst_rec = max(worst_rec, max(float(np.abs(a - b).max()) for a, b in zip((r32[0], r32[2], r32[3]),
                                                                               (r64[0], r64[2], r64[3]))))
        a0 = np.asarray(ev["init_acc"][k]) / np.linalg.norm(ev["init_acc"][k])
        m0 = np.asarray(ev["init_mag"][k]) / np.linalg.norm(ev["init_mag"][k])
        x32, _, _ = ekf_numpy.run_filter(r32[0], r32[1].astype(np.float64), r32[2], r32[3], a0, m0, record=False)
        x64, _, _ = ekf_numpy.run_filter(r64[0], r64[1].astype(np.float64), r64[2], r64[3], a0, m0, record=False)
        worst_x = max(worst_x, float(np.abs(x32 - x64).max()))
    print("f32 events vs the server's values: records %.2e, final X %.2e" % (worst_rec, worst_x))
    assert 1e-9 < worst_rec < 1e-6 and 1e-11 < worst_x < 1e-7


def test_wire_parse_number_forms():
    """pekf_wire_parse reads the client's plain decimals in place (one IEEE multiply or divide when that is
    exact) and anything else through strtod, as std::stod does: every form gives strtod's value -- the
    correctly rounded decimal -- whichever way it went."""
    rng = np.random.default_rng(11)
    toks = []
    for _ in range(3000):
        nd = int(rng.integers(1, 26))
        digits = "".join(str(d) for d in rng.integers(0, 10, nd))
        point = int(rng.integers(0, nd + 1))
        lead = "0" * int(rng.integers(0, 3))
        mant = lead + digits[:point] + "." + digits[point:] if rng.random() < 0.8 else lead + digits
        if mant.startswith(".") and rng.random() < 0.5:
            mant = "0" + mant
        exp = ""
        if rng.random() < 0.4:
            exp = rng.choice(["e", "E"]) + rng.choice(["", "+", "-"]) + str(int(rng.integers(0, 40)))
        toks.append(rng.choice(["", "-", "+"]) + mant + exp)
    toks += ["0.0", "-0.0", "+0.0", "1.", ".5", "-.5", "9007199254740993", "9007199254740992.0", "1e22", "1e23",
             "123456789012345678901234567890", "0.000000000000000000000000001", "4.9e-300", "1.7976931348623157e308"]
    toks = [t for t in toks if t.strip("+-.eE")]
    text = "".join("#3,0:%s,%s,%s,t:%d%s\n" % (a, b, c, i, " " * 40) for i, (a, b, c) in
                   enumerate(zip(toks[0::3], toks[1::3], toks[2::3])))
    got = wire.parse(text)
    want = np.array([float(t) for t in toks[: 3 * (len(toks) // 3)]]).reshape(-1, 3)
    assert _same_bits(got["values"], want)
    assert np.array_equal(got["times"], np.arange(len(want)))
    # forms std::stod takes and the client never prints: strtod's values
    odd = {" 1.5": 1.5, "0x1p3": 8.0, "inf": np.inf, "-Infinity": -np.inf, "1.5abc": 1.5, "1e": 1.0, "1e+": 1.0,
           "\t-2.25": -2.25, "1_000": 1.0}
    text = "".join("#3,1:%s,0.5,0.25,t:%s%s\n" % (k, t, " " * 40) for k, t in zip(odd, ["+5", " 7", "-3", "9x"] * 3))
    got = wire.parse(text)
    assert got["values"][:, 0].tolist() == list(odd.values()) and np.all(got["values"][:, 1:] == [0.5, 0.25])
    assert got["times"].tolist() == [5, 7, -3, 9, 5, 7, -3, 9, 5]
    nan = wire.parse("#3,1:nan,-NaN,0.25,t:1" + " " * 40 + "\n")["values"][0]
    assert np.isnan(nan[0]) and np.isnan(nan[1])
