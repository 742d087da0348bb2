"""Server front-end: raw phone events -> records -> filter, and the phase-2
initial means / variances that phase 3 starts from (KFS/Parser.cpp:36-58,84-140, InitialValues.cpp).

PARTLY PINNED: the checker is oracle/frontend_numpy.py, a restatement of the C++ front-end
(KFS/Parser.cpp, KFS/KalmanFilter.cpp), which cannot be built here (Eigen, Windows headers) and
ships no fixtures.  Its low-pass stage is pinned by the reference's own Test.py
(tests/golden/lpf_testpy.npz, made by tests/golden/make_lpf_golden.py); the state machine,
interpolation and normalisation are not.  The filter that consumes the records is pinned as
everywhere else."""
import numpy as np
import pytest

from oracle import frontend_numpy as fe
from poseestimationkf_amd import synth


def _oracle_records(ev, k, server=False):
    """Filter k's records by the restatement; server=True feeds it the server's own sample values
    (std::stod of the phone's Float.toString text, wire.server_values) instead of the floats widened."""
    if server:
        from poseestimationkf_amd import wire
        vals = wire.server_values(ev["values"][:, k])
    else:
        vals = ev["values"][:, k].astype(np.float64)
    return fe.run_frontend(ev["types"][:, k], vals, ev["times"][:, k], ev["init_acc"][k], ev["init_mag"][k],
                           ev["t_init"][k])


def test_oracle_lpf_matches_reference_test_py():
    """The alpha = 0.1 low-pass from a zero state, bit for bit against Test.py's own output."""
    import os
    from .conftest import GOLDEN
    d = np.load(os.path.join(GOLDEN, "lpf_testpy.npz"))
    alpha = float(d["alpha"][0])
    assert np.array_equal(fe.lpf(d["acc_raw"], alpha), d["acc_lpf"])
    assert np.array_equal(fe.lpf(d["mag_raw"], alpha), d["mag_lpf"])


def test_oracle_state_machine_basics():
    # acc0/mag0 from phase 2 at t=0; gyro @10, acc @20, mag @30 -> one record interpolated to t=10
    types = [synth.EV_GYRO, synth.EV_ACC, synth.EV_MAG]
    vals = np.array([[0.1, 0.2, 0.3], [0.0, 0.0, 2.0], [4.0, 0.0, 0.0]])
    g, dt, a, m = fe.run_frontend(types, vals, [10, 20, 30], [0.0, 0.0, 1.0], [2.0, 0.0, 0.0], 0)
    assert g.tolist() == [[0.1, 0.2, 0.3]] and dt.tolist() == [10]
    # acc at t=10 between (0,0,1)@0 and (0,0,2)@20 = (0,0,1.5) -> unit (0,0,1) -> LPF from 0: 0.1
    assert np.allclose(a, [[0.0, 0.0, 0.1]]) and np.allclose(m, [[0.1, 0.0, 0.0]])
    # a second gyro before the pair completes shifts acc_1 into acc_0 and restarts the pairing
    types = [synth.EV_GYRO, synth.EV_ACC, synth.EV_GYRO, synth.EV_ACC, synth.EV_MAG]
    vals = np.array([[0, 0, 0], [0, 0, 1.0], [9, 9, 9], [0, 0, 1.0], [1.0, 0, 0]], float)
    g, dt, a, m = fe.run_frontend(types, vals, [1, 2, 3, 4, 5], [0, 0, 1.0], [1.0, 0, 0], 0)
    assert g.tolist() == [[9, 9, 9]] and dt.tolist() == [3]


def test_oracle_records_are_lpf_of_unit_vectors():
    ev = synth.generate_events(np.arange(2), 1500)
    g, dt, a, m = _oracle_records(ev, 0)
    assert len(dt) > 100 and (dt > 0).all() and (dt < 2 ** 31).all()
    assert np.linalg.norm(a, axis=1).max() <= 1.0 + 1e-12
    assert abs(np.linalg.norm(a[0]) - 0.1) < 1e-12            # first LPF output from the zero state


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _f32_ulps(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b).max(initial=0)


@pytest.mark.gpu
def test_frontend_kernel_vs_oracle(eng):
    """Records equal the oracle's up to 1 f32 ulp (the kernel divides by reciprocal / rsqrt)."""
    K, E = 300, 1200
    ev = synth.generate_events(np.arange(K), E, seed=7)
    win, counts = eng.run_frontend(ev)
    n = int(counts.max())
    rec = win.download_filters(np.arange(K))
    for k in range(0, K, 37):
        g, dt, a, m = _oracle_records(ev, k)
        r = len(dt)
        assert counts[k] == r
        assert np.array_equal(rec.gyro[:r, k], g.astype(np.float32))
        assert np.array_equal(rec.dtw[:r, k], dt.astype(np.uint32))
        assert _f32_ulps(rec.acc[:r, k], a) <= 1
        assert _f32_ulps(rec.mag[:r, k], m) <= 1
        an = np.asarray(ev["init_acc"][k]) / np.sqrt(((ev["init_acc"][k] ** 2).sum()))
        assert np.abs(rec.acc0[k] - an).max() < 1e-15
    assert n <= E // 3 + 1


@pytest.mark.gpu
@pytest.mark.parametrize("events", ["f32", "f64"])
def test_frontend_other_messages_and_padding(eng, events):
    """Phase 3 skips a message no sensor takes (EV_OTHER, Parser.cpp:148-219 matches no Type) -- also one
    at the previous event's time or after a long pause (f32 events: time events around it) -- and
    padding (EV_NONE): the records equal the restatement's on the streams with them, and the fused kernel
    equals the split pipeline bit for bit."""
    K, E = 200, 900
    ev = synth.generate_events(np.arange(K), E, seed=17)
    ty, t = ev["types"].copy(), ev["times"].copy()
    rng = np.random.default_rng(17)
    for k in range(K):
        for e in rng.choice(np.arange(1, E - 100), 12, replace=False):
            ty[e, k] = synth.EV_OTHER
            if k % 3 == 0:
                t[e:, k] -= t[e, k] - t[e - 1, k]
            elif k % 3 == 1:
                t[e:, k] += 3 << 30
        if k % 4 == 1:
            ty[E - 90:, k] = synth.EV_NONE
    ev = dict(ev, types=ty, times=t)
    win, counts = eng.run_frontend(ev, events=events)
    for k in range(0, K, 7):
        og, odt, oa, om = _oracle_records(ev, k, server=events == "f64")
        r = len(odt)
        assert counts[k] == r and r > 20
        if events == "f64":
            g, dt, a, m, _ = win.download_filters([k])
            assert np.array_equal(g[:r, 0], og) and np.array_equal(dt[:r, 0], odt.astype(np.float64))
            assert np.abs(a[:r, 0] - oa).max() < 1e-15 and np.abs(m[:r, 0] - om).max() < 1e-15
        else:
            rec = win.download_filters([k])
            assert np.array_equal(rec.gyro[:r, 0], og.astype(np.float32))
            assert np.array_equal(rec.dt_ns[:r, 0], odt.astype(np.float64))
            assert _f32_ulps(rec.acc[:r, 0], oa) <= 1 and _f32_ulps(rec.mag[:r, 0], om) <= 1
    split = eng.BatchedEKF(K)
    split.run(win)
    fused = eng.BatchedEKF(K)
    c, _ = fused.run_events(ev, records="f64" if events == "f64" else "f32", events=events)
    assert np.array_equal(c, counts)
    assert np.array_equal(fused.get_state()[0], split.get_state()[0])
    assert np.array_equal(fused.get_state()[1], split.get_state()[1])


@pytest.mark.gpu
def test_events_to_filter_end_to_end(eng, oracle_c):
    """raw events -> front-end kernel -> fused filter, vs oracle front-end -> C oracle filter."""
    K, E = 256, 1500
    ev = synth.generate_events(np.arange(K), E, seed=8)
    win, counts = eng.run_frontend(ev)
    n = int(counts.min())
    f = eng.BatchedEKF(K)
    f.run(win, n_steps=n)
    X, _ = f.get_state()
    cols = np.arange(0, K, 16)
    gy, dtw, acc, mag = [], [], [], []
    for k in cols:
        g, dt, a, m = _oracle_records(ev, k)
        gy.append(g[:n]); dtw.append(dt[:n]); acc.append(a[:n]); mag.append(m[:n])
    refs = win.refs.download((K, 6), np.float64)[cols]
    rec = synth.Records(np.stack(gy, 1).astype(np.float32), np.stack(acc, 1).astype(np.float32),
                        np.stack(mag, 1).astype(np.float32), np.stack(dtw, 1).astype(np.uint32),
                        refs[:, :3], refs[:, 3:])
    Xo, _, _ = oracle_c.run(rec)
    err = float(np.abs(X[cols] - Xo).max())
    print("events -> front-end -> filter vs oracle chain: max |dq| = %.3e over %d records" % (err, n))
    assert err < 1e-9


def _events(K, spec):
    """Hand-made event streams: spec = list of (type, gap_ns) applied to every filter, values
    from a fixed pattern.  Returns the generate_events-style dict."""
    E = len(spec)
    types = np.array([[t] * K for t, _ in spec], np.uint32).reshape(E, K)
    gaps = np.array([[g] * K for _, g in spec], np.int64).reshape(E, K)
    times = synth.T_INIT_NS + np.cumsum(gaps, axis=0)
    e = np.arange(E)[:, None, None]
    vals = (np.cos(0.3 * e + np.arange(3)[None, None, :] + 0.01 * np.arange(K)[None, :, None]) +
            np.where(types[..., None] == synth.EV_ACC, [0, 0, 9.0], [0, 0, 0])).astype(np.float32)
    return dict(types=types, values=vals, times=times, init_acc=np.tile([0.1, 0.2, 9.8], (K, 1)),
                init_mag=np.tile([20.0, 1.0, -40.0], (K, 1)), t_init=np.full(K, synth.T_INIT_NS, np.int64))


@pytest.mark.gpu
def test_frontend_row_queue_with_drifting_lanes(eng):
    """k_frontend queues each 8-lane group's records in a shared pool of LDS slots and writes whole
    rows; records more than 32 rows ahead of the group's base, or met by an empty pool, are stored
    directly.  Lanes drifting 0-12 rows apart (acc-only lead-ins), a slow lane (a record per 5
    events), a late lane, one with no records (its group's base never moves, so the pool runs dry),
    one never ready, and a partial last wave (a group of 5 lanes): every record of every filter
    equals the restatement's."""
    A, G, M = synth.EV_ACC, synth.EV_GYRO, synth.EV_MAG
    K, E = 64 * 2 + 5, 600
    types = np.empty((E, K), np.uint32)
    for k in range(K):
        lane = k % 64
        if lane < 58:      # triples after a lead-in of (lane % 13) x 3 acc events
            seq = [A] * (3 * (lane % 13)) + [G, A, M] * E
        elif lane < 60:    # slow: G A M G A, one record per 5 events
            seq = [G, A, M, G, A] * E
        elif lane < 62:    # late: half the stream acc only
            seq = [A] * (E // 2) + [G, A, M] * E
        else:              # no record (62), or never ready (63)
            seq = [A, M] * E
            if lane == 63:
                seq = [G, A, M] * E
        types[:, k] = seq[:E]
    e = np.arange(E)[:, None]
    gaps = 900 + (e * 7 + np.arange(K)[None, :] * 13) % 400
    times = synth.T_INIT_NS + np.cumsum(gaps, axis=0)
    vals = (np.sin(0.05 * e[..., None] + 0.1 * np.arange(K)[None, :, None] + np.arange(3)[None, None, :]) +
            np.where(types[..., None] == A, [0, 0, 9.0], [0, 0, 0])).astype(np.float32)
    init_acc = np.tile([0.1, 0.2, 9.8], (K, 1))
    init_acc[np.arange(K) % 64 == 63] = np.nan
    ev = dict(types=types, values=vals, times=times, init_acc=init_acc,
              init_mag=np.tile([20.0, 1.0, -40.0], (K, 1)), t_init=np.full(K, synth.T_INIT_NS, np.int64))
    win, counts = eng.run_frontend(ev)
    rec = win.download_filters(np.arange(K))
    spread = []
    for k in range(K):
        if k % 64 == 63:
            assert counts[k] == 0
            continue
        g, dt, a, m = _oracle_records(ev, k)
        r = len(dt)
        spread.append(r)
        assert counts[k] == r
        assert np.array_equal(rec.gyro[:r, k], g.astype(np.float32))
        assert np.array_equal(rec.dtw[:r, k], dt.astype(np.uint32))
        assert _f32_ulps(rec.acc[:r, k], a) <= 1
        assert _f32_ulps(rec.mag[:r, k], m) <= 1
    assert max(spread) - min(spread) > 100 and 0 in spread


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 2, 3, 5, 7, 8, 9, 15, 17, 70])
def test_frontend_partial_lane_groups(eng, K):
    """Batches that end inside an 8-lane group (the pooled queue's unit): the group's ring of free
    slots is filled by the lanes it has, and every record of every filter equals the restatement's."""
    E = 240
    ev = synth.generate_events(np.arange(K), E, seed=100 + K)
    win, counts = eng.run_frontend(ev)
    rec = win.download_filters(np.arange(K))
    for k in range(K):
        g, dt, a, m = _oracle_records(ev, k)
        r = len(dt)
        assert counts[k] == r
        assert np.array_equal(rec.gyro[:r, k], g.astype(np.float32))
        assert np.array_equal(rec.dtw[:r, k], dt.astype(np.uint32))
        assert _f32_ulps(rec.acc[:r, k], a) <= 1
        assert _f32_ulps(rec.mag[:r, k], m) <= 1


@pytest.mark.gpu
def test_frontend_streams_without_records(eng):
    K = 70
    for spec in ([], [(synth.EV_ACC, 10), (synth.EV_MAG, 10)] * 5,            # nothing, or no gyro at all
                 [(synth.EV_GYRO, 10), (synth.EV_ACC, 10), (synth.EV_GYRO, 10)] * 3):  # never a mag after a gyro
        _, counts = eng.run_frontend(_events(K, spec), r_max=8)
        assert np.all(counts == 0)


@pytest.mark.gpu
def test_frontend_r_max_overflow_is_reported(eng):
    spec = [(synth.EV_GYRO, 1000), (synth.EV_ACC, 1000), (synth.EV_MAG, 1000)] * 6  # 6 records
    with pytest.raises(ValueError, match="r_max"):
        eng.run_frontend(_events(4, spec), r_max=5)
    _, counts = eng.run_frontend(_events(4, spec), r_max=6)
    assert np.all(counts == 6)


@pytest.mark.gpu
def test_frontend_zero_time_gaps_follow_ieee_like_the_cpp(eng):
    """Equal acc (or mag) timestamps make the interpolation divide by zero: the C++ server's double
    arithmetic gives inf/nan there (no exception), and so do the oracle and the kernel."""
    K = 8
    # acc_0 and acc_1 both at t = 500 (zero gaps): the first record's acc is 0/0 -> nan, and the
    # low-pass carries the nan into the second record; the magnetometer channel stays finite
    spec = [(synth.EV_ACC, 500), (synth.EV_GYRO, 0), (synth.EV_ACC, 0), (synth.EV_MAG, 500),
            (synth.EV_GYRO, 500), (synth.EV_ACC, 500), (synth.EV_MAG, 500)]
    ev = _events(K, spec)
    win, counts = eng.run_frontend(ev, r_max=4)
    rec = win.download_filters(np.arange(K))
    for k in range(K):
        g, dt, a, m = _oracle_records(ev, k)
        r = len(dt)
        assert counts[k] == r == 2
        assert np.isnan(a).all() and np.isnan(rec.acc[:r, k]).all()
        fin = np.isfinite(a)
        assert _f32_ulps(rec.acc[:r, k][fin], a[fin]) <= 1
        assert _f32_ulps(rec.mag[:r, k], m) <= 1


# ------------------------------------------------------------------ phase 2: initial means / variances

def test_oracle_initial_values_state_machine():
    """Parser.cpp:36-58,84-140 with n_avg = 2: each sensor is initialised at its first sample after
    two, the KalmanFilter at the next event after all three, and later events move t_init."""
    A, G, M = synth.EV_ACC, synth.EV_GYRO, synth.EV_MAG
    spec = [(A, 10), (A, 10), (G, 10), (G, 10), (M, 10), (M, 10), (A, 10), (G, 10)]
    ev = _events(1, spec)
    o = fe.initial_values(ev["types"][:, 0], ev["values"][:, 0], ev["times"][:, 0], n_avg=2)
    assert not o["ready"]                                   # the magnetometer has no third sample yet
    ev = _events(1, spec + [(M, 10), (A, 10), (G, 20)])     # M initialises it; A builds the filter; G moves time
    o = fe.initial_values(ev["types"][:, 0], ev["values"][:, 0], ev["times"][:, 0], n_avg=2)
    assert o["ready"] and o["t_init"] == int(ev["times"][-1, 0])
    acc = ev["values"][:2, 0].astype(np.float64)           # the first two acc samples only
    assert np.allclose(o["acc"], acc.mean(0), rtol=0, atol=1e-15)
    assert np.allclose(o["var_acc"], acc.var(0, ddof=1), rtol=1e-15, atol=1e-15)


def test_oracle_initial_values_match_numpy_statistics():
    ev = synth.generate_events(np.arange(3), 700, seed=21)
    for k in range(3):
        o = fe.initial_values(ev["types"][:, k], ev["values"][:, k], ev["times"][:, k])
        assert o["ready"] and o["t_init"] == int(ev["times"][-1, k])
        for ty, name in ((synth.EV_ACC, "acc"), (synth.EV_MAG, "mag"), (synth.EV_GYRO, "gyro")):
            x = ev["values"][:, k][ev["types"][:, k] == ty][:100].astype(np.float64)
            assert np.allclose(o[name], x.mean(0), rtol=1e-15, atol=1e-12)
            assert np.allclose(o["var_" + name], x.var(0, ddof=1), rtol=1e-12, atol=1e-15)


def test_oracle_initial_values_other_messages_and_padding():
    """Any message counts in phase 2 (Parser.cpp:36-62 switches on the phase, not the sensor type): one
    no sensor takes (EV_OTHER) adds no sample but builds the filter or moves its time; no message
    (EV_NONE, padding) does neither."""
    A, G, M, O, N = synth.EV_ACC, synth.EV_GYRO, synth.EV_MAG, synth.EV_OTHER, synth.EV_NONE
    spec = [(A, 10), (A, 10), (G, 10), (G, 10), (M, 10), (M, 10), (A, 10), (G, 10), (M, 10)]
    for tail, ready, t_last in (([(O, 10)], True, 100), ([(N, 10)], False, None), ([(N, 10), (O, 30)], True, 130),
                                ([(O, 10), (O, 0), (N, 50)], True, 100)):
        ev = _events(1, spec + tail)
        o = fe.initial_values(ev["types"][:, 0], ev["values"][:, 0], ev["times"][:, 0], n_avg=2)
        assert o["ready"] == ready, tail
        assert o["t_init"] == (None if t_last is None else synth.T_INIT_NS + t_last), tail
    # an EV_OTHER message before the sensors are initialised is no sample
    ev = _events(1, [(O, 10)] * 3 + spec + [(A, 10)])
    o = fe.initial_values(ev["types"][:, 0], ev["values"][:, 0], ev["times"][:, 0], n_avg=2)
    r = fe.initial_values(ev["types"][3:, 0], ev["values"][3:, 0], ev["times"][3:, 0], n_avg=2)
    assert o["ready"] and o == r


def _kalman_event(types, n_avg):
    """The index of the phase-2 event that builds the KalmanFilter (Parser.cpp:41-55), or None."""
    cnt, done = {0: 0, 1: 0, 2: 0}, {0: False, 1: False, 2: False}
    for i, ty in enumerate(types):
        ty = int(ty)
        if all(done.values()):
            return i
        if ty in cnt:
            if cnt[ty] < n_avg:
                cnt[ty] += 1
            else:
                done[ty] = True
    return None


@pytest.mark.gpu
@pytest.mark.parametrize("events", ["f32", "f64"])
def test_frontend_init_other_messages_and_padding(eng, events):
    """Phase 2 on streams holding messages no sensor takes (EV_OTHER) -- among them the one that builds
    the filter, some at the previous event's time (f32 events: gap 0 needs a time event before it) or
    after a pause of 2^30 ns and more -- and padding (EV_NONE) after the last message: the kernel against
    the restatement, bit for bit."""
    from poseestimationkf_amd import wire
    K, E, n_avg = 96, 700, 100
    ev = synth.generate_events(np.arange(K), E, seed=13)
    ty, t = ev["types"].copy(), ev["times"].copy()
    rng = np.random.default_rng(13)
    for k in range(K):
        i = _kalman_event(ty[:, k], n_avg)
        assert i is not None
        if k % 2 == 0:
            ty[i, k] = synth.EV_OTHER                         # the message that builds the filter
        for e in rng.choice(np.arange(1, E - 60), 5, replace=False):
            ty[e, k] = synth.EV_OTHER
            if k % 3 == 0:
                t[e:, k] -= t[e, k] - t[e - 1, k]             # at the previous event's time
            elif k % 3 == 1:
                t[e:, k] += 3 << 30                           # after a long pause
        if k % 4 == 1:
            ty[E - 50:, k] = synth.EV_NONE                    # a shorter stream, padded
        if k % 8 == 5:
            i = _kalman_event(ty[:, k], n_avg)
            ty[i:, k] = synth.EV_NONE                         # ends as the last sensor initialises: not ready
    ev = dict(ev, types=ty, times=t)
    got = eng.frontend_init(ev, n_avg=n_avg, events=events)
    vals = wire.server_values(ev["values"]) if events == "f64" else ev["values"].astype(np.float64)
    n_ready = 0
    for k in range(K):
        o = fe.initial_values(ty[:, k], vals[:, k], t[:, k], n_avg=n_avg)
        assert got["ready"][k] == o["ready"], k
        assert not (k % 8 == 5 and o["ready"])
        if not o["ready"]:
            assert np.isnan(got["init"][k]).all()
            continue
        n_ready += 1
        assert got["t_init"][k] == o["t_init"]
        assert np.array_equal(got["init"][k], np.array(o["acc"] + o["mag"]))
        for name in ("acc", "mag", "gyro"):
            assert np.array_equal(got["var_" + name][k], np.array(o["var_" + name]))
    assert n_ready >= K // 2


@pytest.mark.gpu
@pytest.mark.parametrize("E,n_avg", [(700, 100), (520, 100), (40, 2)])
def test_frontend_init_kernel_vs_oracle(eng, E, n_avg):
    """pekf_frontend_init_dev against the restatement, bit for bit (the same sequential FP64 sums and
    IEEE divisions), including filters that never get ready (520 events: about a third lack a
    magnetometer sample after their first 100)."""
    K = 300
    ev = synth.generate_events(np.arange(K), E, seed=8)
    got = eng.frontend_init(ev, n_avg=n_avg)
    n_ready = 0
    for k in range(K):
        o = fe.initial_values(ev["types"][:, k], ev["values"][:, k], ev["times"][:, k], n_avg=n_avg)
        assert got["ready"][k] == o["ready"]
        if not o["ready"]:
            assert np.isnan(got["init"][k]).all()
            continue
        n_ready += 1
        assert got["t_init"][k] == o["t_init"]
        assert np.array_equal(got["init"][k], np.array(o["acc"] + o["mag"]))
        assert np.array_equal(got["gyro_mean"][k], np.array(o["gyro"]))
        for name in ("acc", "mag", "gyro"):
            assert np.array_equal(got["var_" + name][k], np.array(o["var_" + name]))
    assert n_ready > 0 and (E != 520 or n_ready < K)
    # without stats (run_session's call) the kernel skips the variance pass; the rest is unchanged
    means = eng.frontend_init(ev, n_avg=n_avg, stats=False)
    assert set(means) == {"init", "t_init", "ready"}
    assert np.array_equal(means["ready"], got["ready"]) and np.array_equal(means["t_init"], got["t_init"])
    assert np.array_equal(means["init"], got["init"], equal_nan=True)


@pytest.mark.gpu
def test_phase2_then_phase3_events_to_filter(eng, oracle_c):
    """The whole server front-end on the device: phase-2 events -> initial means and time
    (pekf_frontend_init_dev) -> phase-3 events -> records (pekf_frontend_dev) -> the fused filter,
    against the oracle chain (restatements of both phases + the C filter)."""
    K = 96
    ph2 = synth.generate_events(np.arange(K), 800, seed=31)
    ini = eng.frontend_init(ph2)
    assert ini["ready"].all()
    ph3 = synth.generate_events(np.arange(K), 400, seed=32)
    # phase 3 continues from the phase-2 means at the last phase-2 event's time
    shift = ini["t_init"] - ph3["t_init"]
    ph3 = dict(ph3, times=ph3["times"] + shift[None, :], t_init=ini["t_init"],
               init_acc=ini["init"][:, :3], init_mag=ini["init"][:, 3:])
    win, counts = eng.run_frontend(ph3)
    cols = np.array([0, 1, 47, 95])
    for k in cols:
        o = fe.initial_values(ph2["types"][:, k], ph2["values"][:, k], ph2["times"][:, k])
        assert o["t_init"] == ini["t_init"][k] and np.array_equal(np.array(o["acc"] + o["mag"]), ini["init"][k])
    n = int(counts[cols].min())
    gy, dtw, acc, mag = [], [], [], []
    for k in cols:
        g, dt, a, m = _oracle_records(ph3, k)
        gy.append(g[:n]); dtw.append(dt[:n]); acc.append(a[:n]); mag.append(m[:n])
    refs = win.refs.download((K, 6), np.float64)[cols]
    rec = synth.Records(np.stack(gy, 1).astype(np.float32), np.stack(acc, 1).astype(np.float32),
                        np.stack(mag, 1).astype(np.float32), np.stack(dtw, 1).astype(np.uint32),
                        refs[:, :3], refs[:, 3:])
    Xo, _, _ = oracle_c.run(rec)
    f2 = eng.BatchedEKF(K)
    f2.run(win, n_steps=n, counts=np.full(K, n))
    X2, _ = f2.get_state()
    err = float(np.abs(X2[cols] - Xo).max())
    print("phase 2 + phase 3 + filter vs oracle chain: max |dq| = %.3e over %d records" % (err, n))
    assert err < 1e-9


# ------------------------------------------------------------------ FP64 events (PEKF_EV_F64_EVENTS)

@pytest.mark.gpu
def test_frontend_fp64_events_records_vs_oracle(eng):
    """k_frontend on FP64 events writes FP64 records (pekf_run_rec64_dev's planes): against the
    restatement fed the server's values, gyro and dt exactly, acc / mag within 1e-15 (the kernel's
    reciprocal / rsqrt with a Newton step against IEEE divisions), the pooled queue's rows intact.  The
    f32 events' records against the same oracle differ by the samples' f32 rounding (~1e-7)."""
    K, E = 300, 1200
    ev = synth.generate_events(np.arange(K), E, seed=7)
    win, counts = eng.run_frontend(ev, events="f64")
    g, dt, a, m, refs = win.download_filters(np.arange(K))
    win32, _ = eng.run_frontend(ev)
    rec32 = win32.download_filters(np.arange(K))
    worst = worst32 = 0.0
    for k in range(K):
        og, odt, oa, om = _oracle_records(ev, k, server=True)
        r = len(odt)
        assert counts[k] == r
        assert np.array_equal(g[:r, k], og) and np.array_equal(dt[:r, k], odt.astype(np.float64))
        worst = max(worst, float(np.abs(a[:r, k] - oa).max()), float(np.abs(m[:r, k] - om).max()))
        worst32 = max(worst32, float(np.abs(rec32.acc[:r, k] - oa).max()), float(np.abs(rec32.mag[:r, k] - om).max()))
        an = np.asarray(ev["init_acc"][k]) / np.sqrt(((ev["init_acc"][k] ** 2).sum()))
        assert np.abs(refs[k, :3] - an).max() < 1e-15
    print("FP64-event records vs the server-value restatement %.2e; f32-event records vs it %.2e" % (worst, worst32))
    assert worst < 1e-15 and 1e-9 < worst32 < 1e-6


@pytest.mark.gpu
def test_frontend_fp64_events_drifting_lanes_and_padding(eng):
    """The FP64-record pool (32 slots per 8-lane group) under lanes drifting apart, a slow lane, one with
    no record, and streams padded with no-sample events: every record equals the restatement's."""
    A, G, M = synth.EV_ACC, synth.EV_GYRO, synth.EV_MAG
    K, E = 64 * 2 + 5, 600
    types = np.empty((E, K), np.uint32)
    for k in range(K):
        lane = k % 64
        if lane < 58:
            seq = [A] * (3 * (lane % 13)) + [G, A, M] * E
        elif lane < 62:
            seq = [G, A, M, G, A] * E
        else:
            seq = [A, M] * E
        types[:, k] = seq[:E]
    types[E - 40:, ::3] = 3                                  # padded tails
    e = np.arange(E)[:, None]
    gaps = 900 + (e * 7 + np.arange(K)[None, :] * 13) % 400
    times = synth.T_INIT_NS + np.cumsum(gaps, axis=0)
    vals = (np.sin(0.05 * e[..., None] + 0.1 * np.arange(K)[None, :, None] + np.arange(3)[None, None, :]) +
            np.where(types[..., None] == A, [0, 0, 9.0], [0, 0, 0])).astype(np.float32)
    ev = dict(types=types, values=vals, times=times, init_acc=np.tile([0.1, 0.2, 9.8], (K, 1)),
              init_mag=np.tile([20.0, 1.0, -40.0], (K, 1)), t_init=np.full(K, synth.T_INIT_NS, np.int64))
    win, counts = eng.run_frontend(ev, events="f64")
    g, dt, a, m, _ = win.download_filters(np.arange(K))
    for k in range(K):
        og, odt, oa, om = _oracle_records(ev, k, server=True)
        r = len(odt)
        assert counts[k] == r
        assert np.array_equal(g[:r, k], og) and np.array_equal(dt[:r, k], odt.astype(np.float64))
        if r:
            assert np.abs(a[:r, k] - oa).max() < 1e-15 and np.abs(m[:r, k] - om).max() < 1e-15
    assert counts.max() - counts.min() > 100 and counts.min() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("E,n_avg", [(700, 100), (520, 100), (40, 2)])
def test_frontend_init_fp64_events_vs_oracle(eng, E, n_avg):
    """Phase 2 on FP64 events: the means and variances of the server's own values, bit for bit against
    the restatement fed the same doubles (the same sequential sums and IEEE divisions)."""
    from poseestimationkf_amd import wire
    K = 300
    ev = synth.generate_events(np.arange(K), E, seed=8)
    v64 = wire.server_values(ev["values"])
    got = eng.frontend_init(ev, n_avg=n_avg, events="f64")
    n_ready = 0
    for k in range(K):
        o = fe.initial_values(ev["types"][:, k], v64[:, k], ev["times"][:, k], n_avg=n_avg)
        assert got["ready"][k] == o["ready"]
        if not o["ready"]:
            assert np.isnan(got["init"][k]).all()
            continue
        n_ready += 1
        assert got["t_init"][k] == o["t_init"]
        assert np.array_equal(got["init"][k], np.array(o["acc"] + o["mag"]))
        assert np.array_equal(got["gyro_mean"][k], np.array(o["gyro"]))
        for name in ("acc", "mag", "gyro"):
            assert np.array_equal(got["var_" + name][k], np.array(o["var_" + name]))
    assert n_ready > 0 and (E != 520 or n_ready < K)


@pytest.mark.gpu
def test_fp64_event_arguments_are_checked(eng):
    """PEKF_EV_F64_EVENTS takes no time-event, f32-record or dt-side-plane companion."""
    from poseestimationkf_amd._lib import EV_F32_RECORDS, EV_F64_EVENTS, EV_TIME_EVENTS, PekfError, lib, check
    K, E = 8, 30
    ev = synth.generate_events(np.arange(K), E, seed=9)
    with pytest.raises(ValueError, match="FP64 events make FP64 records"):
        eng.BatchedEKF(K).run_events(ev, records="f32", events="f64")
    buf = eng.DeviceBuffer(32 * K * E)
    st = eng.DeviceBuffer(4096)
    f = eng.BatchedEKF(K)
    for fl in (EV_F64_EVENTS | EV_TIME_EVENTS, EV_F64_EVENTS | EV_F32_RECORDS):
        with pytest.raises(PekfError, match="PEKF_EV_F64_EVENTS"):
            check(lib.pekf_live_ext_dev(K, E, buf.ptr, st.ptr, st.ptr, 0.1, f.X.ptr, f.P.ptr, 1.0, 0.1, st.ptr,
                                        st.ptr, fl, None, None))
    with pytest.raises(PekfError, match="FP64 events"):
        check(lib.pekf_frontend_ext_dev(K, E, buf.ptr, st.ptr, st.ptr, 0.1, 10, buf.ptr, buf.ptr, buf.ptr, st.ptr,
                                        st.ptr, st.ptr, EV_F64_EVENTS, None, None))
