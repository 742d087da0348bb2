"""Any float64 time difference the reference accepts, on every stream path (VERDICT r2 "missing" #3).

The reference forms dt = T - previousT in float64 (ExtendedKalmanFilter.py:62) and takes whatever
it gets: a pause of seconds, a clock that steps back, a fractional difference.  The 40 B record
carries dt as a 31-bit ns count, so such a record's dt word is the escape (PEKF_DT_ESCAPE) and its
float64 dt sits in the window's side plane (include/pekf.h); raw phone events carry a 30-bit gap,
so a longer or negative gap is a time event (word 3, the float64 step in x / y).

Pinned by tests/golden/gaps.npz, which tests/golden/make_gaps_golden.py made by running the reference's
own KalmanFilter over streams with such differences (5 s and 33 s pauses, negative and fractional
differences, 2^31 - 1 and 2^31 ns exactly).  CPU: the packing round trips, the NumPy restatement
reproduces the reference bit for bit and the C oracle within 1e-10 on those records.  GPU: the
per-record drop-in loop (the per-call kernels, dt = T - previousT) and the fused
kernel (multi-record, trajectory, counts, one-record and handle launches) against the reference's
trajectories and the oracles, the front-end, the fused front-end + filter kernel and phase 2 against
the oracles."""
import numpy as np
import pytest

from oracle import ekf_numpy
from oracle import frontend_numpy as fe
from poseestimationkf_amd import synth

from .test_frontend import _oracle_records

ODD_DTS = [5e9, -2e7, 1e7 + 0.5, float(0x7FFFFFFF), 3.3e10, 0.0]


def _escaped_records(K=256, W=64, seed=41):
    """A synthetic window with odd dts at scattered (row, filter) places, escaped into dtx."""
    rec = synth.generate(np.arange(K), W, seed=seed)
    dt = rec.dt_ns.copy()
    rng = np.random.default_rng(seed)
    for i, (r, k) in enumerate(zip(rng.integers(0, W, 40), rng.integers(0, K, 40))):
        dt[r, k] = ODD_DTS[i % len(ODD_DTS)]
    dt[:, 5] = 5e9                                        # one filter with a pause on every record
    return with_dts(rec, dt)


def with_dts(rec, dt):
    fits = (dt >= 0) & (dt < synth.DT_ESCAPE) & (dt == np.floor(dt))
    field = np.where(fits, dt, synth.DT_ESCAPE).astype(np.uint32)
    dtw = (rec.dtw & np.uint32(synth.MISSING_BIT)) | field
    return synth.Records(rec.gyro, rec.acc, rec.mag, dtw, rec.acc0, rec.mag0, np.where(fits, 0.0, dt))


def _decode_events(planes, t_init):
    """Host decoder of an event plane: per filter, the (type, time) of its sample events."""
    words = np.ascontiguousarray(planes[..., 3]).view(np.uint32)
    out = []
    for k in range(planes.shape[1]):
        t, evs = int(t_init[k]), []
        for e in range(planes.shape[0]):
            w = int(words[e, k])
            if w == synth.EV_TIME:
                t += int(planes[e, k, :2].copy().view(np.float64)[0])
            else:
                t += w >> 2
                evs.append((w & 3, t))
        out.append(evs)
    return out


def test_pack_events_time_events_round_trip():
    K, E = 6, 40
    ev = synth.generate_events(np.arange(K), E, seed=3)
    t = ev["times"].copy()
    t[10:, 1] += 5_000_000_000          # a 5 s pause
    t[20:, 3] -= 700_000_000            # the clock steps back 0.7 s
    t[5:, 4] += 2_000_000_000           # two pauses on one filter
    t[30:, 4] += 1 << 30
    ev = dict(ev, times=t)
    planes = synth.pack_events(ev)
    assert planes.shape[0] == E + 2 and synth.has_time_events(planes)
    got = _decode_events(planes, ev["t_init"])
    for k in range(K):
        assert got[k] == [(int(ev["types"][e, k]), int(t[e, k])) for e in range(E)]
    assert not synth.has_time_events(synth.pack_events(synth.generate_events(np.arange(K), E, seed=3)))


def test_pack_events_other_and_none_round_trip():
    """A message no sensor takes (EV_OTHER) keeps its time and stays a message -- also at the previous
    event's time and after a long pause, where word 3 would read as a time event (it goes after a time
    event of gap - 1 ns, with a gap field of 1) --; no message (EV_NONE) only moves the clock.  FP64 events:
    EV_OTHER is type 3 at its time, EV_NONE the -0.0 sentinel."""
    K, E = 5, 30
    ev = synth.generate_events(np.arange(K), E, seed=5)
    ty, t = ev["types"].copy(), ev["times"].copy()
    ty[3, 0] = synth.EV_OTHER
    ty[7, 1] = synth.EV_OTHER
    t[7:, 1] -= t[7, 1] - t[6, 1]                      # at the previous event's time: gap 0
    ty[9, 2] = synth.EV_OTHER
    t[9:, 2] += 3 << 30                                 # after a pause the gap field cannot hold
    ty[0, 3] = synth.EV_OTHER                           # the first event, at t_init
    t[:, 3] -= t[0, 3] - ev["t_init"][3]
    ty[E - 6:, 3] = synth.EV_NONE                       # padding
    ty[10, 4] = synth.EV_NONE
    t[10:, 4] += 5 << 30                                # a no-message clock step past the gap field
    ev = dict(ev, types=ty, times=t)
    planes = synth.pack_events(ev)
    got = _decode_events(planes, ev["t_init"])
    for k in range(K):
        assert got[k] == [(int(ty[e, k]), int(t[e, k])) for e in range(E) if ty[e, k] != synth.EV_NONE]
    p64 = synth.pack_events64(ev)
    w = np.ascontiguousarray(p64[..., 3]).view(np.uint64)
    none = ty == synth.EV_NONE
    assert np.all(w[none] == np.uint64(synth.EV64_NONE_W)) and np.all(p64[none][:, :3] == 0)
    assert np.array_equal(w[~none] & np.uint64(3), ty[~none].astype(np.uint64))
    assert np.array_equal((w[~none] & ~np.uint64(3)).view(np.float64), t[~none].astype(np.float64))
    with pytest.raises(ValueError, match="event types"):
        synth.pack_events(dict(ev, types=np.full_like(ty, 5)))


def test_records_dt_ns_and_oracles_agree_on_escapes(oracle_c):
    rec = _escaped_records(K=16, W=40)
    dt = rec.dt_ns
    assert (rec.dtw & np.uint32(synth.DT_MASK) == synth.DT_ESCAPE).sum() > 10
    assert dt[0, 5] == 5e9 and np.isin(ODD_DTS, dt).sum() >= 4
    Xo, Po, _ = oracle_c.run(rec)
    for k in (0, 5, 9):
        g, d, a, m = rec.filter(k)
        Xn, Pn = ekf_numpy.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k], record=False)[:2]
        assert np.abs(Xn - Xo[k]).max() < 1e-10


def _golden():
    import os

    from .conftest import GOLDEN
    with np.load(os.path.join(GOLDEN, "gaps.npz")) as z:
        d = {k: z[k] for k in z}
    base = synth.Records(d["gyro"], d["acc"], d["mag"], np.zeros(d["dt"].shape, np.uint32), d["acc0"], d["mag0"])
    return with_dts(base, d["dt"]), d


def test_golden_gaps_pin_the_oracles(oracle_c):
    """The reference's own trajectories over odd time differences: the NumPy restatement bit for bit,
    the C oracle (escaped records from the side plane) within 1e-10."""
    rec, d = _golden()
    assert (rec.dtw & np.uint32(synth.DT_MASK) == synth.DT_ESCAPE).sum() >= 300 + 5 * 12 // 2
    assert np.array_equal(rec.dt_ns, d["dt"])
    for k in range(rec.dtw.shape[1]):
        g, dt, a, m = rec.filter(k)
        _, _, tr = ekf_numpy.run_filter(g, dt, a, m, rec.acc0[k], rec.mag0[k])
        assert np.array_equal(tr, d["traj"][:, k]), k
    _, _, tro = oracle_c.run(rec, want_traj=True)
    assert np.abs(tro.transpose(1, 0, 2) - d["traj"]).max() < 1e-10


# ------------------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _err(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max())


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_fused_escapes_match_the_reference_trajectories(eng, layout):
    """tests/golden/gaps.npz through the fused kernel: every record's X within 1e-9 of the reference's,
    from the multi-record launch (trajectory variant) and from one-record launches alike."""
    rec, d = _golden()
    K = rec.dtw.shape[1]
    win = eng.IMUWindow.from_records(rec)
    tr = eng.BatchedEKF(K, layout=layout).run(win, want_traj=True)
    err = _err(tr, d["traj"])
    f1 = eng.BatchedEKF(K, layout=layout)
    for t in range(40):
        f1.run(win, n_steps=1, step0=t)
    err1 = _err(f1.get_state()[0], d["traj"][39])
    print("escaped dts vs the reference (%s): max |dq| = %.3e (multi-record), %.3e (one-record)" % (layout, err, err1))
    assert err < 1e-9 and err1 < 1e-9


@pytest.mark.gpu
def test_dropin_loop_over_odd_time_differences(eng, monkeypatch):
    """The per-record drop-in (main_file.py's loop through dropin/ExtendedKalmanFilter.py) on the golden
    streams, with the absolute timestamps the reference saw: pauses, a clock stepping back, fractional
    differences reach the per-call kernels as T - previousT, and every X matches the reference's."""
    import os
    import sys

    from .conftest import ROOT
    rec, d = _golden()
    monkeypatch.syspath_prepend(os.path.join(ROOT, "poseestimationkf_amd", "dropin"))
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "_bootstrap"):
        sys.modules.pop(m, None)
    from ExtendedKalmanFilter import KalmanFilter
    W, K = d["dt"].shape
    err = 0.0
    for k in (1, 3, 5):   # filter 3 pauses 5 s before every record
        kf = KalmanFilter(d["t0"][k], d["mag0"][k], d["acc0"][k], 0.5)
        kf.setQ(1)
        kf.setR(0.1)
        X, P, T = np.asarray([1., 0., 0., 0.]), np.identity(4), d["t0"][k]
        for i in range(W):
            T = T + d["dt"][i, k]
            z, Pm, Kk = kf.Prediction(d["gyro"][i, k].astype(np.float64), T, X, P)
            X, P = kf.Correction(d["mag"][i, k].astype(np.float64), d["acc"][i, k].astype(np.float64), z, Pm, Kk)
            err = max(err, _err(X, d["traj"][i, k]))
    for m in ("ExtendedKalmanFilter", "Wahba", "UtilityFunctions", "_bootstrap"):
        sys.modules.pop(m, None)
    print("drop-in loop over odd time differences vs the reference: max |dq| = %.3e" % err)
    assert err < 1e-11


@pytest.mark.gpu
def test_fused_escapes_with_missing_magnetometer(eng, oracle_c):
    """Escaped dt words with the missing-magnetometer bit set (word 0xFFFFFFFF): the Wahba-skip rule and
    the side plane's dt apply together (config 5's stream with pauses)."""
    K, W = 512, 48
    rec = synth.generate(np.arange(K), W, seed=43, missing=True)
    dt = rec.dt_ns.copy()
    dt[::5, ::3] = 7.5e9
    dt[3::7, 1::4] = -4e6
    rec = with_dts(rec, dt)
    both = ((rec.dtw & np.uint32(synth.DT_MASK)) == synth.DT_ESCAPE) & rec.missing
    assert both.sum() > 100
    win = eng.IMUWindow.from_records(rec)
    f = eng.BatchedEKF(K)
    f.run(win, n_steps=90, step0=11)
    Xo, Po, _ = oracle_c.run(rec, n_steps=90, step0=11)
    X, P = f.get_state()
    assert _err(X, Xo) < 1e-9 and _err(P, Po) < 1e-9


@pytest.mark.gpu
def test_fused_run_with_escaped_dts(eng, oracle_c):
    """Every launch shape of the fused kernel reads escaped records' dt from the side plane."""
    rec = _escaped_records()
    K, W = rec.dtw.shape[1], rec.dtw.shape[0]
    win = eng.IMUWindow.from_records(rec)
    assert win.dtx is not None
    Xo, Po, tro = oracle_c.run(rec, n_steps=100, step0=7, want_traj=True)
    f = eng.BatchedEKF(K)                                     # multi-record launch, wraps the window
    f.run(win, n_steps=100, step0=7)
    X, P = f.get_state()
    assert _err(X, Xo) < 1e-9 and _err(P, Po) < 1e-9
    tr = eng.BatchedEKF(K).run(win, n_steps=100, step0=7, want_traj=True)   # trajectory variant
    assert _err(tr, tro.transpose(1, 0, 2)) < 1e-9
    cnt = np.arange(K) % 100                                  # ragged counts
    fc = eng.BatchedEKF(K)
    fc.run(win, n_steps=100, step0=7, counts=cnt)
    Xc, _ = fc.get_state()
    for k in (1, 5, 37, 99, 200):
        Xk, _, _ = oracle_c.run(synth.Records(*(a[:, k:k + 1] for a in (rec.gyro, rec.acc, rec.mag, rec.dtw)),
                                              rec.acc0[k:k + 1], rec.mag0[k:k + 1], rec.dtx[:, k:k + 1]),
                                n_steps=int(cnt[k]), step0=7)
        assert _err(Xc[k], Xk[0]) < 1e-9
    fo = eng.BatchedEKF(K)                                    # one-record launches (online serving)
    for t in range(12):
        fo.run(win, n_steps=1, step0=7 + t)
    X1, _ = fo.get_state()
    X1o, _, _ = oracle_c.run(rec, n_steps=12, step0=7)
    assert _err(X1, X1o) < 1e-9
    h = eng.FilterHandle(rec.acc0, rec.mag0)                  # the handle's stream path
    h.run(win, n_steps=30)
    Xh, _ = h.get_state()
    X30, _, _ = oracle_c.run(rec, n_steps=30)
    assert _err(Xh, X30) < 1e-9
    fm = eng.BatchedEKF(K, precision="mixed")                 # mixed precision: same records
    fm.run(win, n_steps=100, step0=7)
    assert _err(fm.get_state()[0], Xo) < 1e-5
    fs = eng.BatchedEKF(K, layout="soa")
    fs.run(win, n_steps=100, step0=7)
    assert np.array_equal(fs.get_state()[0], X)


def _paused_events(K, E, seed):
    ev = synth.generate_events(np.arange(K), E, seed=seed)
    t = ev["times"].copy()
    rng = np.random.default_rng(seed)
    for k in range(K):
        if k % 3 == 0:                          # a 5 s pause (records across it have dt > 2^31 ns)
            t[rng.integers(1, E):, k] += 5_000_000_000
        if k % 4 == 1:                          # the phone clock steps back 0.5 s
            t[rng.integers(1, E):, k] -= 500_000_000
        if k % 7 == 2:                          # a pause just over the 30-bit event field
            t[rng.integers(1, E):, k] += (1 << 30) + 12345
        if k % 5 == 3:                          # the very first event 4 s after t_init
            t[:, k] += 4_000_000_000
        if k % 11 == 6:                         # the very first event before t_init
            t[:, k] -= 30_000_000
    return dict(ev, times=t)


@pytest.mark.gpu
def test_frontend_records_across_pauses_and_clock_steps(eng):
    K, E = 192, 900
    ev = _paused_events(K, E, seed=51)
    win, counts = eng.run_frontend(ev)
    assert win.dtx is not None                                # some record needed the side plane
    rec = win.download_filters(np.arange(K))
    dt_dev = rec.dt_ns
    n_esc = 0
    for k in range(K):
        g, dt, a, m = _oracle_records(ev, k)
        r = len(dt)
        assert counts[k] == r
        assert np.array_equal(dt_dev[:r, k], dt.astype(np.float64))
        assert np.array_equal(rec.gyro[:r, k], g.astype(np.float32))
        n_esc += int(((rec.dtw[:r, k] & np.uint32(synth.DT_MASK)) == synth.DT_ESCAPE).sum())
    assert n_esc >= K // 3


@pytest.mark.gpu
def test_live_and_split_pipelines_across_pauses(eng, oracle_c):
    """k_live (time events + escaped records in its LDS queue) equals the split pipeline bit for bit,
    and both match the oracle chain."""
    from .test_live import _fused, _same, _split
    K, E = 320, 1000
    ev = _paused_events(K, E, seed=52)
    fused, split = _fused(eng, ev, K), _split(eng, ev, K)
    _same(fused, split)
    X, _, counts, refs = fused
    worst = 0.0
    for k in range(0, K, 9):
        g, dt, a, m = _oracle_records(ev, k)
        base = synth.Records(g[:, None].astype(np.float32), a[:, None].astype(np.float32),
                             m[:, None].astype(np.float32), np.zeros((len(dt), 1), np.uint32),
                             refs[k:k + 1, :3], refs[k:k + 1, 3:])
        Xo, _, _ = oracle_c.run(with_dts(base, dt[:, None].astype(np.float64)))
        worst = max(worst, _err(X[k], Xo[0]))
    print("events with pauses / clock steps -> filter vs oracle chain: max |dq| = %.3e" % worst)
    assert worst < 1e-9
    # FP64 records (the default) across the same pauses, against the unrounded oracle chain
    from .test_live import ATOL_F64_CHAIN, _oracle_chain_f64
    X64, _, c64, r64 = _fused(eng, ev, K, records="f64")
    assert np.array_equal(c64, counts) and np.array_equal(r64, refs)
    worst64 = max(float(np.abs(X64[k] - _oracle_chain_f64(ev, k, refs)[0]).max()) for k in range(0, K, 9))
    print("FP64 records across pauses vs the unrounded chain: %.3e" % worst64)
    assert worst64 < ATOL_F64_CHAIN


@pytest.mark.gpu
def test_phase2_with_pauses_and_clock_steps(eng):
    K, E = 200, 700
    ev = _paused_events(K, E, seed=53)
    got = eng.frontend_init(ev)
    for k in range(K):
        o = fe.initial_values(ev["types"][:, k], ev["values"][:, k], ev["times"][:, k])
        assert got["ready"][k] == o["ready"]
        if o["ready"]:
            assert got["t_init"][k] == o["t_init"]
            assert np.array_equal(got["init"][k], np.array(o["acc"] + o["mag"]))


@pytest.mark.gpu
def test_gyro_chain_reads_escaped_dts(eng):
    """The pure-gyro side output (KFS/KalmanFilter.cpp:149, RungeKutta4 of ExtendedKalmanFilter.py:25-41 on
    the gyro records alone) takes an escaped record's dt from the window's side plane, as the filter does:
    a 5 s pause or a clock stepping back integrates that dt, never the escape word's 2^31 - 1 ns."""
    from oracle import ekf_numpy as npo
    rec = _escaped_records(K=64, W=40)
    win = eng.IMUWindow.from_records(rec)
    assert win.dtx is not None
    qf, tr = win.gyro_chain(n_steps=50, step0=3, want_traj=True)   # wraps the 40-record window
    dt = rec.dt_ns
    err = 0.0
    for k in (0, 5, 17, 63):
        q = np.array([1.0, 0, 0, 0])
        for t in range(50):
            row = (3 + t) % 40
            q = npo.rk4(q, dt[row, k], rec.gyro[row, k].astype(np.float64))
            err = max(err, _err(tr[t, k], q))
    assert np.array_equal(qf, tr[-1])
    print("gyro chain over escaped dts vs the NumPy restatement: max |dq| = %.3e" % err)
    assert err < 1e-12
