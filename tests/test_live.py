"""The front-end fused into the filter (pekf_live_dev): raw phone events -> records ->
Prediction + Correction in one launch, no record window.

Two record precisions (pekf_live_ext_dev's PEKF_EV_F32_RECORDS):
* f32 records (the 40 B stream record): bit for bit against the split pipeline it replaces
  (pekf_frontend_dev writing the records, pekf_run_dev with counts applying them), and against the
  oracle chain on f32-rounded records (oracle/frontend_numpy.py -> the C oracle filter);
* FP64 records (the default, what the server's filter receives: KFS/KalmanFilter.cpp:279-303) against
  the unrounded oracle chain (oracle/frontend_numpy.py float64 records -> oracle/ekf_numpy.py, the
  reference's own arithmetic), where the f32 records' rounding shows as ~1e-8 (measured, asserted).
The oracle's front-end half is partly pinned (see tests/test_frontend.py)."""
import numpy as np
import pytest

from poseestimationkf_amd import synth

from .test_frontend import _events, _oracle_records

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    return engine


def _split(eng, ev, K, X0=None, P0=None):
    win, counts = eng.run_frontend(ev)
    f = eng.BatchedEKF(K)
    if X0 is not None:
        f.set_state(X0, P0)
    if counts.max(initial=0) > 0:  # >= 2 steps: the multi-record kernel (one record takes the online kernel)
        f.run(win, n_steps=max(2, int(counts.max())))
    X, P = f.get_state()
    return X, P, counts, win.refs.download((K, 6), np.float64)


def _fused(eng, ev, K, X0=None, P0=None, records="f32", events="f32"):
    """pekf_live_ext_dev; f32 records by default here: the split pipeline's, for bit-for-bit checks."""
    f = eng.BatchedEKF(K)
    if X0 is not None:
        f.set_state(X0, P0)
    counts, refs = f.run_events(ev, records=records, events=events)
    X, P = f.get_state()
    return X, P, counts, refs


def _same(a, b):
    for u, v in zip(a, b):
        assert np.array_equal(u, v, equal_nan=True)


@pytest.mark.parametrize("K,E,seed", [(1000, 1500, 21), (64, 37, 22), (4096, 300, 23), (512, 200, 27)])
def test_live_equals_split_pipeline_bit_for_bit(eng, K, E, seed):
    """Ragged record counts, a partial last wave (K = 1000), event counts that are no multiple of the
    3-event ring (E = 37, 200: the last block padded with 2 or 1 null events) and short streams where the
    end-of-stream drain does most of the steps."""
    ev = synth.generate_events(np.arange(K), E, seed=seed)
    fused, split = _fused(eng, ev, K), _split(eng, ev, K)
    assert fused[2].min() >= 0 and fused[2].max() > 0
    _same(fused, split)


def test_live_continues_from_a_given_state(eng):
    """Not from reset: random unit X and SPD P going in, as a filter resumed from a checkpoint."""
    K, E = 512, 400
    rng = np.random.default_rng(5)
    X0 = rng.standard_normal((K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    A = rng.standard_normal((K, 4, 4)) * 0.3
    P0 = A @ A.transpose(0, 2, 1) + 0.5 * np.eye(4)
    ev = synth.generate_events(np.arange(K), E, seed=24)
    _same(_fused(eng, ev, K, X0, P0), _split(eng, ev, K, X0, P0))


def _oracle_chain_f64(ev, k, refs, X0=None, P0=None, server=False):
    """Filter k's float64 records from the front-end restatement, through the NumPy restatement of
    main_file.py's loop (bit-identical to the reference) with the device's reference pair.
    server=True: the front-end is fed the server's own sample values (std::stod of the phone's
    Float.toString text, wire.server_values) instead of the floats widened."""
    from oracle import ekf_numpy
    g, dt, a, m = _oracle_records(ev, k, server=server)
    X, _, _ = ekf_numpy.run_filter(g, dt.astype(np.float64), a, m, refs[k, :3], refs[k, 3:], X0=X0, P0=P0,
                                   record=False)
    return X, len(dt)


# FP64 records vs the unrounded oracle chain: the fused kernel's FP64 arithmetic (reference basis,
# closed-form polar Wahba) against the reference's (SVD), ~1e-14 measured over ~100 records
ATOL_F64_CHAIN = 1e-12
# f32 records vs the same unrounded chain: the records' f32 rounding (measured 1.4e-8 on seed 25's
# sampled filters, 5.3e-8 on 24 filters in round 4's review), within the north_star's 1e-5
ATOL_F32_ROUNDING = 1e-7
# f32 EVENTS vs the chain fed the server's own values (std::stod of the phone's text): the samples
# differ by up to half an f32 ulp (records ~1e-7), final X ~1e-8 (7.5e-9 in round 5's review, 4.7e-9 on
# 6 filters x 400 events in tests/test_wire.py); within the north_star's 1e-5
ATOL_F32_EVENTS = 1e-7


def test_live_vs_oracle_chain(eng, oracle_c):
    """Each filter's own records (ragged) through the oracle front-end and the oracle filter: f32 records
    against the C oracle on the same f32-rounded records (1e-9), and against the unrounded chain (the
    rounding, <= ATOL_F32_ROUNDING); FP64 records against the unrounded chain (<= ATOL_F64_CHAIN)."""
    K, E = 256, 1200
    ev = synth.generate_events(np.arange(K), E, seed=25)
    X, _, counts, refs = _fused(eng, ev, K, records="f32")
    X64, _, counts64, refs64 = _fused(eng, ev, K, records="f64")
    assert np.array_equal(counts, counts64) and np.array_equal(refs, refs64)
    worst = worst_round = worst64 = 0.0
    for k in range(0, K, 23):
        g, dt, a, m = _oracle_records(ev, k)
        assert counts[k] == len(dt)
        rec = synth.Records(g[:, None].astype(np.float32), a[:, None].astype(np.float32),
                            m[:, None].astype(np.float32), dt[:, None].astype(np.uint32),
                            refs[k:k + 1, :3], refs[k:k + 1, 3:])
        Xo, _, _ = oracle_c.run(rec)
        worst = max(worst, float(np.abs(X[k] - Xo[0]).max()))
        Xu, _ = _oracle_chain_f64(ev, k, refs)
        worst_round = max(worst_round, float(np.abs(X[k] - Xu).max()))
        worst64 = max(worst64, float(np.abs(X64[k] - Xu).max()))
    print("fused events -> filter: f32 records vs the f32 oracle chain %.3e, vs the unrounded chain %.3e; "
          "FP64 records vs the unrounded chain %.3e" % (worst, worst_round, worst64))
    assert worst < 1e-9
    assert worst_round < ATOL_F32_ROUNDING
    assert worst64 < ATOL_F64_CHAIN


def test_live_f64_records_full_batch_sampled(eng):
    """FP64 records at full scale (1,048,576 filters x 192 events, 16,384 streams tiled x64): sampled
    filters against the unrounded oracle chain, and every filter within the f32 rounding of the f32-record
    run (same counts and reference pairs)."""
    K0, E, tile = 16384, 192, 64
    ev0 = synth.generate_events(np.arange(K0), E, seed=26)
    ev = dict(types=np.tile(ev0["types"], (1, tile)), values=np.tile(ev0["values"], (1, tile, 1)),
              times=np.tile(ev0["times"], (1, tile)), init_acc=np.tile(ev0["init_acc"], (tile, 1)),
              init_mag=np.tile(ev0["init_mag"], (tile, 1)), t_init=np.tile(ev0["t_init"], tile))
    K = K0 * tile
    X64, _, c64, r64 = _fused(eng, ev, K, records="f64")
    X32, _, c32, r32 = _fused(eng, ev, K, records="f32")
    assert np.array_equal(c64, c32) and np.array_equal(r64, r32) and c64.sum() > 10 * K
    assert np.isfinite(X64).all() and float(np.abs(X64 - X32).max()) < ATOL_F32_ROUNDING
    worst = 0.0
    for k in (0, 1, 4095, K0 - 1, K0, 7 * K0 + 77, K - 1):
        Xu, n = _oracle_chain_f64(ev0, k % K0, r64)      # tiled: filter k runs stream k % K0
        assert c64[k] == n
        worst = max(worst, float(np.abs(X64[k] - Xu).max()))
    print("FP64 records, 1M filters: sampled vs the unrounded chain %.3e" % worst)
    assert worst < ATOL_F64_CHAIN


def test_live_f64_records_across_escaped_gaps(eng):
    """FP64 records whose dt does not fit the dt word (3 x (2^30 - 1) ns apart: escaped, the float64 dt
    in the LdsQueue64 side entry), from a resumed state, against the unrounded oracle chain."""
    K = 64
    g = (1 << 30) - 1
    spec = [(synth.EV_GYRO, g), (synth.EV_GYRO, g), (synth.EV_GYRO, g), (synth.EV_ACC, 10), (synth.EV_MAG, 10)] * 5
    ev = _events(K, spec)
    rng = np.random.default_rng(9)
    X0 = rng.standard_normal((K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.tile(np.eye(4) * 0.4, (K, 1, 1))
    X, _, counts, refs = _fused(eng, ev, K, X0, P0, records="f64")
    assert np.all(counts == 5)
    worst = 0.0
    for k in range(0, K, 7):
        Xu, _ = _oracle_chain_f64(ev, k, refs, X0[k], P0[k])
        worst = max(worst, float(np.abs(X[k] - Xu).max()))
    print("FP64 records across escaped gaps vs the unrounded chain: %.3e" % worst)
    assert worst < ATOL_F64_CHAIN


def test_live_streams_without_records_leave_the_state(eng):
    K = 70
    rng = np.random.default_rng(6)
    X0 = rng.standard_normal((K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.tile(np.eye(4) * 0.7, (K, 1, 1))
    for spec in ([], [(synth.EV_ACC, 10), (synth.EV_MAG, 10)] * 5,
                 [(synth.EV_GYRO, 10), (synth.EV_ACC, 10), (synth.EV_GYRO, 10)] * 3):
        X, P, counts, _ = _fused(eng, _events(K, spec), K, X0, P0)
        assert np.all(counts == 0)
        assert np.array_equal(X, X0) and np.array_equal(P, P0)


def test_live_lockstep_streams(eng):
    """Every lane completes its records on the same events (one record per 3 events: the densest
    stream, so every block pushes the most records a queue must hold)."""
    K = 192
    spec = [(synth.EV_GYRO, 1000), (synth.EV_ACC, 1000), (synth.EV_MAG, 1000)] * 40
    ev = _events(K, spec)
    fused = _fused(eng, ev, K)
    assert np.all(fused[2] == 40)
    _same(fused, _split(eng, ev, K))


def test_live_applies_a_dt_past_31_bits(eng):
    """Records 3 x (2^30 - 1) ns apart (dt past the 31-bit word: escaped, the float64 dt kept in the
    queue's side entry) apply exactly as the split pipeline's (side plane + pekf_run_ext_dev)."""
    K = 4
    g = (1 << 30) - 1
    spec = [(synth.EV_GYRO, g), (synth.EV_GYRO, g), (synth.EV_GYRO, g), (synth.EV_ACC, 10), (synth.EV_MAG, 10)] * 3
    fused, split = _fused(eng, _events(K, spec), K), _split(eng, _events(K, spec), K)
    assert np.all(fused[2] == 3)
    _same(fused, split)
    with pytest.raises(ValueError, match="FP64 filter on AoS"):
        eng.BatchedEKF(K, layout="soa").run_events(_events(K, spec))


def test_live_full_batch_equals_split(eng):
    """1,048,576 filters (16,384 generated event streams tiled x64) x 192 events: every filter's
    final state, count and reference pair equal the split pipeline's bit for bit at full scale."""
    K0, E, tile = 16384, 192, 64
    ev0 = synth.generate_events(np.arange(K0), E, seed=26)
    ev = dict(types=np.tile(ev0["types"], (1, tile)), values=np.tile(ev0["values"], (1, tile, 1)),
              times=np.tile(ev0["times"], (1, tile)), init_acc=np.tile(ev0["init_acc"], (tile, 1)),
              init_mag=np.tile(ev0["init_mag"], (tile, 1)), t_init=np.tile(ev0["t_init"], tile))
    K = K0 * tile
    fused, split = _fused(eng, ev, K), _split(eng, ev, K)
    assert fused[2].sum() > 10 * K
    _same(fused, split)


def test_session_phase2_then_fused_phase3(eng):
    """engine.run_session (phase 2 on the device, its means and time handed to pekf_live_dev in device
    memory) equals frontend_init -> run_frontend -> BatchedEKF.run bit for bit."""
    K = 320
    ph2 = synth.generate_events(np.arange(K), 800, seed=33)
    ph3 = synth.generate_events(np.arange(K), 500, seed=34)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    f = eng.BatchedEKF(K)
    got = eng.run_session(ph2, ph3, f, records="f32")
    assert got["ready"].all()
    ini = eng.frontend_init(ph2)
    assert np.array_equal(ini["t_init"], ph2["times"][-1])
    ev3 = dict(ph3, t_init=ini["t_init"], init_acc=ini["init"][:, :3], init_mag=ini["init"][:, 3:])
    split = _split(eng, ev3, K)
    X, P = f.get_state()
    _same((X, P, got["counts"], got["refs"]), split)
    # the default FP64 records: the session equals the fused launch on the same phase-2 results
    f64 = eng.BatchedEKF(K)
    got64 = eng.run_session(ph2, ph3, f64)
    _same(f64.get_state() + (got64["counts"], got64["refs"]), _fused(eng, ev3, K, records="f64"))


def test_session_leaves_filters_that_never_got_ready(eng):
    """Filters whose phase 2 never completed (pekf_frontend_init_dev: not ready, NaN means) apply no
    phase-3 record: counts 0 and their state untouched (not overwritten with NaN); the ready ones equal
    the split pipeline run on them alone."""
    K = 384
    ph2 = synth.generate_events(np.arange(K), 520, seed=36)     # about a third never get ready
    ph3 = synth.generate_events(np.arange(K), 400, seed=37)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    rng = np.random.default_rng(38)
    X0 = rng.standard_normal((K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.tile(np.eye(4) * 0.3, (K, 1, 1))
    f = eng.BatchedEKF(K)
    f.set_state(X0, P0)
    got = eng.run_session(ph2, ph3, f, records="f32")
    ready = got["ready"]
    assert 0 < ready.sum() < K
    X, P = f.get_state()
    assert np.all(got["counts"][~ready] == 0)
    assert np.array_equal(X[~ready], X0[~ready]) and np.array_equal(P[~ready], P0[~ready])
    assert np.all(got["counts"][ready] > 0) and np.isfinite(X[ready]).all()
    ini = eng.frontend_init(ph2)
    ev = dict(ph3, t_init=ini["t_init"], init_acc=ini["init"][:, :3], init_mag=ini["init"][:, 3:])
    Xs, Ps, cs, _ = _split(eng, ev, K, X0, P0)
    assert np.all(cs[~ready] == 0)                               # the split front-end skips them too
    assert np.array_equal(X, Xs) and np.array_equal(P, Ps)


def test_live_dense_jittered_streams(eng):
    """Records every 3-6 events at lane-dependent positions (each group of three events a random
    permutation of gyro / acc / mag): the queues fill fastest and the overflow rule decides most
    filter steps."""
    K, G = 448, 200
    rng = np.random.default_rng(35)
    perms = np.array([[0, 1, 2], [0, 2, 1], [1, 0, 2], [1, 2, 0], [2, 0, 1], [2, 1, 0]])
    kinds = np.array([synth.EV_GYRO, synth.EV_ACC, synth.EV_MAG], np.uint32)
    types = kinds[perms[rng.integers(0, 6, size=(G, K))]].transpose(0, 2, 1).reshape(3 * G, K)
    E = 3 * G
    gaps = rng.integers(1_000_000, 3_000_000, size=(E, K))
    times = synth.T_INIT_NS + np.cumsum(gaps, axis=0)
    vals = rng.standard_normal((E, K, 3)).astype(np.float32)
    vals[..., 2] += np.where(types == synth.EV_ACC, 9.8, 0.0).astype(np.float32)
    ev = dict(types=types, values=vals, times=times, init_acc=np.tile([0.1, 0.2, 9.8], (K, 1)),
              init_mag=np.tile([20.0, 1.0, -40.0], (K, 1)), t_init=np.full(K, synth.T_INIT_NS, np.int64))
    fused = _fused(eng, ev, K)
    assert fused[2].min() >= G // 2 and fused[2].max() <= G
    _same(fused, _split(eng, ev, K))


# ------------------------------------------------------------------ FP64 events (PEKF_EV_F64_EVENTS)

def test_live_fp64_events_vs_the_servers_values(eng):
    """The server's own input values end to end: FP64 events carrying std::stod of the phone's text
    (wire.server_values) -> k_live -> X within ATOL_F64_CHAIN of the oracle chain fed the same doubles.
    The f32 events (16 B, the float itself) against that same chain: their distance is the f32 rounding
    of the SAMPLES, stated and bounded (ATOL_F32_EVENTS) -- the chain fed (double)f cannot see it."""
    K, E = 256, 1200
    ev = synth.generate_events(np.arange(K), E, seed=25)
    X64, _, c64, r64 = _fused(eng, ev, K, records="f64", events="f64")
    X32, _, c32, r32 = _fused(eng, ev, K, records="f64")
    assert np.array_equal(c64, c32) and np.array_equal(r64, r32)
    worst64 = worst32 = 0.0
    for k in range(0, K, 23):
        Xs, n = _oracle_chain_f64(ev, k, r64, server=True)
        assert c64[k] == n
        worst64 = max(worst64, float(np.abs(X64[k] - Xs).max()))
        worst32 = max(worst32, float(np.abs(X32[k] - Xs).max()))
    print("FP64 events vs the server-value chain %.3e; f32 events vs it %.3e" % (worst64, worst32))
    assert worst64 < ATOL_F64_CHAIN
    assert 1e-12 < worst32 < ATOL_F32_EVENTS


def _split64(eng, ev, K, X0=None, P0=None):
    win, counts = eng.run_frontend(ev, events="f64")
    f = eng.BatchedEKF(K)
    if X0 is not None:
        f.set_state(X0, P0)
    if counts.max(initial=0) > 0:
        f.run(win, n_steps=max(2, int(counts.max())))
    X, P = f.get_state()
    return X, P, counts, win.refs.download((K, 6), np.float64)


@pytest.mark.parametrize("K,E,seed", [(1000, 1500, 41), (64, 37, 42), (512, 200, 43)])
def test_live_fp64_events_equal_the_fp64_split_pipeline(eng, K, E, seed):
    """FP64 events fused (k_live) = the FP64 split pipeline (k_frontend writing FP64 records, then
    pekf_run_rec64_dev with counts) bit for bit: the same records, applied with the same arithmetic."""
    ev = synth.generate_events(np.arange(K), E, seed=seed)
    _same(_fused(eng, ev, K, records="f64", events="f64"), _split64(eng, ev, K))


def test_live_fp64_events_any_gap_and_clock_step(eng):
    """FP64 events carry absolute times, so pauses past 2^30 / 2^31 ns, a clock stepping back and
    zero gaps need no time events or escapes: against the server-value oracle chain, from a resumed
    state, and equal to the FP64 split pipeline.  (The stream opens with an acc and a mag sample: a first
    record interpolated from the phase-2 means 1 us into a 2 s gap lands within 1e-7 of the reference
    pair, an all-but-identity rotation where the reference's R->q divides by sqrt of rounding noise and
    its own two restatements disagree by 2e-2 -- ill-posed, DESIGN.md §2.  With the lead-in the NumPy and
    C restatements agree to 6e-15.)"""
    K = 64
    g = (1 << 31) + 12345
    spec = [(synth.EV_ACC, 1_000_000), (synth.EV_MAG, 1_000_000)] + [
        (synth.EV_GYRO, 1000), (synth.EV_ACC, g), (synth.EV_MAG, 10), (synth.EV_GYRO, -5_000_000),
        (synth.EV_ACC, 700), (synth.EV_MAG, 0), (synth.EV_GYRO, 3 * g), (synth.EV_ACC, 10), (synth.EV_MAG, 10)] * 4
    ev = _events(K, spec)
    rng = np.random.default_rng(44)
    X0 = rng.standard_normal((K, 4))
    X0 /= np.linalg.norm(X0, axis=1, keepdims=True)
    P0 = np.tile(np.eye(4) * 0.4, (K, 1, 1))
    got = _fused(eng, ev, K, X0, P0, records="f64", events="f64")
    assert np.all(got[2] == 12)
    worst = 0.0
    for k in range(0, K, 7):
        Xs, _ = _oracle_chain_f64(ev, k, got[3], X0[k], P0[k], server=True)
        worst = max(worst, float(np.abs(got[0][k] - Xs).max()))
    print("FP64 events across long / negative gaps vs the server-value chain: %.3e" % worst)
    assert worst < ATOL_F64_CHAIN
    _same(got, _split64(eng, ev, K, X0, P0))


def test_live_fp64_events_full_batch(eng):
    """1,048,576 filters (16,384 streams tiled x64) x 192 FP64 events: sampled filters against the
    server-value chain, and every filter within ATOL_F32_EVENTS of the f32-event run."""
    K0, E, tile = 16384, 192, 64
    ev0 = synth.generate_events(np.arange(K0), E, seed=26)
    ev = dict(types=np.tile(ev0["types"], (1, tile)), values=np.tile(ev0["values"], (1, tile, 1)),
              times=np.tile(ev0["times"], (1, tile)), init_acc=np.tile(ev0["init_acc"], (tile, 1)),
              init_mag=np.tile(ev0["init_mag"], (tile, 1)), t_init=np.tile(ev0["t_init"], tile))
    K = K0 * tile
    X64, _, c64, r64 = _fused(eng, ev, K, records="f64", events="f64")
    X32, _, c32, _ = _fused(eng, ev, K, records="f64")
    assert np.array_equal(c64, c32) and c64.sum() > 10 * K
    assert np.isfinite(X64).all() and float(np.abs(X64 - X32).max()) < ATOL_F32_EVENTS
    worst = 0.0
    for k in (0, 1, 4095, K0 - 1, K0, 7 * K0 + 77, K - 1):
        Xs, n = _oracle_chain_f64(ev0, k % K0, r64, server=True)
        assert c64[k] == n
        worst = max(worst, float(np.abs(X64[k] - Xs).max()))
    print("FP64 events, 1M filters: sampled vs the server-value chain %.3e" % worst)
    assert worst < ATOL_F64_CHAIN


def test_session_fp64_events(eng):
    """engine.run_session with FP64 events: phase 2 averages the server's values (pekf_frontend_init_ext_dev)
    and phase 3 runs fused on them; equal to frontend_init(events="f64") -> the fused launch, and the
    phase-2 means equal the restatement's on the server's values bit for bit."""
    from oracle import frontend_numpy as fe
    from poseestimationkf_amd import wire
    K = 320
    ph2 = synth.generate_events(np.arange(K), 800, seed=33)
    ph3 = synth.generate_events(np.arange(K), 500, seed=34)
    ph3 = dict(ph3, times=ph3["times"] - ph3["t_init"][None, :] + ph2["times"][-1][None, :])
    f = eng.BatchedEKF(K)
    got = eng.run_session(ph2, ph3, f, events="f64")
    assert got["ready"].all()
    ini = eng.frontend_init(ph2, events="f64")
    v2 = wire.server_values(ph2["values"])
    for k in (0, 5, K - 1):
        o = fe.initial_values(ph2["types"][:, k], v2[:, k], ph2["times"][:, k])
        assert np.array_equal(ini["init"][k], np.array(o["acc"] + o["mag"])) and ini["t_init"][k] == o["t_init"]
    ev3 = dict(ph3, t_init=ini["t_init"], init_acc=ini["init"][:, :3], init_mag=ini["init"][:, 3:])
    _same(f.get_state() + (got["counts"], got["refs"]), _fused(eng, ev3, K, records="f64", events="f64"))


def test_live_from_wire_text(eng):
    """The phone's text through the server's parse (wire.events_from_wire: pekf_wire_parse) into FP64
    events: the same launch as the packer's server values of the same floats, bit for bit, with ragged
    streams padded by no-sample events."""
    from poseestimationkf_amd import wire
    K, E = 96, 300
    ev = synth.generate_events(np.arange(K), E, seed=45)
    n = [E - (k % 5) * 20 for k in range(K)]
    texts = [wire.events_text(ev["types"][:n[k], k], ev["values"][:n[k], k], ev["times"][:n[k], k]) for k in range(K)]
    evw = wire.events_from_wire(texts, ev["init_acc"], ev["init_mag"], ev["t_init"])
    got = _fused(eng, evw, K, records="f64", events="f64")
    cut = dict(ev, types=np.where(np.arange(E)[:, None] < np.array(n)[None, :], ev["types"], 3))
    want = _fused(eng, cut, K, records="f64", events="f64")
    _same(got, want)
    assert got[2].min() > 0
