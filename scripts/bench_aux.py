#!/usr/bin/env python3
"""Measurements of the kernels beside the headline fused run (one JSON object on stdout).

  frontend      pekf_frontend_dev: raw phone events -> records; HBM-bound:
                16 B read per event + 40 B written per record
  frontend_then_filter   the filter over those records (pekf_run_dev with counts): the split pipeline
  live          pekf_live_dev: the same events -> filter in one launch (no record window); 16 B read per
                event + the state once (PEKF_AUX_ONLY=live stops after it)
  gyro_chain    pekf_gyro_chain_dev (§8f-3): 16 B read per filter-record
  wahba_stream  pekf_wahba_stream_dev (§8f-3): 24 B read + 32 B written per filter-record
  predict_dev / correct_dev   per-call operators at n = 1M items (device pointers)
  online_step_aos / _soa   1M filters x 1 record per launch (state through HBM every launch)
  ctypes_call / dropin_call   host-pointer per-call latency at n = 1 via ctypes / via the CPython
                binding the drop-in modules use (the path main_file.py takes)
  c1_loop       config 1: main_file.py's loop over the committed log, drop-ins vs NumPy on the host

Kernel times are HIP events on the launch stream; run under rocprofv3 --kernel-trace --stats
for the per-kernel summary committed in profiles/.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from poseestimationkf_amd import engine, synth  # noqa: E402
from poseestimationkf_amd._lib import check, lib  # noqa: E402

HBM = 8000.0


def log(m):
    print("[aux] " + m, file=sys.stderr, flush=True)


def timed(fn, stream, reps=3):
    e0, e1 = engine.Event(), engine.Event()
    fn()
    check(lib.pekf_stream_sync(stream))
    out = []
    for _ in range(reps):
        e0.record(stream)
        fn()
        e1.record(stream)
        e1.sync()
        out.append(e0.elapsed_ms(e1))
    return float(np.median(out))


def c1_loop():
    """Config 1: main_file.py:38-46 over the committed 1,550-record log, once through the drop-in
    modules (GPU per-call kernels) and once through oracle/ekf_numpy.py (the NumPy restatement,
    bit-identical to the reference) on this host's CPU: microseconds per record."""
    import gzip
    import importlib
    import tempfile
    from oracle import ekf_numpy as npo
    golden = os.path.join(ROOT, "tests", "golden")
    with gzip.open(os.path.join(golden, "c1_log.txt.gz"), "rt") as fh:
        text = fh.read()
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as fh:
        fh.write(text)
    os.environ["PEKF_LOG_PATH"] = fh.name
    sys.path.insert(0, os.path.join(ROOT, "poseestimationkf_amd", "dropin"))
    ReadFile = importlib.import_module("ReadFile")
    EKF = importlib.import_module("ExtendedKalmanFilter")
    Wahba = importlib.import_module("Wahba")
    g = ReadFile.getData()
    os.unlink(fh.name)
    T = [t[0] for t in g.timestamp]
    n = len(g.acc_1)

    def dropin():
        w = Wahba.Wahba(g.acc_0, g.mag_0)
        k = EKF.KalmanFilter(T[0], g.mag_0, g.acc_0, 0.5)
        k.setQ(1)
        k.setR(0.1)
        X, P = np.asarray([1., 0., 0., 0.]), np.identity(4)
        for i in range(n):
            z, P, K = k.Prediction(g.gyro[i], T[i + 1], X, P)
            w.getQuarternion(g.acc_1[i], g.mag_1[i], 0.5, 0.5)
            X, P = k.Correction(g.mag_1[i], g.acc_1[i], z, P, K)
        return X

    def numpy_port():
        Q, R = np.identity(3), np.identity(4) * 0.1
        X, P, prev = np.asarray([1., 0., 0., 0.]), np.identity(4), T[0]
        a0, m0 = np.asarray(g.acc_0, float), np.asarray(g.mag_0, float)
        for i in range(n):
            z, P, K = npo.predict(np.asarray(g.gyro[i], float), T[i + 1] - prev, X, P, Q, R)
            prev = T[i + 1]
            npo.wahba_quat(a0, m0, np.asarray(g.acc_1[i], float), np.asarray(g.mag_1[i], float), 0.5, 0.5)
            X, P = npo.correct(np.asarray(g.mag_1[i], float), np.asarray(g.acc_1[i], float), z, P, K, a0, m0)
        return X

    out = {"records": n}
    for name, fn in (("dropin_gpu_us_per_record", dropin), ("numpy_port_cpu_us_per_record", numpy_port)):
        fn()
        t0 = time.perf_counter()
        X = fn()
        out[name] = (time.perf_counter() - t0) / n * 1e6
        out[name.replace("us_per_record", "final_X")] = X.tolist()
    return out


def main():
    st = engine.Stream()
    s = st.handle
    res = {}

    # ---- front-end: 16K generated event streams tiled x64 -> 1,048,576 filters x 1,024 events
    K0, E, tile = 16384, 1024, 64
    log("generating %d x %d events" % (K0, E))
    ev = synth.generate_events(np.arange(K0), E, seed=11)
    planes = np.ascontiguousarray(np.tile(synth.pack_events(ev), (1, tile, 1)))
    K = K0 * tile
    init = np.tile(np.concatenate([ev["init_acc"], ev["init_mag"]], axis=1), (tile, 1))
    tinit = np.tile(ev["t_init"], tile)
    evb = engine.DeviceBuffer(planes.nbytes).upload(planes)
    del planes
    ib = engine.DeviceBuffer(init.nbytes).upload(init)
    tb = engine.DeviceBuffer(tinit.nbytes).upload(tinit.astype(np.int64))
    r_max = E // 3 + 1
    win = engine.IMUWindow(K, r_max)
    cnt = engine.DeviceBuffer(4 * K)
    err = engine.DeviceBuffer(4).upload(np.zeros(1, np.int32))
    ms = timed(lambda: check(lib.pekf_frontend_dev(K, E, evb.ptr, ib.ptr, tb.ptr, 0.1, r_max, win.gd.ptr,
                                                   win.am.ptr, win.my.ptr, cnt.ptr, win.refs.ptr, err.ptr, s)), s)
    counts = cnt.download((K,), np.int32)
    recs = int(counts.sum())
    byts = K * E * 16 + recs * 40
    res["frontend"] = {"filters": K, "events_per_filter": E, "records": recs, "kernel_ms": ms,
                       "events_per_s": K * E / (ms * 1e-3), "gbs": byts / (ms * 1e-3) / 1e9,
                       "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM, "bytes": byts}
    log("frontend: %.2f ms, %.2e events/s, %.0f GB/s" % (ms, K * E / (ms * 1e-3), byts / (ms * 1e-3) / 1e9))
    # phase 2 on the same event planes: two passes (the means, then the variances of the first 100
    # samples of each type; the second pass stops once every type has had its 100)
    ib2, tb2, sb2, rb2 = (engine.DeviceBuffer(k * K) for k in (48, 8, 96, 4))
    ms = timed(lambda: check(lib.pekf_frontend_init_dev(K, E, evb.ptr, tb.ptr, 100, ib2.ptr, tb2.ptr, sb2.ptr,
                                                        rb2.ptr, s)), s)
    # algorithmic bytes: pass 1 reads every event; pass 2 a filter's events up to the one that brings
    # its last sensor type to 100 samples
    ty = ev["types"]
    last = np.zeros(K0, np.int64)
    for t in (synth.EV_ACC, synth.EV_GYRO, synth.EV_MAG):
        c = np.cumsum(ty == t, axis=0)
        last = np.maximum(last, np.argmax(c >= 100, axis=0) + 1)
    byts = 16 * (K * E + tile * int(last.sum()))
    res["frontend_init"] = {"filters": K, "events_per_filter": E, "kernel_ms": ms, "events_per_s": K * E / (ms * 1e-3),
                            "ready": int(rb2.download((K,), np.int32).sum()), "bytes": byts,
                            "gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
    log("frontend phase 2: %.2f ms" % ms)
    # the means alone (stats = NULL, as engine.run_session asks): pass 1 only
    ms = timed(lambda: check(lib.pekf_frontend_init_dev(K, E, evb.ptr, tb.ptr, 100, ib2.ptr, tb2.ptr, None,
                                                        rb2.ptr, s)), s)
    byts = 16 * K * E
    res["frontend_init_means"] = {"filters": K, "events_per_filter": E, "kernel_ms": ms,
                                  "events_per_s": K * E / (ms * 1e-3), "bytes": byts,
                                  "gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
    log("frontend phase 2, means only: %.2f ms" % ms)
    del ib2, tb2, sb2, rb2
    # the filter over the front-end's records (split pipeline, second half): one multi-record launch
    # with counts, as engine.BatchedEKF.run does for a front-end window
    n_rec = int(counts.max())
    f = engine.BatchedEKF(K)
    ms_run = timed(lambda: f.run_async(win, n_rec, 0, s, None, cnt), s)
    del f
    res["frontend_then_filter"] = {"filters": K, "records": recs, "frontend_ms": res["frontend"]["kernel_ms"],
                                   "filter_ms": ms_run, "total_ms": res["frontend"]["kernel_ms"] + ms_run}
    log("split pipeline: front-end %.2f + filter %.2f ms" % (res["frontend"]["kernel_ms"], ms_run))
    del win
    # the same events -> filter in one launch (pekf_live_dev): 16 B read per event, the state
    # (160 B per filter) read and written once
    f = engine.BatchedEKF(K)
    cnt2, refs2 = engine.DeviceBuffer(4 * K), engine.DeviceBuffer(48 * K)
    ms = timed(lambda: f.run_events_async(evb, E, ib, tb, cnt2, refs2, 0.1, s), s)
    assert np.array_equal(cnt2.download((K,), np.int32), counts)
    byts = K * E * 16 + K * (160 + 160 + 48 + 48 + 8 + 4)
    res["live"] = {"filters": K, "events_per_filter": E, "records": recs, "kernel_ms": ms,
                   "events_per_s": K * E / (ms * 1e-3), "records_per_s": recs / (ms * 1e-3), "bytes": byts,
                   "gbs": byts / (ms * 1e-3) / 1e9, "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM,
                   "vs_split": res["frontend_then_filter"]["total_ms"] / ms}
    log("fused front-end + filter: %.2f ms (split %.2f ms)" % (ms, res["frontend_then_filter"]["total_ms"]))
    del f, cnt2, refs2, evb
    if os.environ.get("PEKF_AUX_ONLY") == "live":
        print(json.dumps(res))
        return

    # ---- side outputs on a config-3-sized window
    B, W, N = 1 << 20, 1024, 10000
    win = engine.IMUWindow(B, W).synthesize(stream=s)
    q = engine.DeviceBuffer(32 * B).upload(np.tile([1.0, 0, 0, 0], (B, 1)))
    ms = timed(lambda: check(lib.pekf_gyro_chain_dev(B, N, W, 0, win.gd.ptr, q.ptr, None, s)), s)
    res["gyro_chain"] = {"filters": B, "records": N, "kernel_ms": ms, "steps_per_s": B * N / (ms * 1e-3),
                         "gbs": B * N * 16 / (ms * 1e-3) / 1e9, "hbm_frac": B * N * 16 / (ms * 1e-3) / 1e9 / HBM}
    log("gyro chain: %.1f ms" % ms)
    Nw = 1024
    out = engine.DeviceBuffer(32 * B * Nw)
    ms = timed(lambda: check(lib.pekf_wahba_stream_dev(B, Nw, W, 0, win.am.ptr, win.my.ptr, win.refs.ptr, 0.5, 0.5,
                                                       out.ptr, s)), s)
    res["wahba_stream"] = {"filters": B, "records": Nw, "kernel_ms": ms, "quats_per_s": B * Nw / (ms * 1e-3),
                           "gbs": B * Nw * 56 / (ms * 1e-3) / 1e9, "hbm_frac": B * Nw * 56 / (ms * 1e-3) / 1e9 / HBM}
    log("wahba stream: %.1f ms" % ms)
    del win, out

    # ---- online serving: every launch advances 1M filters by ONE new record; the state X, P and
    # the reference vectors are read and the state written through HBM each launch.  AoS: 40 B
    # record + 48 B refs + 32+128 B state read (P's cache lines come whole) + 32+128 B written;
    # SoA (X[4][B], P[10][B]): 40 + 48 + 32+80 + 32+80 B.
    B1 = 1 << 20
    win1 = engine.IMUWindow(B1, 8).synthesize(stream=s)
    for layout, per in (("aos", 40 + 48 + 32 + 128 + 32 + 128), ("soa", 40 + 48 + 32 + 80 + 32 + 80)):
        f1 = engine.BatchedEKF(B1, layout=layout)
        k = [0]

        def one_step():
            f1.run_async(win1, 1, k[0] % 8, s)
            k[0] += 1
        ms = timed(one_step, s, reps=20)
        res["online_step_" + layout] = {
            "filters": B1, "records_per_launch": 1, "kernel_ms": ms, "steps_per_s": B1 / (ms * 1e-3),
            "bytes_per_filter_step": per, "gbs": B1 * per / (ms * 1e-3) / 1e9,
            "hbm_frac": B1 * per / (ms * 1e-3) / 1e9 / HBM}
        log("online step %s (1M filters x 1 record): %.3f ms" % (layout, ms))
        del f1
    del win1

    # ---- filter handle: one FP64 record per filter per pekf_filter_update_dev (device pointers).
    # Bytes: gyro/acc/mag 72 + t 8 + prev_t 8+8 + refs 48 + state (AoS 32+128 / SoA 32+80) read and
    # written + X_out 32.
    rng = np.random.default_rng(3)
    a0 = rng.normal(size=(B1, 3))
    m0 = rng.normal(size=(B1, 3))
    ub = {k: engine.DeviceBuffer(8 * B1 * w).upload(np.ascontiguousarray(rng.normal(size=(B1, w)) if w == 3 else
                                                                          np.full((B1, 1), 10_000_000, np.int64)))
          for k, w in (("g", 3), ("a", 3), ("m", 3), ("t", 1))}
    xo = engine.DeviceBuffer(32 * B1)
    for layout, st_b in (("aos", 2 * (32 + 128)), ("soa", 2 * (32 + 80))):
        h = engine.FilterHandle(a0, m0, layout=layout)
        per = 72 + 8 + 16 + 48 + st_b + 32
        ms = timed(lambda: check(lib.pekf_filter_update_dev(h.h, ub["g"].ptr, ub["t"].ptr, ub["a"].ptr, ub["m"].ptr,
                                                            None, xo.ptr, s)), s, reps=20)
        res["handle_update_" + layout] = {
            "filters": B1, "kernel_ms": ms, "updates_per_s": B1 / (ms * 1e-3), "bytes_per_filter": per,
            "gbs": B1 * per / (ms * 1e-3) / 1e9, "hbm_frac": B1 * per / (ms * 1e-3) / 1e9 / HBM}
        log("handle update %s (1M filters, FP64 records): %.3f ms" % (layout, ms))
        del h
    del ub, xo
    # the same update from HOST arrays (pekf_filter_update: records in over PCIe through the pinned
    # staging buffer, X out): the PCIe-inclusive rate of the host-buffer boundary (never the headline)
    hg, ha, hm = (np.ascontiguousarray(rng.normal(size=(B1, 3))) for _ in range(3))
    h = engine.FilterHandle(a0, m0, layout="soa")
    for i in range(13):
        if i == 3:
            t0 = time.perf_counter()
        xh = h.update(hg, np.full(B1, 10_000_000 * (i + 1), np.int64), ha, hm)
    ms = (time.perf_counter() - t0) / 10 * 1e3
    res["handle_update_host_soa"] = {"filters": B1, "wall_ms": ms, "updates_per_s": B1 / (ms * 1e-3),
                                     "pcie_bytes_per_filter": 80 + 32,
                                     "pcie_gbs": B1 * 112 / (ms * 1e-3) / 1e9, "x_finite": bool(np.isfinite(xh).all())}
    log("handle update from host arrays (1M filters, PCIe-inclusive): %.3f ms" % ms)
    del h

    # ---- per-call operators at n = 1M (device pointers)
    n = 1 << 20
    rng = np.random.default_rng(0)
    X = rng.normal(size=(n, 4))
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    bufs = {k: engine.DeviceBuffer(a.nbytes).upload(np.ascontiguousarray(a)) for k, a in dict(
        g=rng.normal(size=(n, 3)), dt=np.full(n, 1e7), X=X, P=np.tile(np.eye(4), (n, 1, 1)),
        Q=np.tile(np.eye(3), (n, 1, 1)), R=np.tile(np.eye(4) * 0.1, (n, 1, 1)), acc=X[:, :3].copy(),
        mag=X[:, 1:].copy(), a0=np.tile([0, 0, 1.0], (n, 1)), m0=np.tile([0.5, 0, -0.86], (n, 1))).items()}
    z, Pm, Kk, Xo, Po = (engine.DeviceBuffer(8 * n * k) for k in (4, 16, 16, 4, 16))
    b = bufs
    ms = timed(lambda: check(lib.pekf_predict_dev(n, b["g"].ptr, b["dt"].ptr, b["X"].ptr, b["P"].ptr, b["Q"].ptr,
                                                  b["R"].ptr, z.ptr, Pm.ptr, Kk.ptr, None, s)), s)
    byts = n * 8 * (3 + 1 + 4 + 16 + 9 + 16 + 4 + 16 + 16)
    res["predict_dev"] = {"n": n, "kernel_ms": ms, "items_per_s": n / (ms * 1e-3), "gbs": byts / (ms * 1e-3) / 1e9,
                          "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
    ms = timed(lambda: check(lib.pekf_correct_dev(n, b["mag"].ptr, b["acc"].ptr, z.ptr, Pm.ptr, Kk.ptr, b["a0"].ptr,
                                                  b["m0"].ptr, Xo.ptr, Po.ptr, s)), s)
    byts = n * 8 * (3 + 3 + 4 + 16 + 16 + 3 + 3 + 4 + 16)
    res["correct_dev"] = {"n": n, "kernel_ms": ms, "items_per_s": n / (ms * 1e-3), "gbs": byts / (ms * 1e-3) / 1e9,
                          "hbm_frac": byts / (ms * 1e-3) / 1e9 / HBM}
    log("per-call predict %.2f ms, correct %.2f ms at n=1M" % (res["predict_dev"]["kernel_ms"], ms))

    # ---- per-call latency at n = 1 (host pointers): the ctypes engine wrappers, and the CPython
    # binding the drop-in KalmanFilter.Prediction / Correction use (what main_file.py pays per call)
    from poseestimationkf_amd import _fastcall
    gy, X1, P1, Q1, R1 = [0.1, 0.2, 0.3], np.array([1.0, 0, 0, 0]), np.eye(4), np.eye(3), np.eye(4) * 0.1
    mg, ac, a0, m0 = [0.5, 0, -0.86], [0, 0.1, 0.99], [0, 0, 1.0], [0.5, 0, -0.86]
    for key, pred, corr in (("ctypes_call_us", engine.predict, engine.correct),
                            ("dropin_call_us", _fastcall.predict, _fastcall.correct)):
        lat = {"predict": [], "correct": []}
        for i in range(300):
            t0 = time.perf_counter()
            zz, pm, kk = pred(gy, 1e7, X1, P1, Q1, R1)
            t1 = time.perf_counter()
            corr(mg, ac, zz, pm, kk, a0, m0)
            t2 = time.perf_counter()
            if i >= 50:
                lat["predict"].append(t1 - t0)
                lat["correct"].append(t2 - t1)
        res[key] = {k: float(np.median(v) * 1e6) for k, v in lat.items()}
        log("%s: %s" % (key, res[key]))
    res["c1_loop"] = c1_loop()
    log("config-1 loop: %s" % res["c1_loop"])
    res["device"] = engine.device_name(0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
