#!/usr/bin/env python3
"""Headline benchmark: EKF steps/s (predict + Wahba + update) at batch = 1M filters per GPU.

One bench "step" = one fused launch (pekf_run_dev) that advances every filter of this
rank's shard by --records IMU records (config 3 of BASELINE.json: 1,048,576 filters,
10,000 records).  Inputs are a resident window of --window records per filter (40 B per
filter-record, 43 GB at config 3 -- far beyond the 256 MB Infinity Cache), generated on
the device by the Philox generator before timing and replayed cyclically, so every
record is read from HBM.  For N > 1 ranks (torchrun, one process per GPU) each rank owns
an equal contiguous shard of filters (weak scaling), and each step ends with ONE gather of
the final quaternions to rank 0 over RCCL.

Prints ONE JSON line on rank 0.  `value` = filter-steps/s over all ranks (max-over-ranks
wall clock).  `roofline` is the fused kernel's achieved algorithmic HBM read rate
(40 B x filters x records / kernel time, HIP events on the launch stream) against the
8 TB/s peak; `cpu_baseline` times the NumPy restatement of the reference loop on the
host cores (rank 0, N = 1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REC_BYTES = 40          # algorithmic bytes per filter-record
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level table)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak (spec)


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


class StdoutForTheResult:
    """Native libraries print on the process's stdout (RCCL writes a version banner there when a
    communicator is created, on every rank): point file descriptor 1 at stderr for the whole run
    and restore it only to print the result line, so stdout carries exactly one JSON line."""

    def __init__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def emit(self, line):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        print(line, flush=True)
        os.dup2(2, 1)


# ----------------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    """Runs in a forked child (before any GPU initialisation): NumPy restatement of main_file.py's loop."""
    import numpy as np

    from oracle import ekf_numpy
    from poseestimationkf_amd import synth
    ids, n_rec, seed, missing, barrier = args
    rec = synth.generate(np.asarray(ids), n_rec, seed=seed, missing=missing)
    barrier.wait()
    t0 = time.perf_counter()
    for k in range(len(ids)):
        g, d, a, m = rec.filter(k)
        ekf_numpy.run_filter(g, d, a, m, rec.acc0[k], rec.mag0[k], missing=rec.missing[:, k] if missing else None,
                             record=False)
    return len(ids) * n_rec, time.perf_counter() - t0


def cpu_baseline(seed, missing, filters_per_core=160, n_rec=1500):
    import multiprocessing as mp
    cores = len(os.sched_getaffinity(0))
    workers = max(1, min(16, cores))
    ctx = mp.get_context("fork")
    mgr = ctx.Manager()
    barrier = mgr.Barrier(workers)
    jobs = [(list(range(w * filters_per_core, (w + 1) * filters_per_core)), n_rec, seed, missing, barrier)
            for w in range(workers)]
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, jobs)
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": steps / wall, "unit": "EKF steps/s", "cores": workers, "kind": "port",
            "sample": "NumPy restatement of main_file.py's per-record loop (oracle/ekf_numpy.py, bit-identical "
                      "to the reference), %d processes x %d filters x %d records of the same synthetic stream; "
                      "%d host cores visible" % (workers, filters_per_core, n_rec, cores),
            "seconds": wall}


def c_oracle_rate(seed, missing, n_filters=64, n_rec=1000):
    import numpy as np

    from oracle import oracle_c
    from poseestimationkf_amd import synth
    rec = synth.generate(np.arange(n_filters), n_rec, seed=seed, missing=missing)
    t0 = time.perf_counter()
    oracle_c.run(rec)
    dt = time.perf_counter() - t0
    return {"value": n_filters * n_rec / dt, "threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())),
            "what": "C FP64 restatement (oracle/ekf_oracle.c, Jacobi SVD), OpenMP over filters"}


# ----------------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1 << 20, help="filters per GPU (config 3: 1,048,576)")
    ap.add_argument("--records", type=int, default=10000, help="records per filter per bench step")
    ap.add_argument("--window", type=int, default=1024, help="resident records per filter")
    ap.add_argument("--missing", action="store_true", help="config 5: 30%% magnetometer-missing records")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--cpu-baseline", choices=["port", "none"], default="port")
    ap.add_argument("--parity-samples", type=int, default=16)
    ap.add_argument("--precision", choices=["f64", "mixed"], default="f64",
                    help="f64 (default, as the reference) or mixed (covariance recursion in f32)")
    ap.add_argument("--dist", action="store_true",
                    help="use the RCCL path (pekf_gather_dev) even at world size 1 (exercises the gather)")
    args = ap.parse_args()
    out_fd = StdoutForTheResult()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    assert world == args.gpus or "RANK" not in os.environ, "WORLD_SIZE and --gpus disagree"

    # CPU baseline first, in forked workers, before anything touches the GPU.
    cpu = None
    if args.cpu_baseline == "port" and rank == 0 and world == 1:
        log("cpu baseline (NumPy restatement) ...")
        cpu = cpu_baseline(args.seed, args.missing)
        try:
            cpu["c_oracle"] = c_oracle_rate(args.seed, args.missing)
        except Exception as e:  # the C oracle is optional for the baseline line
            cpu["c_oracle"] = {"error": str(e)}
        log("cpu baseline: %.0f steps/s on %d cores" % (cpu["value"], cpu["cores"]))

    dist = None
    use_dist = world > 1 or args.dist
    if use_dist:
        # torch.distributed only for the rendezvous (gloo, CPU): the RCCL id broadcast and the
        # host barrier.  The data-path collectives are RCCL through libpekf (shard.Communicator).
        # torch is imported before libpekf so that the process has ONE HIP runtime and ONE RCCL
        # (the ones PyTorch-ROCm bundles; libpekf binds them by SONAME).
        import torch  # noqa: F401
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    import numpy as np

    from poseestimationkf_amd import engine, shard, synth
    engine.set_device(local)
    first, B = shard.shard_range(args.batch * world, rank, world)
    N, W = args.records, args.window

    own_stream = engine.Stream()  # keep the object alive for the whole run
    stream = own_stream.handle
    comm = shard.Communicator(shard.exchange_unique_id(rank, world), world, rank) if use_dist else None
    if comm is not None:
        log("rank %d/%d: RCCL %d communicator on device %d" % (rank, world, shard.rccl_version(), comm.device))

    def sync():
        engine.check(engine.lib.pekf_stream_sync(stream))

    def barrier():
        if use_dist:
            dist.barrier()

    log("rank %d/%d: synthesizing %d filters x %d records (%.1f GB resident)" %
        (rank, world, B, W, synth.window_bytes(B, W) / 1e9))
    win = engine.IMUWindow(B, W).synthesize(seed=args.seed, first_filter=first, missing=args.missing,
                                            stream=stream)
    filt = engine.BatchedEKF(B, q=1.0, r=0.1, precision=args.precision)
    recv = engine.DeviceBuffer(32 * B * world) if (use_dist and rank == 0) else None
    sync()

    total = args.warmup + args.steps
    ev = [(engine.Event(), engine.Event()) for _ in range(total)]

    def bench_step(k):
        e0, e1 = ev[k]
        e0.record(stream)
        filt.run_async(win, N, (k * N) % W, stream)
        e1.record(stream)
        if use_dist:  # ONE RCCL gather of the final quaternions to rank 0 (pekf_gather_dev)
            shard.gather_quaternions(comm, filt.X.ptr, B, recv, 0, stream)

    for k in range(args.warmup):
        bench_step(k)
        sync()
        log("warmup %d: kernel %.1f ms" % (k, ev[k][0].elapsed_ms(ev[k][1])))

    sync()
    barrier()
    t0 = time.perf_counter()
    for k in range(args.warmup, total):
        bench_step(k)
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if use_dist:  # the slowest rank's time (RCCL max all-reduce)
        tb = engine.DeviceBuffer(8).upload(np.array([elapsed], np.float64), stream)
        comm.allreduce_max(tb.ptr, 1, stream)
        elapsed = float(tb.download((1,), np.float64, stream)[0])
        sync()
    kms = [ev[k][0].elapsed_ms(ev[k][1]) for k in range(args.warmup, total)]
    log("timed: %.3f s for %d steps; kernel ms %s" % (elapsed, args.steps, ", ".join("%.1f" % v for v in kms)))

    # parity at scale: sampled filters re-run on the host by the C oracle
    parity = None
    if args.parity_samples > 0:
        from oracle import oracle_c
        X, _ = filt.get_state()
        cols = np.linspace(0, B - 1, args.parity_samples).astype(np.int64)
        rec = synth.generate(cols + first, W, seed=args.seed, missing=args.missing)
        Xo, _, _ = oracle_c.run(rec, n_steps=total * N)
        err = float(np.abs(X[cols] - Xo).max())
        parity = {"filters": int(args.parity_samples), "records": total * N, "max_abs_err_vs_oracle": err,
                  "tolerance": 1e-5, "ok": bool(err < 1e-5)}
        log("parity: max |dq| = %.3e over %d sampled filters" % (err, args.parity_samples))

    if rank == 0:
        steps_total = world * B * N * args.steps
        value = steps_total / elapsed
        k_s = float(np.mean(kms)) / 1e3
        achieved = B * N * REC_BYTES / k_s / 1e9
        flop = ISA_COUNTS[args.precision]["flop"]
        valu = ISA_COUNTS[args.precision]["valu_instr"]
        # the committed PMC pass is of the FP64 command without missing records
        traffic, tsrc = measured_traffic(B, N) if args.precision == "f64" and not args.missing else (None, None)
        clk = tsrc[1].get("effective_clock_ghz") if tsrc else None
        issue_frac = (4.0 * (B / 64.0) * N * valu / (1024 * clk * 1e9 * k_s)) if clk else None
        out = {
            "metric": "EKF steps/sec (predict+Wahba+update) at batch=1M; HBM-roofline %",
            "value": value,
            "unit": "EKF filter-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "f64" else "f64 quaternion path + f32 covariance (P, S^-1)",
            "data": "synthetic (on-device Philox IMU generator, bit-identical host mirror; 40 B records, "
                    "%d-record resident window replayed cyclically)" % W,
            "config": {"workload": workload_name(B, N, args.missing),
                       "filters_per_gpu": B, "global_filters": B * world, "records_per_step": N,
                       "window_records": W, "parallelism": "dp%d (filter-batch shards, 1 RCCL gather via pekf_gather_dev)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": (os.path.relpath(tsrc[0], ROOT) + " (2 x FETCH_SIZE, separate "
                                            "rocprofv3 --pmc pass of this command)") if tsrc else None,
                         "kernel": "k_run<false> (pekf_run_dev)", "kernel_ms": k_s * 1e3,
                         "bytes_per_launch": B * N * REC_BYTES},
            "fp64_valu": {"flop_per_step": flop, "fp64_instr_per_step": ISA_COUNTS[args.precision]["fp64_instr"],
                          "valu_instr_per_step": valu,
                          "achieved_tflops": B * N * flop / k_s / 1e12, "peak_tflops": FP64_PEAK_TFLOPS,
                          "frac": B * N * flop / k_s / 1e12 / FP64_PEAK_TFLOPS,
                          "valu_busy_pmc": tsrc[1].get("valu_busy") if tsrc else None,
                          "issue_frac": issue_frac,
                          "clock_ghz_pmc": clk,
                          "note": "the kernel is VALU-issue-bound at a power-limited clock: issue_frac = 4 cycles x "
                                  "wave-instructions / (1024 SIMDs x PMC effective clock x kernel time); the same "
                                  "launch with cache-resident records runs at 2.11 GHz instead of 1.80 "
                                  "(profiles/r1/power_probe); HBM frac is capped by it"},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        out_fd.emit(json.dumps(out))
    if use_dist:
        if rank == 0:  # the gathered quaternions are the filters' final X, rank 0's shard first
            Xr, _ = filt.get_state()
            got = recv.download((world * B, 4), np.float64)
            assert np.array_equal(got[:B], Xr), "gather mismatch on rank 0"
            assert np.isfinite(got).all() and np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-12), \
                "gathered quaternions of other ranks are not unit"
            log("gather: %d quaternions on rank 0 (RCCL via pekf_gather_dev) match rank 0's shard" % got.shape[0])
        comm.close()
        dist.destroy_process_group()

# FP64 work per filter-step of the fused kernel, counted from its gfx950 ISA hot loop by
# scripts/isa_count.py (DESIGN.md "FP64 budget"): FP64 VALU instructions, and the FLOP of
# the arithmetic ones with an FMA counted as 2.
# per filter-step: the VALU instructions of the basic blocks a tracked lane executes in k_run's hot
# loop (scripts/loop_blocks.py on the hipcc -S listing: the fallback bodies sit behind
# s_cbranch_execz); FP64 instructions and FLOP from scripts/isa_count.py on the same blocks.  The
# PMC pass in profiles/ counts the executed total (SQ_INSTS_VALU per wave-step).
ISA_COUNTS = {"f64": {"flop": 436, "fp64_instr": 298, "valu_instr": 301},
              "mixed": {"flop": 240, "fp64_instr": 191, "valu_instr": 329}}  # mixed: + ~130 f32 instructions
FLOP_PER_STEP = ISA_COUNTS["f64"]["flop"]
FP64_INSTR_PER_STEP = ISA_COUNTS["f64"]["fp64_instr"]


def workload_name(batch, records, missing):
    """BASELINE.json's configuration this run is (configs 2, 3 and 5 are 10,000 records)."""
    if records == 10000 and batch == 1 << 20:
        return ("config 5: batch=1,048,576/GPU, 30% missing-mag" if missing else
                "config 3: batch=1,048,576 filters/GPU x 10,000 records")
    if records == 10000 and batch == 65536 and not missing:
        return "config 2: batch=65,536 filters/GPU x 10,000 records"
    return "custom: batch=%d filters/GPU x %d records%s" % (batch, records, ", 30% missing-mag" if missing else "")


def measured_traffic(batch, records):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of the current build
    (profiles/HEADLINE_PMC names it; scripts/refresh.sh produces it), if its config matches."""
    try:
        with open(os.path.join(ROOT, "profiles", "HEADLINE_PMC")) as fh:
            path = os.path.join(ROOT, fh.read().strip())
        with open(path) as fh:
            s = json.load(fh)
    except OSError:
        return None, None
    if s.get("config") != {"batch": batch, "records": records}:
        return None, None
    return s["hbm_traffic_bytes"], (path, s)

if __name__ == "__main__":
    main()
