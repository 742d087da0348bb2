#!/usr/bin/env python3
"""Headline benchmark: EKF steps/s (predict + Wahba + update) at batch = 1M filters per GPU.

One bench "step" = one fused launch (pekf_run_dev) per GPU that advances every filter of that
GPU's shard by --records IMU records (config 3 of BASELINE.json: 1,048,576 filters, 10,000
records).  When more than one GPU takes part, the timed run ends with ONE RCCL gather of the final
quaternions to the root (the north_star's single gather; the shards exchange nothing per step, so
the GPUs run their steps independently).  Inputs are a resident window of --window records per filter (40 B per
filter-record, 43 GB at config 3 -- far beyond the 256 MB Infinity Cache), generated on the device
by the Philox generator before timing and replayed cyclically, so every record is read from HBM.

`--gpus N` measures N GPUs by itself, with no PyTorch anywhere in the process:
  * launched by torchrun (or any launcher that sets RANK / WORLD_SIZE / LOCAL_RANK): one process
    per GPU; rank 0's RCCL id goes through a file on the node (shard.FileRendezvous), and the
    barriers and the max-over-ranks time are RCCL all-reduces through libpekf;
  * launched plainly: one process drives GPUs 0..N-1 (shard.MultiDeviceEKF: ncclCommInitAll,
    per-device streams, one grouped gather).
Either way each GPU owns an equal contiguous shard of filters (weak scaling), and the run exits
non-zero when fewer than N GPUs are visible.

Prints ONE JSON line on rank 0.  `value` = filter-steps/s over all GPUs (the slowest rank's wall
clock, the final gather included).  `roofline` is the fused kernel's achieved algorithmic HBM read rate per
GPU (40 B x filters x records / kernel time, HIP events on the launch stream) against the 8 TB/s
peak; `valu_roofline` is the resource that binds it, FP64 VALU issue; `cpu_baseline` times the
NumPy restatement of the reference loop on the job's host cores (rank 0, at every N, a bounded
sample, before any GPU work; the core count comes from the cgroup's CPU quota / cpuset);
`kernel_ms_per_gpu` / `gather_ms_per_gpu` attribute each GPU's time to its launches and the gather.
A rank that never joins or dies mid-run fails the job within PEKF_COMM_TIMEOUT_S (status 2).
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
# FP64 VALU issue ceiling: 256 CUs x 4 SIMDs, a wave64 FP64 instruction occupies a 16-lane SIMD for
# 4 cycles, at the 2.4 GHz peak engine clock -> 614.4 G wave-instructions/s (= 78.6 TFLOP/s of FMA)
SIMDS, CYCLES_PER_WAVE_INSTR, PEAK_CLOCK_GHZ = 1024, 4, 2.4
VALU_PEAK_GWIPS = SIMDS * PEAK_CLOCK_GHZ / CYCLES_PER_WAVE_INSTR


class BenchError(SystemExit):
    """A refused configuration: message on stderr, exit status 2."""

    def __init__(self, msg):
        print("[bench] error: " + msg, file=sys.stderr, flush=True)
        super().__init__(2)


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


# ----------------------------------------------------------------------------------- launch plan
def launch_plan(gpus, environ, shard_of=None, one_process=False):
    """How this process takes part: dict(mode, rank, world, devices, first_shard).

    mode "ranks":  a launcher set RANK and WORLD_SIZE (torchrun): this process is one rank, on
                   device LOCAL_RANK; WORLD_SIZE must equal --gpus.
    mode "single": --gpus 1, no launcher: GPU 0.
    mode "multi":  --gpus N > 1, no launcher: this process drives GPUs 0..N-1.
    shard_of (R, W): a one-GPU run of rank R's shard of a W-way job (its filters keep their global
    ids, so any rank's workload can be rehearsed on one GPU).
    one_process: mode "multi" even for --gpus 1 (the plain --gpus N code path, rehearsed on one GPU)."""
    if gpus < 1:
        raise BenchError("--gpus must be >= 1")
    if "RANK" in environ and "WORLD_SIZE" in environ:
        rank, world = int(environ["RANK"]), int(environ["WORLD_SIZE"])
        if world != gpus:
            raise BenchError("WORLD_SIZE=%d from the launcher but --gpus %d" % (world, gpus))
        if shard_of is not None:
            raise BenchError("--shard-of is a one-process rehearsal; not under a launcher")
        local = int(environ.get("LOCAL_RANK", rank))
        return dict(mode="ranks", rank=rank, world=world, devices=[local], first_shard=rank)
    if shard_of is not None:
        r, w = shard_of
        if gpus != 1 or not 0 <= r < w:
            raise BenchError("--shard-of R/W needs --gpus 1 and 0 <= R < W")
        return dict(mode="single", rank=0, world=1, devices=[0], first_shard=r)
    if gpus == 1 and not one_process:
        return dict(mode="single", rank=0, world=1, devices=[0], first_shard=0)
    return dict(mode="multi", rank=0, world=gpus, devices=list(range(gpus)), first_shard=0)


def shard_plan(batch_per_gpu, world):
    """[(first_filter, count)] of every GPU's shard (shard.shard_range over the global batch)."""
    from poseestimationkf_amd import shard
    return [shard.shard_range(batch_per_gpu * world, r, world) for r in range(world)]


def parse_shard_of(s):
    try:
        r, w = (int(v) for v in s.split("/"))
    except ValueError:
        raise argparse.ArgumentTypeError("expected R/W, e.g. 7/8")
    return r, w


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


def _cpulist_count(text):
    """Number of CPUs in a cpuset list such as "0-3,8,10-11" (0 for an empty list)."""
    n = 0
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        lo, _, hi = part.partition("-")
        n += (int(hi) - int(lo) + 1) if hi else 1
    return n


def _read(path):
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return None


def cgroup_cpu_limits(proc_cgroup="/proc/self/cgroup", root="/sys/fs/cgroup"):
    """The CPU limits of this process's cgroup (v2 unified, or v1 cpu + cpuset controllers).

    Every existing level from the process's own cgroup directory up to the mount root is read (a
    cgroup namespace may hide the leaf, as on the GPU box): the quota is the smallest
    quota / period on the path (v2 cpu.max "Q P" or "max P"; v1 cpu.cfs_quota_us / cpu.cfs_period_us,
    -1 = none), the cpuset the deepest level's effective list.  Returns dict(quota_cores, quota_at,
    cpuset_cores, cpuset_at, version); a limit that is not found is None."""
    out = dict(quota_cores=None, quota_at=None, cpuset_cores=None, cpuset_at=None, version=None)
    text = _read(proc_cgroup)
    if text is None:
        return out
    paths = {}
    for line in text.splitlines():
        parts = line.split(":", 2)
        if len(parts) == 3:
            for ctl in (parts[1].split(",") if parts[1] else [""]):
                paths[ctl] = parts[2]

    def levels(base, rel):
        rel = rel.strip("/")
        segs = rel.split("/") if rel else []
        for i in range(len(segs), -1, -1):
            d = os.path.join(base, *segs[:i]) if i else base
            if os.path.isdir(d):
                yield d

    def take_quota(q, where):
        if q is not None and (out["quota_cores"] is None or q < out["quota_cores"]):
            out["quota_cores"], out["quota_at"] = q, where

    if "" in paths and os.path.exists(os.path.join(root, "cgroup.controllers")):   # v2
        out["version"] = 2
        for d in levels(root, paths[""]):
            v = _read(os.path.join(d, "cpu.max"))
            if v:
                f = v.split()
                if f[0] != "max" and len(f) == 2 and float(f[1]) > 0:
                    take_quota(max(1, int(float(f[0]) // float(f[1]))), os.path.join(d, "cpu.max"))
            c = _read(os.path.join(d, "cpuset.cpus.effective"))
            if c and out["cpuset_cores"] is None:
                out["cpuset_cores"], out["cpuset_at"] = _cpulist_count(c), os.path.join(d, "cpuset.cpus.effective")
        return out
    for ctl, rel in paths.items():                                                   # v1
        names = ctl.split(",")
        if "cpu" in names:
            out["version"] = 1
            for mount in ("cpu,cpuacct", "cpu", "cpuacct,cpu"):
                base = os.path.join(root, mount)
                if not os.path.isdir(base):
                    continue
                for d in levels(base, rel):
                    q, per = _read(os.path.join(d, "cpu.cfs_quota_us")), _read(os.path.join(d, "cpu.cfs_period_us"))
                    if q and per and int(q) > 0 and int(per) > 0:
                        take_quota(max(1, int(q) // int(per)), os.path.join(d, "cpu.cfs_quota_us"))
                break
        if "cpuset" in names:
            out["version"] = 1
            base = os.path.join(root, "cpuset")
            for d in levels(base, rel):
                c = _read(os.path.join(d, "cpuset.effective_cpus")) or _read(os.path.join(d, "cpuset.cpus"))
                if c:
                    out["cpuset_cores"], out["cpuset_at"] = _cpulist_count(c), d
                    break
    return out


def cpu_share(environ=os.environ, proc_cgroup="/proc/self/cgroup", cgroup_root="/sys/fs/cgroup", affinity=None):
    """The host cores this job may use: min(affinity, cgroup CPU quota, cgroup cpuset).  On the GPU box
    sched_getaffinity shows the whole machine (256) while the cgroup's cpu.max gives the job its share
    (16 per GPU).  Only when no cgroup limit exists is OMP_NUM_THREADS taken as the declared share
    (a launcher's per-job setting), and only when nothing at all limits the job, every affinity core.
    Returns dict(use, affinity, quota_cores, cpuset_cores, omp_num_threads, share_source)."""
    aff = len(os.sched_getaffinity(0)) if affinity is None else int(affinity)
    lim = cgroup_cpu_limits(proc_cgroup, cgroup_root)
    cands = [(aff, "sched_getaffinity")]
    if lim["quota_cores"] is not None:
        cands.append((lim["quota_cores"], "cgroup v%d CPU quota (%s)" % (lim["version"], lim["quota_at"])))
    if lim["cpuset_cores"] is not None:
        cands.append((lim["cpuset_cores"], "cgroup v%d cpuset (%s)" % (lim["version"], lim["cpuset_at"])))
    use, source = min(cands, key=lambda c: c[0])
    omp = environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    if use == aff and lim["quota_cores"] is None and omp is not None and omp < aff:
        use, source = omp, "OMP_NUM_THREADS (no cgroup CPU quota found)"
    return dict(use=max(1, use), affinity=aff, quota_cores=lim["quota_cores"], cpuset_cores=lim["cpuset_cores"],
                omp_num_threads=omp, share_source=source)


def cpu_baseline(seed, missing, filters_per_core=160, n_rec=1500):
    import multiprocessing as mp
    share = cpu_share()
    workers, cores = share["use"], share["affinity"]
    ctx = mp.get_context("fork")
    mgr = ctx.Manager()
    barrier = mgr.Barrier(workers)
    jobs = [(list(range(w * filters_per_core, (w + 1) * filters_per_core)), n_rec, seed, missing, barrier)
            for w in range(workers)]
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, jobs)
    mgr.shutdown()
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": steps / wall, "unit": "EKF steps/s", "cores": workers, "kind": "port",
            "per_core": steps / wall / workers, "cores_visible": cores, "share_source": share["share_source"],
            "cgroup_quota_cores": share["quota_cores"], "cgroup_cpuset_cores": share["cpuset_cores"],
            "sample": "NumPy restatement of main_file.py's per-record loop (oracle/ekf_numpy.py, bit-identical "
                      "to the reference), %d processes (one per core of this job's CPU share: %s; %d cores in "
                      "the affinity mask) x %d filters x %d records of the same synthetic stream"
                      % (workers, share["share_source"], cores, filters_per_core, n_rec),
            "seconds": wall}


def c_oracle_rate(seed, missing, n_filters=64, n_rec=1000):
    import numpy as np

    from oracle import oracle_c
    from poseestimationkf_amd import synth
    rec = synth.generate(np.arange(n_filters), n_rec, seed=seed, missing=missing)
    t0 = time.perf_counter()
    oracle_c.run(rec)
    dt = time.perf_counter() - t0
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return {"value": n_filters * n_rec / dt,
            "threads": int(omp) if omp.isdigit() else len(os.sched_getaffinity(0)),
            "threads_source": "OMP_NUM_THREADS" if omp.isdigit() else "OpenMP default (affinity mask)",
            "what": "C FP64 restatement (oracle/ekf_oracle.c, Jacobi SVD), OpenMP over filters"}


# ----------------------------------------------------------------------------------- the runs
class RankRun:
    """One process = one GPU (modes "single" and "ranks"): this rank's shard as an IMUWindow +
    BatchedEKF on device `dev`; with a communicator, gather() sends its final quaternions to rank 0."""

    def __init__(self, args, plan, rdzv=None):
        import numpy as np

        from poseestimationkf_amd import engine, shard
        self.np, self.engine, self.shard = np, engine, shard
        self.rank, self.world = plan["rank"], plan["world"]
        engine.set_device(plan["devices"][0])
        self.B = args.batch
        self.first = plan["first_shard"] * self.B
        self.own_stream = engine.Stream()
        self.stream = self.own_stream.handle
        self.comm = None
        if self.world > 1 or args.dist:
            self.comm = shard.connect(self.rank, self.world, rdzv)
            log("rank %d/%d: RCCL %d communicator on device %d" % (self.rank, self.world, shard.rccl_version(),
                                                                  self.comm.device))
        log("rank %d/%d: synthesizing filters [%d, %d) x %d records (%.1f GB resident)" %
            (self.rank, self.world, self.first, self.first + self.B, args.window,
             self.B * args.window * REC_BYTES / 1e9))
        self.win = engine.IMUWindow(self.B, args.window).synthesize(
            seed=args.seed, first_filter=self.first, missing=args.missing, stream=self.stream)
        self.filt = engine.BatchedEKF(self.B, q=1.0, r=0.1, precision=args.precision)
        self.recv = engine.DeviceBuffer(32 * self.B * self.world) if (self.comm and self.rank == 0) else None
        self.sync()
        self.ev = []

    def prepare(self, n_steps):
        """ev[k] = (kernel start, kernel end) HIP events of step k on this rank's stream; gev = (start,
        end) of the last gather."""
        self.ev = [tuple(self.engine.Event() for _ in range(2)) for _ in range(n_steps)]
        self.gev = (self.engine.Event(), self.engine.Event())
        self.gathered = False

    def sync(self):
        if self.comm is not None:  # drains the stream's collectives too, against PEKF_COMM_TIMEOUT_S
            self.comm.wait(self.stream)
        else:
            self.engine.check(self.engine.lib.pekf_stream_sync(self.stream))

    def barrier(self):
        if self.comm is not None:
            self.comm.barrier(self.stream)

    def step(self, k, n_rec, row0):
        e0, e1 = self.ev[k]
        e0.record(self.stream)
        self.filt.run_async(self.win, n_rec, row0, self.stream)
        e1.record(self.stream)

    def gather(self):
        """ONE RCCL gather of the current quaternions to rank 0 (pekf_gather_dev), enqueued after the
        launches; its time includes waiting for the slowest peer's last launch."""
        if self.comm is None:
            return
        g0, g1 = self.gev
        g0.record(self.stream)
        self.shard.gather_quaternions(self.comm, self.filt.X.ptr, self.B, self.recv, 0, self.stream)
        g1.record(self.stream)
        self.gathered = True

    def kernel_ms(self, k):
        return self.ev[k][0].elapsed_ms(self.ev[k][1])

    def gather_ms(self):
        return self.gev[0].elapsed_ms(self.gev[1]) if self.gathered else 0.0

    def slowest(self, elapsed):
        return self.comm.max_over_ranks(elapsed, self.stream) if self.comm is not None else elapsed

    def per_gpu(self, steps):
        """(kernel ms, gather ms) per GPU in rank order -- the mean launch time over `steps` and the final
        gather's time: every rank's own HIP-event times, exchanged with one RCCL all-reduce (collective:
        all ranks call it)."""
        mine = [float(self.np.mean([self.kernel_ms(k) for k in steps])), float(self.gather_ms())]
        if self.comm is None:
            return [mine[0]], [mine[1]]
        allv = self.comm.all_values(mine, self.stream)
        return [float(v) for v in allv[:, 0]], [float(v) for v in allv[:, 1]]

    def final_rows(self):
        """(global first filter id, X rows) available on this rank: every filter's final X on rank 0
        after the gather, this shard's otherwise."""
        np = self.np
        if self.comm is not None and self.rank == 0:
            got = self.recv.download((self.world * self.B, 4), np.float64)
            Xr, _ = self.filt.get_state()
            if not np.array_equal(got[:self.B], Xr):
                raise AssertionError("RCCL gather: rank 0's rows differ from its shard's state")
            return 0 if self.world > 1 else self.first, got
        X, _ = self.filt.get_state()
        return self.first, X

    def close(self):
        if self.comm is not None:
            self.comm.close()


class MultiRun:
    """One process drives GPUs 0..N-1 (mode "multi"): shard.MultiDeviceEKF, the final quaternions
    collected by one grouped RCCL gather.  Times are per-device HIP events on each device's own stream."""

    def __init__(self, args, plan):
        from poseestimationkf_amd import engine, shard
        self.engine = engine
        self.rank, self.world, self.devices = 0, plan["world"], plan["devices"]
        self.B = args.batch
        log("single process over devices %s: %d filters each, %d records resident (%.1f GB per GPU)" %
            (self.devices, self.B, args.window, self.B * args.window * REC_BYTES / 1e9))
        self.m = shard.MultiDeviceEKF(self.devices, self.B, args.window, precision=args.precision)
        log("RCCL %d: %d communicators (ncclCommInitAll)" % (shard.rccl_version(), len(self.devices)))
        self.m.synthesize(seed=args.seed, missing=args.missing)
        self.ev = []

    def prepare(self, n_steps):
        """HIP events are per device: ev[k][i] = (kernel start, kernel end) of step k on device i, gev[i] =
        (start, end) of the last gather on device i."""
        self.ev = []
        for _ in range(n_steps):
            pair = []
            for d in self.devices:
                self.engine.set_device(d)
                pair.append(tuple(self.engine.Event() for _ in range(2)))
            self.ev.append(pair)
        self.gev = []
        for d in self.devices:
            self.engine.set_device(d)
            self.gev.append((self.engine.Event(), self.engine.Event()))
        self.engine.set_device(self.devices[0])
        self.gathered = False

    def sync(self):
        self.m.sync()

    def barrier(self):
        self.m.sync()

    def step(self, k, n_rec, row0):
        for i, d in enumerate(self.devices):
            self.engine.set_device(d)
            e0, e1 = self.ev[k][i]
            s = self.m.streams[i].handle
            e0.record(s)
            self.m.filts[i].run_async(self.m.wins[i], n_rec, row0, s)
            e1.record(s)
        self.engine.set_device(self.devices[0])

    def gather(self):
        """The final quaternions of every device to device 0: one grouped RCCL gather."""
        for i, d in enumerate(self.devices):
            self.engine.set_device(d)
            self.gev[i][0].record(self.m.streams[i].handle)
        self.engine.set_device(self.devices[0])
        self.m.gather_async()
        for i, d in enumerate(self.devices):
            self.engine.set_device(d)
            self.gev[i][1].record(self.m.streams[i].handle)
        self.engine.set_device(self.devices[0])
        self.gathered = True

    def kernel_ms(self, k, device_index=None):
        """The slowest device's kernel time of step k (or one device's)."""
        t = [e[0].elapsed_ms(e[1]) for e in self.ev[k]]
        return max(t) if device_index is None else t[device_index]

    def gather_ms(self, device_index=None):
        if not self.gathered:
            return 0.0
        t = [g[0].elapsed_ms(g[1]) for g in self.gev]
        return max(t) if device_index is None else t[device_index]

    def slowest(self, elapsed):
        return elapsed

    def per_gpu(self, steps):
        n = len(self.devices)
        return ([sum(self.kernel_ms(k, i) for k in steps) / len(steps) for i in range(n)],
                [self.gather_ms(i) for i in range(n)])

    def final_rows(self):
        return 0, self.m.gathered()

    def close(self):
        self.m.close()


def parity_check(first, rows, n_samples, n_records, args):
    """Re-run sampled filters (spread over every GPU's shard when rows hold them all) with the C
    oracle from the host mirror of the generator; max |dq| against the device's final X."""
    import numpy as np

    from oracle import oracle_c
    from poseestimationkf_amd import synth
    n = rows.shape[0]
    cols = np.unique(np.linspace(0, n - 1, max(1, n_samples)).astype(np.int64))
    rec = synth.generate(cols + first, args.window, seed=args.seed, missing=args.missing)
    Xo, _, _ = oracle_c.run(rec, n_steps=n_records)
    err = float(np.abs(rows[cols] - Xo).max())
    shards = sorted({int((c + first) // args.batch) for c in cols})
    return {"filters": int(len(cols)), "records": int(n_records), "max_abs_err_vs_oracle": err,
            "tolerance": 1e-5, "ok": bool(err < 1e-5), "global_filter_ids": [int(cols[0] + first), int(cols[-1] + first)],
            "shards_covered": shards,
            "unit_norm_all": bool(np.isfinite(rows).all() and np.allclose(np.linalg.norm(rows, axis=1), 1.0,
                                                                          atol=1e-12))}


# ----------------------------------------------------------------------------------- main
def parse_args(argv=None):
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
    ap.add_argument("--cpu-filters-per-core", type=int, default=160,
                    help="CPU baseline sample: filters per host process")
    ap.add_argument("--cpu-records", type=int, default=1500, help="CPU baseline sample: records per filter")
    ap.add_argument("--parity-samples", type=int, default=16,
                    help="filters re-run by the C oracle (at least 4 per GPU when N > 1)")
    ap.add_argument("--precision", choices=["f64", "mixed"], default="f64",
                    help="f64 (default, as the reference) or mixed (covariance recursion in f32)")
    ap.add_argument("--dist", action="store_true",
                    help="use the RCCL path (pekf_gather_dev) even at world size 1 (exercises the gather)")
    ap.add_argument("--shard-of", type=parse_shard_of, default=None, metavar="R/W",
                    help="rehearse rank R's shard of a W-way job on one GPU (e.g. 7/8 at config 4)")
    ap.add_argument("--one-process", action="store_true",
                    help="drive the GPUs from one process (MultiDeviceEKF) even for --gpus 1")
    return ap.parse_args(argv)


def main(argv=None):
    """Runs the benchmark; a failed collective (a rank missing at communicator creation, a peer gone
    mid-run: libpekf's PEKF_COMM_TIMEOUT_S deadlines) ends it with status 2, a message on stderr and
    nothing on stdout."""
    from poseestimationkf_amd import _lib
    try:
        return _main(argv)
    except (_lib.CommTimeoutError, _lib.PekfError) as e:
        if isinstance(e, _lib.CommTimeoutError) or e.status == _lib.PEKF_ERR_COMM:
            # an abandoned RCCL init thread (or an aborted communicator) may still hold RCCL's locks, so
            # leave without the interpreter's and the runtimes' exit handlers
            print("[bench] error: collective failed: %s" % e, file=sys.stderr, flush=True)
            os._exit(2)
        raise
    except TimeoutError as e:   # FileRendezvous: no RCCL id from rank 0 within PEKF_RDZV_TIMEOUT_S
        raise BenchError(str(e))
    except RuntimeError as e:   # FileRendezvous: rank 0 failed before it had an id
        from poseestimationkf_amd import shard
        if isinstance(e, shard.RendezvousError):
            raise BenchError(str(e))
        raise


def _main(argv=None):
    args = parse_args(argv)
    plan = launch_plan(args.gpus, os.environ, args.shard_of, args.one_process)
    rank, world = plan["rank"], plan["world"]
    out_fd = StdoutForTheResult()
    rdzv = None
    if plan["mode"] == "ranks" and (world > 1 or args.dist):
        from poseestimationkf_amd import shard
        rdzv = shard.FileRendezvous(rank, world)

    try:
        # CPU baseline first (rank 0, every N), in forked workers, before anything touches the GPU;
        # the other ranks wait for rank 0's RCCL id meanwhile.
        cpu = None
        if args.cpu_baseline == "port" and rank == 0:
            log("cpu baseline (NumPy restatement) ...")
            cpu = cpu_baseline(args.seed, args.missing, args.cpu_filters_per_core, args.cpu_records)
            try:
                cpu["c_oracle"] = c_oracle_rate(args.seed, args.missing)
            except Exception as e:  # the C oracle is optional for the baseline line
                cpu["c_oracle"] = {"error": str(e)}
            log("cpu baseline: %.0f steps/s on %d cores (%s)" % (cpu["value"], cpu["cores"], cpu["share_source"]))

        from poseestimationkf_amd import _lib
        visible = _lib.device_count()
        if plan["mode"] == "ranks" and visible == 1 and plan["devices"][0] > 0:
            plan["devices"] = [0]   # the launcher gave each rank its own GPU (HIP/CUDA_VISIBLE_DEVICES)
        need = max(plan["devices"]) + 1
        if visible < need:
            raise BenchError("--gpus %d (%s) needs %d visible GPU(s), %d visible" %
                             (args.gpus, plan["mode"], need, visible))
    except BaseException as e:
        if rdzv is not None:   # rank 0 exits before it has an id: the other ranks stop waiting for one
            rdzv.fail("%s: %s" % (type(e).__name__, e))
        raise

    run = MultiRun(args, plan) if plan["mode"] == "multi" else RankRun(args, plan, rdzv)
    N, W = args.records, args.window
    total = args.warmup + args.steps
    run.prepare(total)

    for k in range(args.warmup):
        run.step(k, N, (k * N) % W)
        if k == args.warmup - 1:
            run.gather()   # the communicator's first collective pays RCCL's connection setup: not timed
        run.sync()
        log("warmup %d: kernel %.1f ms%s" % (k, run.kernel_ms(k), ", gather %.3f ms" % run.gather_ms()
                                            if k == args.warmup - 1 else ""))

    run.sync()
    run.barrier()
    t0 = time.perf_counter()
    for k in range(args.warmup, total):
        run.step(k, N, (k * N) % W)
    run.gather()           # ONE gather of the final quaternions, inside the timed region
    run.sync()
    run.barrier()
    elapsed = run.slowest(time.perf_counter() - t0)
    timed = range(args.warmup, total)
    kms = [run.kernel_ms(k) for k in timed]
    per_gpu = run.per_gpu(timed)
    log("timed: %.3f s for %d steps on %d GPU(s); kernel ms per GPU %s; gather ms per GPU %s" %
        (elapsed, args.steps, world, ", ".join("%.1f" % v for v in per_gpu[0]),
         ", ".join("%.3f" % v for v in per_gpu[1])))

    # final quaternions of every GPU's filters on rank 0 (the gathered rows), then all ranks part
    rows = run.final_rows() if rank == 0 and args.parity_samples > 0 else None
    run.barrier()
    parity = None
    if rows is not None:
        samples = max(args.parity_samples, 4 * world)
        parity = parity_check(rows[0], rows[1], samples, total * N, args)
        log("parity: max |dq| = %.3e over %d sampled filters of shards %s" %
            (parity["max_abs_err_vs_oracle"], parity["filters"], parity["shards_covered"]))

    if rank == 0:
        out = result_line(args, plan, elapsed, kms, cpu, parity, per_gpu)
        out_fd.emit(json.dumps(out))
    run.close()
    if parity is not None and not (parity["ok"] and parity["unit_norm_all"]):
        raise SystemExit("parity failed: %r" % parity)


def result_line(args, plan, elapsed, kms, cpu, parity, per_gpu=None):
    import numpy as np
    world, B, N = plan["world"], args.batch, args.records
    steps_total = world * B * N * args.steps
    value = steps_total / elapsed
    if per_gpu is None:
        per_gpu = ([float(np.mean(kms))], [0.0])
    # one GPU's launch: the slowest GPU's mean kernel time (the GPU that bounds the step, as ms_per_step)
    k_s = float(np.max(per_gpu[0])) / 1e3
    achieved = B * N * REC_BYTES / k_s / 1e9
    counts = ISA_COUNTS[args.precision]
    valu = counts["valu_instr"]
    wave_instr = (B / 64.0) * N * valu
    cited = cited_profile(B, N) if args.precision == "f64" and not args.missing else None
    launch = {"ranks": "one process per GPU (launcher ranks; RCCL id through shard.FileRendezvous)",
              "single": "one process, one GPU",
              "multi": "one process over GPUs %s (ncclCommInitAll, grouped gather)" % plan["devices"]}[plan["mode"]]
    return {
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
                "%d-record resident window replayed cyclically)" % args.window,
        "config": {"workload": workload_name(B, N, args.missing, world),
                   "filters_per_gpu": B, "global_filters": B * world, "records_per_step": N,
                   "window_records": args.window,
                   "first_filter": plan["first_shard"] * B if plan["mode"] == "single" else 0,
                   "parallelism": "dp%d (filter-batch shards%s)" % (
                       world, ", no per-step exchange, 1 RCCL gather of the final quaternions"
                       if world > 1 or args.dist or plan["mode"] == "multi" else ""),
                   "launch": launch},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": cited["hbm_traffic_bytes"] if cited else None,
                     "traffic_source": ("cited, not measured in this run: %s (2 x FETCH_SIZE of a separate "
                                        "rocprofv3 --pmc pass of this command on an earlier box)" % cited["path"])
                                       if cited else None,
                     "per": "one GPU's launch: the slowest GPU's mean over the timed steps",
                     "kernel": "k_run<false> (pekf_run_dev)", "kernel_ms": k_s * 1e3,
                     "kernel_ms_mean_over_gpus": float(np.mean(per_gpu[0])),
                     "bytes_per_launch": B * N * REC_BYTES,
                     "binding_resource": "FP64 VALU issue, not HBM: see valu_roofline"},
        "valu_roofline": {"bound": "fp64-valu-issue", "achieved": wave_instr / k_s / 1e9, "peak": VALU_PEAK_GWIPS,
                          "unit": "G wave-instr/s", "frac": wave_instr / k_s / 1e9 / VALU_PEAK_GWIPS,
                          "valu_per_filter_step": valu,
                          "valu_source": "static count of the hot loop's executed blocks (scripts/loop_blocks.py, "
                                         "DESIGN.md §4.2); the PMC pass counts %s per wave-step" %
                                         ("%.1f" % cited["valu_insts_per_wave_step"] if cited else "the same"),
                          "peak_note": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 FP64 instruction "
                                       "(= the 78.6 TFLOP/s FP64 vector peak); the clock under this load is "
                                       "power-limited below 2.4 GHz",
                          "flop_per_step": counts["flop"], "fp64_instr_per_step": counts["fp64_instr"],
                          "achieved_tflops": B * N * counts["flop"] / k_s / 1e12, "peak_tflops": FP64_PEAK_TFLOPS},
        "cited_profile": ({"path": cited["path"], "valu_busy": cited.get("valu_busy"),
                           "clock_ghz": cited.get("effective_clock_ghz"),
                           "note": "from the committed rocprofv3 PMC passes of this command, not this run"}
                          if cited else None),
        "cpu_baseline": cpu,
        "parity": parity,
        "kernel_ms_per_gpu": per_gpu[0],
        "gather_ms_per_gpu": per_gpu[1],
        "timing_note": "per GPU, in rank order: the fused launch's mean HIP-event time over the timed steps and "
                       "the final RCCL gather's time on that GPU's stream (it includes waiting for the slowest "
                       "peer's last launch; 0 when nothing is gathered); "
                       "ms_per_step is the slowest rank's wall clock",
    }


# per filter-step: the VALU instructions of the basic blocks a tracked lane executes in k_run's hot
# loop (scripts/loop_blocks.py on the hipcc -S listing: the fallback bodies sit behind
# s_cbranch_execz); FP64 instructions and FLOP (FMA = 2) from scripts/isa_count.py on the same blocks.
# The PMC pass in profiles/ counts the executed total (SQ_INSTS_VALU per wave-step).
ISA_COUNTS = {"f64": {"flop": 436, "fp64_instr": 298, "valu_instr": 301},
              "mixed": {"flop": 240, "fp64_instr": 191, "valu_instr": 329}}  # mixed: + ~130 f32 instructions
FLOP_PER_STEP = ISA_COUNTS["f64"]["flop"]
FP64_INSTR_PER_STEP = ISA_COUNTS["f64"]["fp64_instr"]


def workload_name(batch, records, missing, world=1):
    """BASELINE.json's configuration this run is (configs 2-5 are 10,000 records)."""
    if records == 10000 and batch == 1 << 20:
        if missing:
            return "config 5: batch=1,048,576/GPU, 30% missing-mag" + (" x %d GPUs" % world if world > 1 else "")
        if world == 8:
            return "config 4: batch=8,388,608 filters sharded 8-way x 10,000 records"
        if world > 1:
            return "config 3 per GPU x %d GPUs: batch=%d filters x 10,000 records" % (world, batch * world)
        return "config 3: batch=1,048,576 filters/GPU x 10,000 records"
    if records == 10000 and batch == 65536 and not missing and world == 1:
        return "config 2: batch=65,536 filters/GPU x 10,000 records"
    return "custom: batch=%d filters/GPU x %d records x %d GPU(s)%s" % (
        batch, records, world, ", 30% missing-mag" if missing else "")


def cited_profile(batch, records):
    """The committed rocprofv3 PMC summary of the current build (profiles/HEADLINE_PMC names it;
    scripts/refresh.sh produces it), if its config matches; its numbers are cited, not measured."""
    try:
        with open(os.path.join(ROOT, "profiles", "HEADLINE_PMC")) as fh:
            rel = fh.read().strip()
        with open(os.path.join(ROOT, rel)) as fh:
            s = json.load(fh)
    except OSError:
        return None
    if s.get("config") != {"batch": batch, "records": records}:
        return None
    return dict(s, path=rel)


if __name__ == "__main__":
    main()
