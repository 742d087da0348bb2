"""bench.py's N > 1 code paths, executed end to end on the CPU against a host fake of libpekf
(tests/fake_libpekf.py: host memory for device memory, the C oracle for the fused launch, gloo for
RCCL between processes).  Everything above the C ABI -- bench.py, engine.py, shard.py -- is the
code the driver's 8-GPU run executes:

* one process over 8 devices (`bench.py --gpus 8`: shard.MultiDeviceEKF, ncclCommInitAll, one
  grouped gather of the final quaternions);
* one process per rank (`torchrun ... bench.py --gpus 2`, `4` and `8`: FileRendezvous, RCCL init, the final
  gather, max-over-ranks time, per-GPU timings exchanged by one all-reduce);
* rank 0 failing before it has an RCCL id: the other rank stops waiting and exits 2 at once;
* the one-process mode failing instead of hanging: a grouped gather that never completes on one of
  the 8 devices, or an ncclCommInitAll that never returns, ends bench.py with status 2 within the
  PEKF_COMM_TIMEOUT_S deadline, one stderr line and nothing on stdout.

Filters are independent (PKF/ExtendedKalmanFilter.py:6-80), so each shard's rows must equal the
oracle's run of those global filter ids (main_file.py:38-47's loop), wherever they were computed."""
import json
import os
import socket
import sys
import time

import numpy as np
import pytest

from .conftest import ROOT

SMALL = ["--batch", "256", "--records", "16", "--window", "8", "--steps", "2", "--warmup", "1",
         "--cpu-filters-per-core", "2", "--cpu-records", "10", "--parity-samples", "16"]


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _one_line(text):
    lines = [l for l in text.splitlines() if l.strip()]
    assert len(lines) == 1, text
    return json.loads(lines[0])


def _check_line(d, world, batch=256):
    assert d["n_gpus"] == world and d["config"]["global_filters"] == world * batch
    assert d["config"]["filters_per_gpu"] == batch and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    p = d["parity"]
    assert p["shards_covered"] == list(range(world)), p
    assert p["ok"] and p["max_abs_err_vs_oracle"] == 0.0 and p["unit_norm_all"]
    assert p["global_filter_ids"] == [0, world * batch - 1]
    cpu = d["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["share_source"]
    assert len(d["kernel_ms_per_gpu"]) == world and all(v > 0 for v in d["kernel_ms_per_gpu"])
    assert len(d["gather_ms_per_gpu"]) == world and all(v >= 0 for v in d["gather_ms_per_gpu"])
    assert d["roofline"]["kernel_ms"] == pytest.approx(float(np.max(d["kernel_ms_per_gpu"])))
    assert d["roofline"]["kernel_ms_mean_over_gpus"] == pytest.approx(float(np.mean(d["kernel_ms_per_gpu"])))


def test_one_process_eight_devices(monkeypatch, capfd):
    """`bench.py --gpus 8` with no launcher: one process drives devices 0..7."""
    from . import fake_libpekf
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    fake = fake_libpekf.install(monkeypatch, n_devices=8)
    bench = _bench()
    bench.main(["--gpus", "8"] + SMALL)
    out, err = capfd.readouterr()
    d = _one_line(out)
    _check_line(d, 8)
    assert "ncclCommInitAll" in d["config"]["launch"] and d["config"]["workload"].startswith("custom")
    assert fake.calls.count("pekf_comm_init_all") == 1
    assert fake.calls.count("pekf_gather_multi_dev") == 2          # after the warmup + ONE after the timed steps
    assert sorted({r[0] for r in fake.runs}) == list(range(8))     # every device ran its shard
    assert all(r[1:] == (256, 16, (k // 8) * 16 % 8) for k, r in enumerate(fake.runs))


def _rank_main(rank, world, env, out_path, n_devices):
    """One torchrun-style rank: RANK / WORLD_SIZE / LOCAL_RANK in the environment, bench.main in-process."""
    os.environ.update(env, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    from tests import fake_libpekf
    fake_libpekf.install(None, n_devices=n_devices, gloo_port=int(env["FAKE_GLOO_PORT"]))
    fd = os.open(out_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(fd, 1)
    import bench
    code = 0
    try:
        bench.main(["--gpus", str(world)] + SMALL)
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else 1
    sys.stdout.flush()
    os._exit(code)


def _run_ranks(tmp_path, world, n_devices_of=lambda r: 1, timeout=240):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()), "FAKE_GLOO_PORT": str(_free_port()),
           "PEKF_RDZV_DIR": str(tmp_path), "PEKF_RDZV_TIMEOUT_S": "120"}
    outs = [str(tmp_path / ("rank%d.out" % r)) for r in range(world)]
    procs = [ctx.Process(target=_rank_main, args=(r, world, env, outs[r], n_devices_of(r))) for r in range(world)]
    t0 = time.monotonic()
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    texts = []
    for o in outs:
        with open(o) as fh:
            texts.append(fh.read())
    return codes, texts, time.monotonic() - t0


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_one_process_each(tmp_path, world):
    """`torchrun --nproc-per-node N bench.py --gpus N`: N processes, rank 0 prints the one line."""
    codes, texts, _ = _run_ranks(tmp_path, world)
    assert codes == [0] * world, texts
    d = _one_line(texts[0])
    assert all(t.strip() == "" for t in texts[1:])                 # only rank 0 prints
    _check_line(d, world)
    assert d["config"]["launch"].startswith("one process per GPU")
    assert all(v > 0 for v in d["gather_ms_per_gpu"])              # gloo gathers, host-timed


def test_rank0_failure_releases_the_other_ranks(tmp_path):
    """Rank 0 cannot start (no GPU visible to it): it publishes the failure through the rendezvous file,
    rank 1 stops waiting at once (not after PEKF_RDZV_TIMEOUT_S) and both exit 2 with nothing on stdout."""
    codes, texts, wall = _run_ranks(tmp_path, 2, n_devices_of=lambda r: 0 if r == 0 else 1)
    assert codes == [2, 2], (codes, texts)
    assert texts == ["", ""]
    assert wall < 100


def _plain_main(env, out_path, err_path, t_path, stuck_devices, init_all_stalls):
    """`bench.py --gpus 8` launched plainly (one process over 8 fake devices) with a fault injected."""
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    os.environ.update(env)
    sys.path.insert(0, ROOT)
    from tests import fake_libpekf
    fake = fake_libpekf.install(None, n_devices=8)
    fake.stuck_devices = set(stuck_devices)
    fake.init_all_stalls = init_all_stalls
    for fd, path in ((1, out_path), (2, err_path)):
        os.dup2(os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC), fd)
    import bench
    with open(t_path, "w") as fh:
        fh.write(repr(time.monotonic()))
    code = 0
    try:
        bench.main(["--gpus", "8", "--cpu-baseline", "none"] + SMALL)
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else 1
    sys.stdout.flush()
    os._exit(code)


@pytest.mark.parametrize("fault", ["gather_on_device_5", "init_all"])
def test_one_process_fails_instead_of_hanging(tmp_path, fault):
    """The plain `bench.py --gpus 8` (MultiDeviceEKF) with a collective that never completes: a grouped
    gather stuck on device 5 (MultiRun.sync -> MultiDeviceEKF.sync -> pekf_comm_wait per device), or an
    ncclCommInitAll that never returns (pekf_comm_init_all_timeout).  bench.py exits 2 within the 2 s
    PEKF_COMM_TIMEOUT_S deadline plus its own start-up, with one error line and nothing on stdout."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    out, err, tp = (str(tmp_path / n) for n in ("out", "err", "t0"))
    p = ctx.Process(target=_plain_main, args=({"PEKF_COMM_TIMEOUT_S": "2"}, out, err, tp,
                                              [5] if fault == "gather_on_device_5" else [], fault == "init_all"))
    p.start()
    p.join(timeout=120)
    t_end = time.monotonic()
    if p.exitcode is None:
        p.kill()
    with open(err) as fh:
        err_text = fh.read()
    assert p.exitcode == 2, err_text
    with open(tp) as fh:
        t0 = float(fh.read())
    assert 2.0 <= t_end - t0 < 15, (t_end - t0, err_text)
    with open(out) as fh:
        assert fh.read() == ""
    failed = [l for l in err_text.splitlines() if "collective failed" in l]
    assert len(failed) == 1, err_text
    if fault == "init_all":
        assert "ncclCommInitAll not done within 2 s" in failed[0]
    else:
        assert "did not complete within 2 s" in failed[0] and "rank 5 of 8" in failed[0]


def test_cpu_share_from_cgroup_v2(tmp_path):
    """The GPU box's layout: the leaf cgroup directory hidden by the namespace, an unlimited middle
    level, the job's quota (16 CPUs) at the mount root, and a 256-CPU affinity mask."""
    bench = _bench()
    root = tmp_path / "cg"
    (root / "process_api").mkdir(parents=True)
    (root / "cgroup.controllers").write_text("cpuset cpu io memory\n")
    (root / "cpu.max").write_text("1600000 100000\n")
    (root / "cpuset.cpus.effective").write_text("0-255\n")
    (root / "process_api" / "cpu.max").write_text("max 100000\n")
    pc = tmp_path / "cgroup"
    pc.write_text("0::/process_api/8282ea0a\n")
    s = bench.cpu_share({"OMP_NUM_THREADS": "16"}, str(pc), str(root), affinity=256)
    assert s["use"] == 16 and s["quota_cores"] == 16 and s["cpuset_cores"] == 256
    assert s["share_source"].startswith("cgroup v2 CPU quota") and str(root / "cpu.max") in s["share_source"]
    # a tighter quota deeper down wins; a cpuset narrower than the quota wins over it
    (root / "process_api" / "cpu.max").write_text("250000 100000\n")
    assert bench.cpu_share({}, str(pc), str(root), affinity=256)["use"] == 2
    (root / "process_api" / "cpuset.cpus.effective").write_text("4,7\n")
    (root / "process_api" / "cpu.max").write_text("max 100000\n")
    s = bench.cpu_share({}, str(pc), str(root), affinity=256)
    assert s["use"] == 2 and "cpuset" in s["share_source"]
    assert bench._cpulist_count("0-3,8,10-11") == 7 and bench._cpulist_count("") == 0


def test_cpu_share_from_cgroup_v1(tmp_path):
    bench = _bench()
    root = tmp_path / "cg"
    (root / "cpu,cpuacct" / "job").mkdir(parents=True)
    (root / "cpuset" / "job").mkdir(parents=True)
    (root / "cpu,cpuacct" / "cpu.cfs_quota_us").write_text("-1\n")
    (root / "cpu,cpuacct" / "cpu.cfs_period_us").write_text("100000\n")
    (root / "cpu,cpuacct" / "job" / "cpu.cfs_quota_us").write_text("800000\n")
    (root / "cpu,cpuacct" / "job" / "cpu.cfs_period_us").write_text("100000\n")
    (root / "cpuset" / "job" / "cpuset.effective_cpus").write_text("0-31\n")
    pc = tmp_path / "cgroup"
    pc.write_text("5:cpuset:/job\n4:cpu,cpuacct:/job\n1:name=systemd:/job\n")
    s = bench.cpu_share({}, str(pc), str(root), affinity=64)
    assert s["use"] == 8 and s["quota_cores"] == 8 and s["cpuset_cores"] == 32
    assert "v1 CPU quota" in s["share_source"]


def test_cpu_share_without_cgroup_limits(tmp_path):
    """No quota and no cpuset: OMP_NUM_THREADS is the declared share if set, else every affinity core."""
    bench = _bench()
    missing = str(tmp_path / "none")
    s = bench.cpu_share({}, missing, missing, affinity=12)
    assert s["use"] == 12 and s["share_source"] == "sched_getaffinity"
    s = bench.cpu_share({"OMP_NUM_THREADS": "3"}, missing, missing, affinity=12)
    assert s["use"] == 3 and s["share_source"].startswith("OMP_NUM_THREADS")
