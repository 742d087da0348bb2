"""N > 1 path on CPU.

* Torch-free rendezvous (shard.FileRendezvous, what bench.py uses under torchrun): two processes
  children of one parent -- as torchrun's ranks are -- share rank 0's 128-byte RCCL id through a file,
  with no PyTorch imported; a file from another job (another key) or a torn / foreign file is never
  taken for the id.
* world_size-2 gloo ranks: each takes its contiguous filter shard, runs it (the C oracle stands in
  for the device here -- test only), and the shards' final quaternions, concatenated in rank order
  as pekf_gather_dev lays them out on the root, equal a single-process run.  gloo only stands in
  for the RCCL gather (which needs GPUs: tests/test_gpu_comm.py and bench.py on the box)."""
import os
import re
import socket
import sys

import numpy as np
import pytest

from poseestimationkf_amd import shard, synth

ID = bytes(range(128))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard_rows(rank, world, global_batch, window):
    from oracle import oracle_c
    first, count = shard.shard_range(global_batch, rank, world)
    X, _, _ = oracle_c.run(synth.generate(np.arange(first, first + count), window))
    return X


def _rdzv_rank(rank, world, port, directory, global_batch, window, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    uid = shard.FileRendezvous(rank, world, directory=directory, timeout=60).share_id(make_id=lambda: ID)
    rows = _shard_rows(rank, world, global_batch, window)
    q.put((rank, uid, rows, "torch" in sys.modules))


def test_file_rendezvous_two_processes_torch_free(tmp_path):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rdzv_rank, args=(r, 2, port, str(tmp_path), 16, 24, q)) for r in (1, 0)]
    for p in procs:
        p.start()
    got = dict((r, (uid, rows, torch)) for r, uid, rows, torch in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == ID and got[1][0] == ID            # rank 1 read rank 0's id
    assert not got[0][2] and not got[1][2]                # no PyTorch in either rank
    X, _, _ = __import__("oracle.oracle_c", fromlist=["run"]).run(synth.generate(np.arange(16), 24))
    assert np.array_equal(np.concatenate([got[0][1], got[1][1]]), X)


def test_file_rendezvous_key_isolation_and_cleanup(tmp_path):
    r0 = shard.FileRendezvous(0, 2, key="jobA", directory=str(tmp_path))
    assert r0.share_id(make_id=lambda: ID) == ID
    assert os.path.exists(r0.path)
    # another job's file (other key) is never read
    with pytest.raises(TimeoutError):
        shard.FileRendezvous(1, 2, key="jobB", directory=str(tmp_path), timeout=0.2).share_id()
    assert shard.FileRendezvous(1, 2, key="jobA", directory=str(tmp_path), timeout=5).share_id() == ID
    # a foreign or torn file is not taken for the id
    bad = shard.FileRendezvous(1, 2, key="jobC", directory=str(tmp_path), timeout=0.2)
    with open(bad.path, "wb") as fh:
        fh.write(b"PEKFRDZV1" + ID[:100])
    with pytest.raises(TimeoutError):
        bad.share_id()
    r0.done()
    assert not os.path.exists(r0.path)
    # world 1 needs no file at all; a bad id size is refused
    solo = shard.FileRendezvous(0, 1, key="solo", directory=str(tmp_path))
    assert solo.share_id(make_id=lambda: ID) == ID and not os.path.exists(solo.path)
    with pytest.raises(RuntimeError):
        shard.FileRendezvous(0, 2, key="short", directory=str(tmp_path)).share_id(make_id=lambda: b"x")
    with pytest.raises(ValueError):
        shard.FileRendezvous(2, 2)


def test_default_key_is_shared_by_siblings_only(monkeypatch):
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "29999")
    monkeypatch.delenv("PEKF_RDZV_KEY", raising=False)
    for k in ("TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT"):
        monkeypatch.delenv(k, raising=False)
    a, b = shard.FileRendezvous(0, 2), shard.FileRendezvous(1, 2)
    assert a.path == b.path and str(os.getppid()) in a.path
    monkeypatch.setenv("MASTER_PORT", "29998")
    assert shard.FileRendezvous(1, 2).path != a.path
    monkeypatch.setenv("PEKF_RDZV_KEY", "k/../x")
    assert os.path.basename(shard.FileRendezvous(1, 2).path) == "pekf-rdzv-k_.._x_127.0.0.1_29998.id"


def test_file_rendezvous_under_torchrun(tmp_path):
    """The launcher the driver uses for N > 1 (torchrun, 3 ranks here): every rank gets rank 0's id
    through the file channel, keyed by the torchrun agent (the ranks' common parent), torch-free."""
    import subprocess
    env = dict(os.environ, PEKF_RDZV_DIR=str(tmp_path))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "PEKF_RDZV_KEY"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                          os.path.join(os.path.dirname(__file__), "_rdzv_probe.py")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    # the ranks share torchrun's stdout, so their lines may interleave: take each report wherever it is
    lines = sorted(re.findall(r"RDZV rank=\d+ ok=\d torch=\d", out.stdout))
    assert lines == ["RDZV rank=%d ok=1 torch=0" % r for r in range(3)], out.stdout


def _gloo_rank(rank, world, port, directory, global_batch, window, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    uid = shard.FileRendezvous(rank, world, directory=directory, timeout=60).share_id(make_id=lambda: ID)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X = _shard_rows(rank, world, global_batch, window)
        bufs = [torch.empty_like(torch.from_numpy(X)) for _ in range(world)] if rank == 0 else None
        dist.gather(torch.from_numpy(X), gather_list=bufs, dst=0)  # stands in for RCCL (test only)
        if rank == 0:
            q.put((uid, torch.cat(bufs, dim=0).numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_batch_exactly():
    ranges = [shard.shard_range(1 << 20, r, 8) for r in range(8)]
    assert ranges[0] == (0, 1 << 17) and ranges[-1] == (7 << 17, 1 << 17)
    assert sum(c for _, c in ranges) == 1 << 20
    c4 = [shard.shard_range(8 << 20, r, 8) for r in range(8)]
    assert c4[7] == (7 << 20, 1 << 20) and sum(c for _, c in c4) == 8_388_608
    with pytest.raises(ValueError):
        shard.shard_range(10, 0, 3)


def test_two_rank_gloo_gather_equals_single_process(tmp_path):
    import multiprocessing as mp

    from oracle import oracle_c
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, str(tmp_path), 16, 24, q)) for r in range(2)]
    for p in procs:
        p.start()
    uid, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X, _, _ = oracle_c.run(synth.generate(np.arange(16), 24))
    assert uid == ID
    assert got.shape == (16, 4)
    assert np.array_equal(got, X)


def test_rendezvous_multinode_needs_a_key_and_rank0_failure_is_published(tmp_path):
    """A job spanning nodes (torchrun's GROUP_WORLD_SIZE > 1, or WORLD_SIZE != LOCAL_WORLD_SIZE) has no
    common parent, so the default key is refused at once; with PEKF_RDZV_KEY it is accepted.  A rank 0
    that fails before it has an id publishes the failure, and a waiting rank raises at once."""
    env = {"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "8", "GROUP_WORLD_SIZE": "2"}
    with pytest.raises(ValueError, match="PEKF_RDZV_KEY"):
        shard.FileRendezvous(3, 16, directory=str(tmp_path), environ=env)
    with pytest.raises(ValueError, match="PEKF_RDZV_KEY"):
        shard.FileRendezvous(3, 16, directory=str(tmp_path), environ={"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "8"})
    ok = shard.FileRendezvous(3, 16, directory=str(tmp_path), environ=dict(env, PEKF_RDZV_KEY="job42"))
    assert os.path.basename(ok.path) == "pekf-rdzv-job42.id"
    assert shard.FileRendezvous(1, 8, directory=str(tmp_path),
                                environ={"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}).path   # one node: default key
    r0 = shard.FileRendezvous(0, 2, key="jobF", directory=str(tmp_path))
    r0.fail("BenchError: no GPU")
    r1 = shard.FileRendezvous(1, 2, key="jobF", directory=str(tmp_path), timeout=60)
    import time
    t0 = time.monotonic()
    with pytest.raises(shard.RendezvousError, match="no GPU"):
        r1.share_id()
    assert time.monotonic() - t0 < 5
    assert shard.FileRendezvous(0, 2, key="t", directory=str(tmp_path), environ={"PEKF_RDZV_TIMEOUT_S": "7"}).timeout == 7


def test_rendezvous_relaunch_with_the_same_key_after_a_failure(tmp_path):
    """A launch whose rank 0 failed leaves its failure marker behind.  A relaunch with the same
    PEKF_RDZV_KEY never reads it: a new master port or torchrun run id / restart count gives the
    launch its own file, and with everything equal the new rank 0 removes the stale file when it starts."""
    d = str(tmp_path)
    env1 = {"PEKF_RDZV_KEY": "job7", "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": "29500",
            "TORCHELASTIC_RUN_ID": "none", "TORCHELASTIC_RESTART_COUNT": "0"}
    shard.FileRendezvous(0, 2, directory=d, environ=env1).fail("BenchError: no GPU")
    stale = shard.FileRendezvous(1, 2, directory=d, environ=env1, timeout=0.2)
    assert os.path.basename(stale.path) == "pekf-rdzv-job7_0_10.0.0.1_29500.id" and os.path.exists(stale.path)
    for change in ({"MASTER_PORT": "29501"}, {"TORCHELASTIC_RESTART_COUNT": "1"}, {"TORCHELASTIC_RUN_ID": "abc"}):
        r1 = shard.FileRendezvous(1, 2, directory=d, environ=dict(env1, **change), timeout=0.2)
        assert r1.path != stale.path
        with pytest.raises(TimeoutError):     # waits for its own launch's rank 0, not the stale marker
            r1.share_id()
    # the identical relaunch: its rank 0 removes the marker at start, then publishes a fresh id
    r0 = shard.FileRendezvous(0, 2, directory=d, environ=env1)
    assert not os.path.exists(stale.path)
    assert r0.share_id(make_id=lambda: ID) == ID
    assert shard.FileRendezvous(1, 2, directory=d, environ=env1, timeout=5).share_id() == ID


def test_connect_publishes_the_failure_when_communicator_creation_fails(tmp_path, monkeypatch):
    """When rank 0's communicator creation raises (an init timeout, after which bench.py leaves with
    os._exit), its published id is replaced by the failure marker: a rank that has not read the id yet
    raises at once instead of waiting out PEKF_RDZV_TIMEOUT_S, and no rank can read the spent id.  On
    success the id file is removed."""
    class Boom(RuntimeError):
        pass

    def failing_init(self, uid, nranks, rank, _handle=None):
        raise Boom("init timed out")

    monkeypatch.setattr(shard.Communicator, "__init__", failing_init)
    r0 = shard.FileRendezvous(0, 2, key="jobC", directory=str(tmp_path), environ={})
    monkeypatch.setattr(shard.Communicator, "unique_id", staticmethod(lambda: ID))
    with pytest.raises(Boom):
        shard.connect(0, 2, r0)
    import time
    t0 = time.monotonic()
    with pytest.raises(shard.RendezvousError, match="init timed out"):
        shard.FileRendezvous(1, 2, key="jobC", directory=str(tmp_path), environ={}, timeout=60).share_id()
    assert time.monotonic() - t0 < 5

    def fake_init(self, uid, nranks, rank, _handle=None):
        self.handle = None
    monkeypatch.setattr(shard.Communicator, "__init__", fake_init)
    r0 = shard.FileRendezvous(0, 2, key="jobD", directory=str(tmp_path), environ={})
    assert isinstance(shard.connect(0, 2, r0), shard.Communicator)
    assert not os.path.exists(r0.path)
