"""The sharded path's collective through the C ABI (pekf_comm_* / pekf_gather_dev) on
the GPU: RCCL communicators of world size 1 (the box has one GPU; N > 1 is the driver's 8-GPU bench,
and tests/test_shard_gloo.py covers the rendezvous and shard layout with two CPU ranks)."""
import numpy as np
import pytest

from poseestimationkf_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from poseestimationkf_amd import engine
    from poseestimationkf_amd._lib import device_count
    assert device_count() > 0, "GPU tests need a HIP device"
    engine.set_device(0)
    return engine


@pytest.fixture(scope="module")
def comm(eng):
    from poseestimationkf_amd import shard
    c = shard.Communicator(shard.Communicator.unique_id(), 1, 0)
    yield c
    c.close()


def test_rccl_loaded_and_communicator_fields(eng, comm):
    from poseestimationkf_amd import shard
    assert shard.rccl_version() >= 21800  # ncclGather appeared in RCCL 2.18
    assert (comm.rank, comm.nranks, comm.device) == (0, 1, 0)
    assert len(shard.Communicator.unique_id()) == shard.COMM_ID_BYTES


def test_gather_world1_copies_exactly(eng, comm):
    from poseestimationkf_amd import shard
    B = 1 << 18
    x = np.random.default_rng(3).standard_normal((B, 4))
    src = eng.DeviceBuffer(x.nbytes).upload(x)
    s = eng.Stream()
    out = shard.gather_quaternions(comm, src.ptr, B, stream=s.handle)
    s.sync()
    assert np.array_equal(out.download((B, 4), np.float64), x)


def test_allreduce_max_world1_and_argument_errors(eng, comm):
    from poseestimationkf_amd._lib import PekfError
    v = np.array([3.5, -1.0, np.inf], np.float64)
    buf = eng.DeviceBuffer(v.nbytes).upload(v)
    s = eng.Stream()
    comm.allreduce_max(buf.ptr, 3, s.handle)
    s.sync()
    assert np.array_equal(buf.download((3,), np.float64), v)
    with pytest.raises(PekfError):
        comm.gather(buf.ptr, 3, buf.ptr, root=1)  # root out of range
    with pytest.raises(PekfError):
        comm.gather(buf.ptr, 3, None, root=0)     # the root needs a receive buffer


def test_bad_unique_id_rejected(eng):
    from poseestimationkf_amd import shard
    with pytest.raises(ValueError):
        shard.Communicator(b"short", 1, 0)


def test_multi_device_ekf_equals_single_batch(eng):
    """Single-process sharding (ncclCommInitAll + grouped gather) over the visible GPUs (one here):
    the gathered final X equal a plain BatchedEKF run of the same filters bit for bit."""
    from poseestimationkf_amd import shard
    B, W, n = 4096, 64, 300
    m = shard.MultiDeviceEKF([0], B, W).synthesize(seed=synth.DEFAULT_SEED)
    m.run_async(n, 0)
    m.gather_async()
    m.sync()
    got = m.gathered()
    m.close()
    win = eng.IMUWindow(B, W).synthesize(seed=synth.DEFAULT_SEED)
    f = eng.BatchedEKF(B)
    f.run(win, n, 0)
    X, _ = f.get_state()
    assert np.array_equal(got, X)
    assert np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-12)


def _busy_gather(eng, comm, stream, gib=8):
    """A world-1 gather of `gib` GiB: a collective that stays in flight for milliseconds (>= 2 GiB of HBM
    traffic per GiB at 8 TB/s) -- with one GPU there is no peer to withhold, so this is the stand-in for
    a collective a dead peer never completes.  Returns the buffers (keep them alive until the stream drains)."""
    n = (gib << 30) // 8
    send, recv = eng.DeviceBuffer(8 * n), eng.DeviceBuffer(8 * n)
    comm.gather(send.ptr, n, recv.ptr, 0, stream)
    return send, recv


def test_comm_wait_deadline_charges_collectives_not_compute(eng):
    """pekf_comm_wait's deadline runs per collective from the moment the stream reaches it: ~120 ms of fused
    launches queued ahead of (and between) collectives pass a 5 ms deadline, while a collective that stays
    in flight past it aborts the communicator with CommTimeoutError (a long compute queue was
    reported as a dead peer)."""
    import time

    from poseestimationkf_amd import shard
    from poseestimationkf_amd._lib import CommTimeoutError, PekfError
    c = shard.Communicator(shard.Communicator.unique_id(), 1, 0)
    B = 1 << 18
    win = eng.IMUWindow(B, 64).synthesize(seed=synth.DEFAULT_SEED)
    f = eng.BatchedEKF(B)
    s = eng.Stream()
    c.wait(s.handle, timeout=5)                      # idle stream: returns
    recv = eng.DeviceBuffer(32 * B)
    t0 = time.monotonic()
    for k in range(2):                               # as RankRun queues warmup + timed steps, then waits once
        f.run_async(win, 20000, 0, s.handle)         # ~60 ms of work
        shard.gather_quaternions(c, f.X.ptr, B, recv, 0, s.handle)
    c.wait(s.handle, timeout=0.005)
    assert time.monotonic() - t0 > 0.05               # it did wait for the compute
    X, _ = f.get_state()
    assert np.array_equal(recv.download((B, 4), np.float64), X)
    bufs = _busy_gather(eng, c, s.handle)
    t0 = time.monotonic()
    with pytest.raises(CommTimeoutError, match="ncclGather did not complete within"):
        c.wait(s.handle, timeout=0.0005)
    assert time.monotonic() - t0 < 5   # the deadline, then ncclCommAbort's teardown (~0.5 s on the box)
    with pytest.raises(PekfError, match="aborted"):
        c.allreduce_max(f.X.ptr, 1, s.handle)       # the aborted communicator refuses further work
    s.sync()
    del bufs
    c.close()                                        # an aborted communicator only frees


def test_collectives_past_the_tracking_limit_are_refused_not_untracked(eng):
    """libpekf tracks at most 1,024 incomplete collectives per communicator (pekf_comm_wait's per-collective
    clock needs each one's events).  Behind ~0.3 s of compute, 1,100 all-reduces are enqueued: the 1,025th
    is refused with PEKF_ERR_COMM and never enqueued (an evicted, untracked collective that a
    peer never joined would have stalled the stream with no deadline running); the 1,024 tracked ones
    drain under the deadline, and afterwards the communicator takes collectives again."""
    from poseestimationkf_amd import shard
    from poseestimationkf_amd._lib import PekfError
    c = shard.Communicator(shard.Communicator.unique_id(), 1, 0)
    B = 1 << 18
    win = eng.IMUWindow(B, 64).synthesize(seed=synth.DEFAULT_SEED)
    f = eng.BatchedEKF(B)
    s = eng.Stream()
    buf = eng.DeviceBuffer(8)
    buf.upload(np.array([1.5]))
    f.run_async(win, 100000, 0, s.handle)
    done = 0
    with pytest.raises(PekfError, match="collectives already in flight"):
        for _ in range(1100):
            c.allreduce_max(buf.ptr, 1, s.handle)
            done += 1
    assert done == 1024
    c.wait(s.handle, timeout=30)
    c.allreduce_max(buf.ptr, 1, s.handle)
    c.wait(s.handle, timeout=30)
    assert buf.download((1,), np.float64)[0] == 1.5
    c.close()


def test_multi_device_ekf_sync_has_the_deadline(eng):
    """The one-process N-GPU path (MultiDeviceEKF, what plain `bench.py --gpus N` runs) drains through
    pekf_comm_wait: compute + a grouped gather pass a 5 ms deadline; a grouped-gather communicator with a
    collective in flight past it makes sync() abort every communicator and raise CommTimeoutError."""
    from poseestimationkf_amd import shard
    from poseestimationkf_amd._lib import CommTimeoutError
    B, W = 1 << 18, 64
    m = shard.MultiDeviceEKF([0], B, W).synthesize(seed=synth.DEFAULT_SEED)
    m.run_async(20000, 0)
    m.gather_async()
    m.sync(timeout=0.005)
    got = m.gathered()
    assert np.allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-12)
    bufs = _busy_gather(eng, m.comms[0], m.streams[0].handle)
    with pytest.raises(CommTimeoutError, match="did not complete within"):
        m.sync(timeout=0.0005)
    assert all(c.handle is None for c in m.comms)     # every communicator aborted
    m.streams[0].sync()
    del bufs
    m.close()


def test_after_an_init_timeout_later_inits_fail_fast():
    """An init that passed its deadline leaves its helper thread blocked inside RCCL, so the process must
    exit (include/pekf.h): until it does, pekf_comm_init / pekf_comm_init_all refuse at once instead of
    touching RCCL's bootstrap state.  Run in a child process, which then leaves with os._exit."""
    import os
    import subprocess
    import sys

    from .conftest import ROOT
    code = "\n".join([
        "import os, sys, time",
        "sys.path.insert(0, %r)" % ROOT,
        "from poseestimationkf_amd import engine, shard",
        "from poseestimationkf_amd._lib import CommTimeoutError, PekfError",
        "engine.set_device(0)",
        "t0 = time.monotonic()",
        "try:",
        "    shard.Communicator(shard.Communicator.unique_id(), 2, 0)",   # rank 1 never comes
        "except CommTimeoutError as e:",
        "    print('TIMEOUT %.1f' % (time.monotonic() - t0), flush=True)",
        "for make in (lambda: shard.Communicator.init_all([0]),",
        "             lambda: shard.Communicator(shard.Communicator.unique_id(), 1, 0)):",
        "    t1 = time.monotonic()",
        "    try:",
        "        make()",
        "        print('CREATED', flush=True)",
        "    except PekfError as e:",
        "        print('REFUSED %.2f %s' % (time.monotonic() - t1, 'must exit' in str(e)), flush=True)",
        "os._exit(0)",
    ])
    env = dict(os.environ, PEKF_COMM_TIMEOUT_S="3")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=100, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.split()[0] in ("TIMEOUT", "REFUSED", "CREATED")]
    assert lines[0].startswith("TIMEOUT") and 3.0 <= float(lines[0].split()[1]) < 20, out.stdout
    assert len(lines) == 3 and all(l.startswith("REFUSED") and l.endswith("True") for l in lines[1:]), out.stdout
    assert all(float(l.split()[1]) < 1.0 for l in lines[1:])
