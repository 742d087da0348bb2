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


def test_comm_wait_deadline_aborts(eng):
    """pekf_comm_wait drains a stream against a deadline: on a stream still busy when it passes (here a
    long fused launch standing in for a collective a dead peer never completes) it aborts the
    communicator and raises CommTimeoutError; a drained stream returns at once."""
    import time

    from poseestimationkf_amd import shard
    from poseestimationkf_amd._lib import CommTimeoutError, PekfError
    c = shard.Communicator(shard.Communicator.unique_id(), 1, 0)
    B = 1 << 18
    win = eng.IMUWindow(B, 64).synthesize(seed=synth.DEFAULT_SEED)
    f = eng.BatchedEKF(B)
    s = eng.Stream()
    c.wait(s.handle, timeout=5)                      # idle stream: returns
    f.run_async(win, 20000, 0, s.handle)             # ~60 ms of work
    t0 = time.monotonic()
    with pytest.raises(CommTimeoutError, match="did not complete within"):
        c.wait(s.handle, timeout=0.005)
    assert time.monotonic() - t0 < 5   # the deadline, then ncclCommAbort's teardown (~0.5 s on the box)
    with pytest.raises(PekfError, match="aborted"):
        c.allreduce_max(f.X.ptr, 1, s.handle)       # the aborted communicator refuses further work
    s.sync()
    c.close()                                        # an aborted communicator only frees
