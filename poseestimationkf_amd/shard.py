"""Data-parallel sharding of the independent-filter batch over GPUs.

Filters are independent (no state shared between KalmanFilter instances,
ExtendedKalmanFilter.py:6-80) and the time axis is a strict recurrence, so the only
parallel axis is the batch: rank r owns the contiguous filter range
[r*B_local, (r+1)*B_local) and runs it with no communication at all.  The single
collective is ONE gather of the final quaternions to the root, an RCCL gather over xGMI
issued through libpekf's C ABI (pekf_gather_dev, include/pekf.h) -- no PyTorch on the data
path.  Two ways to drive it:

* one process per GPU (torchrun): `Communicator(exchange_unique_id(rank, world), world, rank)`;
  the 128-byte RCCL id travels over any CPU channel -- here torch.distributed's gloo group,
  which is used for the rendezvous only;
* one process for several GPUs: `MultiDeviceEKF(devices, ...)` (ncclCommInitAll, one host
  thread, the gather as one RCCL group).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib

COMM_ID_BYTES = 128


def shard_range(global_batch, rank, world):
    """(first_filter, count) of rank's contiguous shard; shards are equal-sized."""
    if global_batch % world:
        raise ValueError("global batch %d must divide evenly over %d ranks" % (global_batch, world))
    per = global_batch // world
    return rank * per, per


def rccl_version():
    v = ctypes.c_int()
    check(lib.pekf_comm_version(ctypes.byref(v)))
    return v.value


class Communicator:
    """One rank of an RCCL communicator on the current device, owned through libpekf."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, _handle=None):
        if _handle is not None:  # from init_all
            self.handle = _handle
        else:
            if len(unique_id) != COMM_ID_BYTES:
                raise ValueError("an RCCL unique id is %d bytes" % COMM_ID_BYTES)
            h = ctypes.c_void_p()
            check(lib.pekf_comm_init(bytes(unique_id), int(nranks), int(rank), ctypes.byref(h)))
            self.handle = h.value
        r, n, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.pekf_comm_rank(self.handle, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d)))
        self.rank, self.nranks, self.device = r.value, n.value, d.value

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        check(lib.pekf_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def init_all(cls, devices):
        """One communicator per device of this process (ncclCommInitAll), rank i on devices[i]."""
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        hs = (ctypes.c_void_p * len(devices))()
        check(lib.pekf_comm_init_all(len(devices), devs, hs))
        return [cls(b"", 0, 0, _handle=hs[i]) for i in range(len(devices))]

    def gather(self, send_ptr, count, recv_ptr=None, root=0, stream=None):
        """recv[nranks*count] on root <- every rank's send[count] float64 (device pointers, enqueued)."""
        check(lib.pekf_gather_dev(self.handle, send_ptr, int(count), recv_ptr, int(root), stream))

    def allreduce_max(self, buf_ptr, count, stream=None):
        check(lib.pekf_allreduce_max_dev(self.handle, buf_ptr, int(count), stream))

    def close(self):
        if getattr(self, "handle", None):
            h, self.handle = self.handle, None
            check(lib.pekf_comm_destroy(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def exchange_unique_id(rank, world, make_id=Communicator.unique_id):
    """Rank 0's RCCL id on every rank, over torch.distributed's (CPU, gloo) default group.

    This is rendezvous plumbing only: 128 bytes once per job; the collective itself is RCCL."""
    import torch.distributed as dist

    obj = [make_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(obj, src=0)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != COMM_ID_BYTES:
        raise RuntimeError("bad RCCL unique id from rank 0")
    return bytes(uid)


def gather_quaternions(comm: Communicator, x_dev_ptr, batch_local, recv=None, root=0, stream=None):
    """Gather every rank's final X (batch_local, 4) float64 (device pointer) to root.

    recv: on root, a DeviceBuffer of nranks * batch_local * 32 bytes (rows in filter order);
    returns it (None elsewhere).  One pekf_gather_dev call = one RCCL collective."""
    from .engine import DeviceBuffer

    if comm.rank == root and recv is None:
        recv = DeviceBuffer(32 * batch_local * comm.nranks)
    comm.gather(x_dev_ptr, 4 * batch_local, recv.ptr if comm.rank == root else None, root, stream)
    return recv if comm.rank == root else None


class MultiDeviceEKF:
    """A batch of filters split over several GPUs of ONE process (SURVEY.md §8e's single-process
    form): device i holds filters [i*B_local, (i+1)*B_local) as its own IMUWindow + BatchedEKF,
    the launches run concurrently on per-device streams, and the final quaternions come back to
    the root device with one grouped RCCL gather (pekf_gather_multi_dev)."""

    def __init__(self, devices, batch_per_device, window, q=1.0, r=0.1, precision="f64"):
        from . import engine

        self.devices = [int(d) for d in devices]
        self.batch = int(batch_per_device)
        self.window = int(window)
        self.wins, self.filts, self.streams = [], [], []
        for d in self.devices:
            engine.set_device(d)
            self.streams.append(engine.Stream())
            self.wins.append(engine.IMUWindow(self.batch, self.window))
            self.filts.append(engine.BatchedEKF(self.batch, q=q, r=r, precision=precision))
        engine.set_device(self.devices[0])
        self.comms = Communicator.init_all(self.devices)
        self._recv = None

    def synthesize(self, seed, missing=False):
        from . import engine

        for i, d in enumerate(self.devices):
            engine.set_device(d)
            self.wins[i].synthesize(seed=seed, first_filter=i * self.batch, missing=missing,
                                    stream=self.streams[i].handle)
        self.sync()
        return self

    def run_async(self, n_steps, step0=0):
        from . import engine

        for i, d in enumerate(self.devices):
            engine.set_device(d)
            self.filts[i].run_async(self.wins[i], n_steps, step0, self.streams[i].handle)
        engine.set_device(self.devices[0])

    def gather_async(self, root=0):
        """Enqueue the gather of every device's X into a (n_dev * B_local, 4) buffer on the root."""
        from . import engine

        n = len(self.devices)
        if self._recv is None:
            engine.set_device(self.devices[root])
            self._recv = engine.DeviceBuffer(32 * self.batch * n)
        send = (ctypes.c_void_p * n)(*[f.X.ptr for f in self.filts])
        comms = (ctypes.c_void_p * n)(*[c.handle for c in self.comms])
        streams = (ctypes.c_void_p * n)(*[s.handle for s in self.streams])
        check(lib.pekf_gather_multi_dev(n, comms, send, 4 * self.batch, self._recv.ptr, int(root), streams))
        engine.set_device(self.devices[0])
        return self._recv

    def sync(self):
        from . import engine

        for i, d in enumerate(self.devices):
            engine.set_device(d)
            self.streams[i].sync()
        engine.set_device(self.devices[0])

    def gathered(self, root=0):
        """Host copy of the last gather: (n_dev * B_local, 4) float64, rows in filter order."""
        from . import engine

        engine.set_device(self.devices[root])
        out = self._recv.download((len(self.devices) * self.batch, 4), np.float64)
        engine.set_device(self.devices[0])
        return out

    def close(self):
        for c in self.comms:
            c.close()
        self.comms = []
