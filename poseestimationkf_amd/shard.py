"""Data-parallel sharding of the independent-filter batch over GPUs.

Filters are independent (no state shared between KalmanFilter instances,
ExtendedKalmanFilter.py:6-80) and the time axis is a strict recurrence, so the only
parallel axis is the batch: rank r owns the contiguous filter range
[r*B_local, (r+1)*B_local) and runs it with no communication at all.  The single
collective is ONE gather of the final quaternions to the root, an RCCL gather over xGMI
issued through libpekf's C ABI (pekf_gather_dev, include/pekf.h) -- no PyTorch on the data
path.  Two ways to drive it:

* one process per GPU (torchrun or any launcher that sets RANK / WORLD_SIZE):
  `Communicator(FileRendezvous(rank, world).share_id(Communicator.unique_id), world, rank)`;
  the 128-byte RCCL id travels through a file on the node (no PyTorch in the process), and
  once the communicator exists its barrier and max all-reduce are RCCL too;
* one process for several GPUs: `MultiDeviceEKF(devices, ...)` (ncclCommInitAll, one host
  thread, the gather as one RCCL group) -- no out-of-band exchange at all.
"""
from __future__ import annotations

import ctypes
import os
import tempfile
import time

import numpy as np

from ._lib import check, lib

COMM_ID_BYTES = 128
_RDZV_MAGIC = b"PEKFRDZV1"
_RDZV_FAIL = b"PEKFRDZVX"   # rank 0 failed before it could publish an id; the message follows


class RendezvousError(RuntimeError):
    """Rank 0 published a failure instead of the RCCL id (FileRendezvous.fail)."""


def comm_timeout():
    """Deadline in seconds of each collective step (PEKF_COMM_TIMEOUT_S, default 300; <= 0: none) --
    the same value libpekf applies to communicator creation (include/pekf.h)."""
    try:
        return float(os.environ.get("PEKF_COMM_TIMEOUT_S", "300"))
    except ValueError:
        return 300.0


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
        self._lib = lib   # the library that owns the handle (closes it, even if `lib` is rebound later)
        if _handle is not None:  # from init_all
            self.handle = _handle
        else:
            if len(unique_id) != COMM_ID_BYTES:
                raise ValueError("an RCCL unique id is %d bytes" % COMM_ID_BYTES)
            h = ctypes.c_void_p()   # non-blocking RCCL init polled against PEKF_COMM_TIMEOUT_S (pekf.h)
            check(lib.pekf_comm_init(bytes(unique_id), int(nranks), int(rank), ctypes.byref(h)))
            self.handle = h.value
        r, n, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._lib.pekf_comm_rank(self.handle, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d)))
        self.rank, self.nranks, self.device = r.value, n.value, d.value

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        check(lib.pekf_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def init_all(cls, devices, timeout=None):
        """One communicator per device of this process (ncclCommInitAll), rank i on devices[i], created
        within `timeout` seconds (default comm_timeout()) or CommTimeoutError (then exit the process)."""
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        hs = (ctypes.c_void_p * len(devices))()
        check(lib.pekf_comm_init_all_timeout(len(devices), devs, comm_timeout() if timeout is None else float(timeout),
                                             hs))
        return [cls(b"", 0, 0, _handle=hs[i]) for i in range(len(devices))]

    def gather(self, send_ptr, count, recv_ptr=None, root=0, stream=None):
        """recv[nranks*count] on root <- every rank's send[count] float64 (device pointers, enqueued)."""
        check(self._lib.pekf_gather_dev(self.handle, send_ptr, int(count), recv_ptr, int(root), stream))

    def allreduce_max(self, buf_ptr, count, stream=None):
        check(self._lib.pekf_allreduce_max_dev(self.handle, buf_ptr, int(count), stream))

    def wait(self, stream=None, timeout=None):
        """Drain `stream`, collectives of this communicator included.  Each of its collectives gets the
        deadline (default comm_timeout()) from the moment the stream reaches it, so queued compute is never
        charged; one a peer never joins raises CommTimeoutError and aborts the communicator.  The clock starts
        when this rank's inputs are ready, so the peers' skew (their remaining compute) counts against it:
        the timeout must exceed that skew.  More than 1,024 collectives in flight are refused (pekf.h)."""
        check(self._lib.pekf_comm_wait(self.handle, stream, comm_timeout() if timeout is None else float(timeout)))

    def max_over_ranks_array(self, values, stream=None):
        """Elementwise max of a host float64 vector over all ranks (one RCCL all-reduce, a deadline-bound
        wait).  With every rank writing only its own slots (the rest -inf), it is an all-gather of them."""
        from .engine import DeviceBuffer

        v = np.ascontiguousarray(values, np.float64).ravel()
        b = DeviceBuffer(v.nbytes).upload(v, stream)
        self.allreduce_max(b.ptr, v.size, stream)
        self.wait(stream)
        return b.download(v.shape, np.float64, stream)

    def max_over_ranks(self, value, stream=None):
        """max of a host float over all ranks (one RCCL all-reduce of 8 bytes, then a deadline-bound wait)."""
        return float(self.max_over_ranks_array([value], stream)[0])

    def all_values(self, values, stream=None):
        """Every rank's `values` (same length on each), as an (nranks, len) array on every rank."""
        v = np.ascontiguousarray(values, np.float64).ravel()
        slots = np.full((self.nranks, v.size), -np.inf)
        slots[self.rank] = v
        return self.max_over_ranks_array(slots, stream).reshape(self.nranks, v.size)

    def barrier(self, stream=None):
        """Every rank has reached this point (and its stream has drained up to it)."""
        self.max_over_ranks(0.0, stream)

    def close(self):
        if getattr(self, "handle", None):
            h, self.handle = self.handle, None
            check(self._lib.pekf_comm_destroy(h))

    def abort(self):
        """ncclCommAbort (error paths: the peers' collectives with this rank give up)."""
        if getattr(self, "handle", None):
            h, self.handle = self.handle, None
            check(self._lib.pekf_comm_abort(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _proc_start_ticks(pid):
    """Start time of a process in clock ticks since boot (/proc/<pid>/stat field 22), or 0."""
    try:
        with open("/proc/%d/stat" % pid, "rb") as fh:
            return int(fh.read().rsplit(b")", 1)[1].split()[19])
    except (OSError, IndexError, ValueError):
        return 0


def _launch_tag(env):
    """What tells one launch of a job from a relaunch of it with the same key: torchrun's run id (when it
    is not its "none" default), its restart count (elastic restarts reuse the agent, the ranks' parent)
    and the master address / port -- those of them the launcher set, all equal on every rank of a launch."""
    parts = []
    run_id = env.get("TORCHELASTIC_RUN_ID")
    if run_id and run_id != "none":
        parts.append(run_id)
    for k in ("TORCHELASTIC_RESTART_COUNT", "MASTER_ADDR", "MASTER_PORT"):
        if env.get(k):
            parts.append(env[k])
    return "_".join(parts)


class FileRendezvous:
    """Torch-free out-of-band channel for rank 0's 128-byte RCCL id, through a file on the node.

    A launcher such as torchrun starts every local rank as a child of one process, so the job's
    key is (MASTER_ADDR, MASTER_PORT, the parent's pid and start time, the restart count): unique among
    the launches that ever ran on the node, so a file left behind by another one is never read.  Rank 0
    writes the id atomically (temp file + rename); the others poll for it.  `key` / PEKF_RDZV_KEY
    override the key for launchers whose ranks do not share a parent; the launch tag (torchrun's run id
    and restart count, MASTER_ADDR / MASTER_PORT, whichever are set) is appended to such a key too, so a
    relaunch with the same key but a new port or run id never reads the previous launch's file.
    PEKF_RDZV_DIR names the directory (it must be shared by every rank, e.g. a network file system when
    ranks span nodes).  A job that spans nodes must name its key: the default (the local parent)
    differs between nodes, so it is refused there.
    If rank 0 fails before it has an id, `fail(msg)` publishes the failure and the other ranks raise
    at once instead of waiting out `timeout` (PEKF_RDZV_TIMEOUT_S, default 300 s, as PEKF_COMM_TIMEOUT_S).
    Rank 0 removes whatever an earlier launch left under its path when it is constructed (a failure
    marker, an id whose job died), and `done()` removes its own file once the communicator exists (or
    its creation failed): RCCL's communicator creation is collective, so every rank has read it by then."""

    def __init__(self, rank, world, key=None, directory=None, timeout=None, environ=None):
        env = os.environ if environ is None else environ
        if timeout is None:
            timeout = float(env.get("PEKF_RDZV_TIMEOUT_S", "300"))
        self.rank, self.world, self.timeout = int(rank), int(world), float(timeout)
        if not 0 <= self.rank < self.world:
            raise ValueError("need 0 <= rank < world")
        if key is None:
            key = env.get("PEKF_RDZV_KEY")
        if key is None and self.world > 1 and _spans_nodes(env):
            raise ValueError("FileRendezvous: this job spans nodes (GROUP_WORLD_SIZE / LOCAL_WORLD_SIZE), so its ranks "
                             "have no common parent; set PEKF_RDZV_KEY to one job-wide value and PEKF_RDZV_DIR to a "
                             "directory every node shares")
        if key is None:
            ppid = os.getppid()
            key = "%s_%s_%d_%d" % (env.get("MASTER_ADDR", "local"), env.get("MASTER_PORT", "0"),
                                   ppid, _proc_start_ticks(ppid))
            if env.get("TORCHELASTIC_RESTART_COUNT"):
                key += "_r" + env["TORCHELASTIC_RESTART_COUNT"]
        else:
            tag = _launch_tag(env)
            key = "%s_%s" % (key, tag) if tag else str(key)
        key = "".join(c if c.isalnum() or c in "-_." else "_" for c in str(key))
        directory = directory or env.get("PEKF_RDZV_DIR") or tempfile.gettempdir()
        self.path = os.path.join(directory, "pekf-rdzv-%s.id" % key)
        if self.rank == 0 and self.world > 1:
            self.done()   # a stale file of an earlier launch under this key

    def share_id(self, make_id=None):
        """Rank 0 creates the id (make_id(), default a new RCCL id) and publishes it; every rank returns it."""
        if make_id is None:
            make_id = Communicator.unique_id
        if self.rank == 0:
            uid = bytes(make_id())
            if len(uid) != COMM_ID_BYTES:
                raise RuntimeError("an RCCL unique id is %d bytes" % COMM_ID_BYTES)
            if self.world > 1:
                tmp = "%s.%d.tmp" % (self.path, os.getpid())
                with open(tmp, "wb") as fh:
                    fh.write(_RDZV_MAGIC + uid)
                os.replace(tmp, self.path)
            return uid
        deadline = time.monotonic() + self.timeout
        while True:
            try:
                with open(self.path, "rb") as fh:
                    blob = fh.read()
                if blob.startswith(_RDZV_MAGIC) and len(blob) == len(_RDZV_MAGIC) + COMM_ID_BYTES:
                    return blob[len(_RDZV_MAGIC):]
                if blob.startswith(_RDZV_FAIL):
                    raise RendezvousError("rank %d: rank 0 failed before publishing the RCCL id: %s"
                                       % (self.rank, blob[len(_RDZV_FAIL):].decode(errors="replace")))
            except FileNotFoundError:
                pass
            if time.monotonic() > deadline:
                raise TimeoutError("rank %d: no RCCL id from rank 0 at %s after %.0f s"
                                   % (self.rank, self.path, self.timeout))
            time.sleep(0.01)

    def fail(self, message):
        """Rank 0 could not create the id (it is exiting): publish that, so the others stop waiting."""
        if self.rank == 0 and self.world > 1:
            tmp = "%s.%d.tmp" % (self.path, os.getpid())
            with open(tmp, "wb") as fh:
                fh.write(_RDZV_FAIL + str(message).encode()[:4000])
            os.replace(tmp, self.path)

    def done(self):
        """Rank 0 removes the published id (call after the communicator exists on rank 0)."""
        if self.rank == 0:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


def _spans_nodes(env):
    """True when the launcher says the job has ranks on more than one node (torchrun's variables)."""
    try:
        if int(env.get("GROUP_WORLD_SIZE", "1")) > 1:
            return True
        lws = env.get("LOCAL_WORLD_SIZE")
        return lws is not None and "WORLD_SIZE" in env and int(env["WORLD_SIZE"]) != int(lws)
    except ValueError:
        return False


def connect(rank, world, rendezvous=None):
    """The RCCL communicator of this process's rank on the current device: rank 0's id shared through
    `rendezvous` (default FileRendezvous(rank, world)), then ncclCommInitRank (collective)."""
    rdzv = rendezvous or FileRendezvous(rank, world)
    uid = rdzv.share_id()
    try:
        comm = Communicator(uid, world, rank)
    except BaseException as e:
        # rank 0's creation failed or timed out: ranks that have not read the id yet stop at once
        # (the failure marker replaces the id) instead of waiting out PEKF_RDZV_TIMEOUT_S
        rdzv.fail("rank 0's RCCL communicator creation failed: %s" % e)
        raise
    rdzv.done()   # rank 0: created, the id is spent (a relaunch must not read it)
    return comm


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
    the root device with one grouped RCCL gather (pekf_gather_multi_dev).

    It fails instead of hanging, like the one-process-per-GPU path: the communicators are created
    under the PEKF_COMM_TIMEOUT_S deadline, and sync() drains every device's stream through
    pekf_comm_wait, so a grouped gather that does not complete within the deadline of its inputs
    being ready (or an asynchronous RCCL error) aborts every communicator and raises."""

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

    def sync(self, timeout=None):
        """Drain every device's stream; each collective gets `timeout` (default comm_timeout()) from the
        moment its device's stream reaches it.  On expiry or an RCCL error every communicator is aborted
        (the grouped gather's other members would wait for the failed one forever) and the error raised."""
        from . import engine

        try:
            for i, d in enumerate(self.devices):
                engine.set_device(d)
                self.comms[i].wait(self.streams[i].handle, timeout)
        except Exception:
            self.abort()
            raise
        finally:
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

    def abort(self):
        """ncclCommAbort on every device's communicator (error paths)."""
        for c in self.comms:
            try:
                c.abort()
            except Exception:
                pass
