"""A host fake of libpekf's device / collective entry points -- TEST INFRASTRUCTURE ONLY.

It lets bench.py's multi-GPU code paths (one process over N devices, and one process per rank) run
end to end on a CPU-only machine: every Python layer above the C ABI (bench.py, engine.py,
shard.py) runs unchanged, and only the ctypes library object is replaced.

* "device memory" is host memory (a device pointer is the address of a numpy buffer), streams run
  synchronously, events read the host clock;
* pekf_synth_dev uses the host mirror of the Philox generator (synth.generate, bit-identical to the
  device generator) and pekf_run_dev advances the state with the C oracle (oracle_c.run, the
  restatement of main_file.py:38-47), so parity against the oracle holds exactly;
* collectives: pekf_comm_init_all's communicators live in one process (the grouped gather copies);
  pekf_comm_init's go through torch.distributed's gloo backend between processes (gloo stands in for
  RCCL here, as in test_shard_gloo.py);
* failure injection, for the "fail, don't hang" contract: `stuck_devices` -- a grouped gather enqueued
  on one of these devices never completes, so pekf_comm_wait on it returns PEKF_ERR_TIMEOUT once its
  deadline has passed (as libpekf's does for a collective whose inputs are ready); `init_all_stalls`
  -- ncclCommInitAll never returns, so pekf_comm_init_all_timeout times out.

install(monkeypatch_or_none, n_devices) swaps it into _lib / engine / shard.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np

from oracle import oracle_c
from poseestimationkf_amd import synth


def _set(ref, value):
    """Write through a ctypes.byref(...) argument."""
    ref._obj.value = value


class FakeLib:
    def __init__(self, n_devices=1, gloo_port=None):
        self.n_devices = int(n_devices)
        self.device = 0
        self.mem = {}                # address -> numpy uint8 buffer (keeps it alive)
        self.events = {}
        self.next_handle = 1
        self.comms = {}
        self.gloo_port = gloo_port
        self.calls = []              # names of the entry points called, in order
        self.runs = []               # (device, batch, n_steps, step0) of every fused launch
        self.last_err = b"fake libpekf"
        self.stuck_devices = set()   # failure injection (module docstring)
        self.init_all_stalls = False

    def _handle(self):
        self.next_handle += 1
        return self.next_handle

    def _view(self, addr, nbytes, dtype=np.uint8):
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(addr)).view(dtype)

    def __getattr__(self, name):
        raise AttributeError("fake libpekf has no %s" % name)

    # ------------------------------------------------------------------ runtime
    def pekf_abi_version(self):
        return 1

    def pekf_last_error(self):
        return self.last_err

    def _fail(self, status, msg):
        self.last_err = msg.encode()
        return status

    def pekf_device_count(self, n):
        _set(n, self.n_devices)
        return 0

    def pekf_set_device(self, d):
        assert 0 <= d < self.n_devices, d
        self.device = d
        return 0

    def pekf_malloc(self, p, nbytes):
        buf = np.zeros(max(1, int(nbytes)), np.uint8)
        addr = buf.ctypes.data
        self.mem[addr] = buf
        _set(p, addr)
        return 0

    def pekf_free(self, p):
        self.mem.pop(p, None)
        return 0

    def pekf_memcpy_h2d(self, dst, src, n, stream):
        ctypes.memmove(dst, src, n)
        return 0

    pekf_memcpy_d2h = pekf_memcpy_h2d
    pekf_memcpy_d2d = pekf_memcpy_h2d

    def pekf_stream_create(self, s):
        _set(s, self._handle())
        return 0

    def pekf_stream_destroy(self, s):
        return 0

    def pekf_stream_sync(self, s):
        return 0

    def pekf_device_sync(self):
        return 0

    def pekf_event_create(self, e):
        h = self._handle()
        self.events[h] = None
        _set(e, h)
        return 0

    def pekf_event_destroy(self, e):
        self.events.pop(e, None)
        return 0

    def pekf_event_record(self, e, stream):
        self.events[e] = time.perf_counter()
        return 0

    def pekf_event_elapsed_ms(self, ms, e0, e1):
        _set(ms, (self.events[e1] - self.events[e0]) * 1e3)
        return 0

    # ------------------------------------------------------------------ the path
    def pekf_synth_dev(self, batch, window, first, seed, missing, scales, ar_w, gd, am, my, refs, stream):
        p = synth.SynthParams()
        assert [scales[i] for i in range(5)] == list(p.scales()) and ar_w == p.ar_w, "fake: default params only"
        rec = synth.generate(np.arange(first, first + batch), window, seed=seed, missing=bool(missing))
        g, a, m = synth.pack_planes(rec)
        for dst, src in ((gd, g), (am, a), (my, m)):
            ctypes.memmove(dst, np.ascontiguousarray(src).ctypes.data, src.nbytes)
        r = synth.refs_array(rec.acc0, rec.mag0)
        ctypes.memmove(refs, r.ctypes.data, r.nbytes)
        self.calls.append("pekf_synth_dev")
        return 0

    def pekf_reset_state_dev(self, batch, X, P, stream):
        self._view(X, 32 * batch, np.float64)[:] = np.tile([1.0, 0, 0, 0], batch)
        self._view(P, 128 * batch, np.float64)[:] = np.tile(np.eye(4).ravel(), batch)
        return 0

    def pekf_run_dev(self, batch, n_steps, window, step0, gd, am, my, refs, X, P, q, r, traj, counts, flags, stream):
        assert traj is None and counts is None and flags == 0, "fake: the bench's launch only"
        n = batch * window
        rf = self._view(refs, 48 * batch, np.float64).reshape(batch, 6)
        rec = synth.unpack_planes(self._view(gd, 16 * n, np.float32).reshape(window, batch, 4),
                                  self._view(am, 16 * n, np.float32).reshape(window, batch, 4),
                                  self._view(my, 8 * n, np.float32).reshape(window, batch, 2),
                                  rf[:, :3], rf[:, 3:])
        Xv = self._view(X, 32 * batch, np.float64).reshape(batch, 4)
        Pv = self._view(P, 128 * batch, np.float64).reshape(batch, 4, 4)
        Xn, Pn, _ = oracle_c.run(rec, n_steps=n_steps, step0=step0, q=q, r=r, X=Xv.copy(), P=Pv.copy())
        Xv[:] = Xn
        Pv[:] = Pn
        self.runs.append((self.device, batch, n_steps, step0))
        return 0

    # ------------------------------------------------------------------ collectives
    def pekf_comm_version(self, v):
        _set(v, 22700)
        return 0

    def pekf_comm_unique_id(self, buf):
        ctypes.memmove(buf, os.urandom(128), 128)
        return 0

    def pekf_comm_init(self, uid, nranks, rank, out):
        import torch.distributed as dist
        if nranks > 1:
            dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % self.gloo_port, rank=rank,
                                    world_size=nranks)
        h = self._handle()
        self.comms[h] = dict(rank=rank, nranks=nranks, device=self.device, gloo=nranks > 1)
        _set(out, h)
        self.calls.append("pekf_comm_init")
        return 0

    def pekf_comm_init_all_timeout(self, ndev, devs, timeout, out):
        self.calls.append("pekf_comm_init_all")
        if self.init_all_stalls:
            time.sleep(max(0.0, timeout))
            return self._fail(7, "fake: ncclCommInitAll not done within %.0f s; init abandoned" % timeout)
        for i in range(ndev):
            h = self._handle()
            self.comms[h] = dict(rank=i, nranks=ndev, device=devs[i], gloo=False, pending=False)
            out[i] = h
        return 0

    def pekf_comm_init_all(self, ndev, devs, out):
        return self.pekf_comm_init_all_timeout(ndev, devs, 300.0, out)

    def pekf_comm_rank(self, h, r, n, d):
        c = self.comms[h]
        _set(r, c["rank"])
        _set(n, c["nranks"])
        _set(d, c["device"])
        return 0

    def pekf_comm_destroy(self, h):
        c = self.comms.pop(h, None)
        if c is not None and c["gloo"]:
            import torch.distributed as dist
            dist.destroy_process_group()
        return 0

    pekf_comm_abort = pekf_comm_destroy

    def pekf_comm_wait(self, h, stream, timeout):
        c = self.comms.get(h)
        if c is None:
            return self._fail(1, "fake: null or aborted communicator")
        if c.get("pending") and c["device"] in self.stuck_devices:
            time.sleep(max(0.0, timeout))
            self.comms.pop(h)
            return self._fail(7, "fake: rank %d of %d: ncclGather (grouped) did not complete within %.0f s of its "
                                 "inputs being ready; communicator aborted" % (c["rank"], c["nranks"], timeout))
        return 0

    def pekf_gather_dev(self, h, send, count, recv, root, stream):
        import torch
        import torch.distributed as dist
        c = self.comms[h]
        x = torch.from_numpy(self._view(send, 8 * count, np.float64).copy())
        if not c["gloo"]:
            self._view(recv, 8 * count, np.float64)[:] = x.numpy()
            return 0
        bufs = [torch.empty_like(x) for _ in range(c["nranks"])] if c["rank"] == root else None
        dist.gather(x, gather_list=bufs, dst=root)
        if c["rank"] == root:
            self._view(recv, 8 * count * c["nranks"], np.float64)[:] = torch.cat(bufs).numpy()
        self.calls.append("pekf_gather_dev")
        return 0

    def pekf_allreduce_max_dev(self, h, buf, count, stream):
        import torch
        import torch.distributed as dist
        v = self._view(buf, 8 * count, np.float64)
        if self.comms[h]["gloo"]:
            t = torch.from_numpy(v.copy())
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            v[:] = t.numpy()
        return 0

    def pekf_gather_multi_dev(self, ndev, comms, send, count, recv, root, streams):
        out = self._view(recv, 8 * count * ndev, np.float64).reshape(ndev, count)
        for i in range(ndev):
            assert self.comms[comms[i]]["rank"] == i
            out[i] = self._view(send[i], 8 * count, np.float64)
            self.comms[comms[i]]["pending"] = True
        self.calls.append("pekf_gather_multi_dev")
        return 0


def install(monkeypatch, n_devices=1, gloo_port=None):
    """Replace the loaded libpekf in _lib, engine and shard by a FakeLib; returns it."""
    from poseestimationkf_amd import _lib, engine, shard
    fake = FakeLib(n_devices, gloo_port)
    for mod in (_lib, engine, shard):
        if monkeypatch is None:
            setattr(mod, "lib", fake)
        else:
            monkeypatch.setattr(mod, "lib", fake)
    return fake
