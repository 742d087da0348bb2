"""N > 1 path on CPU: world_size-2 gloo ranks rendezvous exactly as bench.py does (rank 0's
128-byte RCCL id broadcast by shard.exchange_unique_id over the gloo group), each takes a
contiguous filter shard and runs it (the C oracle stands in for the device here -- test only),
and the shards' final quaternions, concatenated in rank order as pekf_gather_dev lays them out on
the root, equal a single-process run.  The RCCL gather itself needs GPUs: tests/test_gpu_parity.py
runs it through libpekf at world size 1 (and bench.py --dist on the box)."""
import os
import socket

import numpy as np
import pytest

from poseestimationkf_amd import shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, global_batch, window, q):
    import torch
    import torch.distributed as dist

    from oracle import oracle_c
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        uid = shard.exchange_unique_id(rank, world, make_id=lambda: bytes(range(128)))
        assert uid == bytes(range(128))  # every rank holds rank 0's id (a failure fails the exit code)
        first, count = shard.shard_range(global_batch, rank, world)
        rec = synth.generate(np.arange(first, first + count), window)
        X, _, _ = oracle_c.run(rec)
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
    with pytest.raises(ValueError):
        shard.shard_range(10, 0, 3)


def test_two_rank_gather_equals_single_process():
    import multiprocessing as mp

    from oracle import oracle_c
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, 16, 24, q)) for r in range(2)]
    for p in procs:
        p.start()
    uid, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X, _, _ = oracle_c.run(synth.generate(np.arange(16), 24))
    assert uid == bytes(range(128))
    assert got.shape == (16, 4)
    assert np.array_equal(got, X)
