"""Helper of tests/test_shard_gloo.py::test_file_rendezvous_under_torchrun: one rank of a torchrun job
shares rank 0's id through shard.FileRendezvous (what bench.py does) and reports on stdout."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from poseestimationkf_amd import shard  # noqa: E402

r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
z = shard.FileRendezvous(r, w, timeout=60)
uid = z.share_id(make_id=lambda: bytes([7]) * 128)
# one write of the whole line (the ranks share the launcher's stdout)
os.write(1, b"RDZV rank=%d ok=%d torch=%d\n" % (r, uid == bytes([7]) * 128, "torch" in sys.modules))
