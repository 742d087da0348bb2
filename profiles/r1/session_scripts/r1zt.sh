#!/usr/bin/env bash
# the torch.distributed/RCCL gather path at world size 1: stdout must carry only the JSON line
exec scripts/gpu_session.sh r1zt \
 "timeout -k 10 400 python bench.py --dist --cpu-baseline none --steps 2 > gpurun_out/r1zt/bench_dist1.json"
