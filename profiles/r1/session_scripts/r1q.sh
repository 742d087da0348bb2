#!/usr/bin/env bash
exec scripts/gpu_session.sh r1q \
 "timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider -x" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none > gpurun_out/r1q/bench.json" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none --precision mixed > gpurun_out/r1q/bench_mixed.json"
