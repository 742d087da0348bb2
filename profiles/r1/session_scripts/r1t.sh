#!/usr/bin/env bash
exec scripts/gpu_session.sh r1t \
 "timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider -x" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none > gpurun_out/r1t/bench.json" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none --precision mixed > gpurun_out/r1t/bench_mixed.json" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none --missing > gpurun_out/r1t/bench_c5.json" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none --batch 65536 > gpurun_out/r1t/bench_c2.json"
