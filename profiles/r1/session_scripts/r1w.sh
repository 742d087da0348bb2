#!/usr/bin/env bash
exec scripts/gpu_session.sh r1w \
 "timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider -x" \
 "timeout -k 10 400 python3 scripts/bench_aux.py > gpurun_out/r1w/aux.json" \
 "timeout -k 10 400 python3 bench.py --cpu-baseline none > gpurun_out/r1w/bench.json"
