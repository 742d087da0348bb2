#!/usr/bin/env bash
exec scripts/gpu_session.sh r1k \
 "timeout -k 10 500 python -m pytest tests -m gpu -q -s -p no:cacheprovider" \
 "timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r1k/trace -o aux --output-format csv -- python3 scripts/bench_aux.py"
