#!/usr/bin/env bash
exec scripts/gpu_session.sh r1n \
 "timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider" \
 "timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r1n/trace -o aux --output-format csv -- python3 scripts/bench_aux.py"
