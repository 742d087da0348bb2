#!/usr/bin/env bash
exec scripts/gpu_session.sh r1x \
 "timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r1x/auxtrace -o aux --output-format csv -- python3 scripts/bench_aux.py"
