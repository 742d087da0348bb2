#!/usr/bin/env bash
exec scripts/gpu_session.sh r1j \
 "timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r1j/trace -o aux --output-format csv -- python3 scripts/bench_aux.py"
