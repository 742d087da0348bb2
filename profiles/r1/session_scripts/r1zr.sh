#!/usr/bin/env bash
# reference-frame basis build, final form: parity suite and the headline bench
exec scripts/gpu_session.sh r1zr \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "timeout -k 10 300 python bench.py --cpu-baseline none > gpurun_out/r1zr/bench_c3_f64.json"
