#!/usr/bin/env bash
# u-vector covariance propagation + Q4 z quaternion extraction: parity suite, then the headline bench
exec scripts/gpu_session.sh r1zc \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "timeout -k 10 400 python bench.py --cpu-baseline none > gpurun_out/r1zc/bench_f64.json" \
 "timeout -k 10 400 python bench.py --missing --cpu-baseline none > gpurun_out/r1zc/bench_c5.json"
