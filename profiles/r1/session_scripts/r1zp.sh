#!/usr/bin/env bash
# multi-record launches in the reference frame's basis (RefW): parity suite, A/B against the 354-VALU build
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zp \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/v354.so timeout -k 10 300 $B > gpurun_out/r1zp/v354_1.json" \
 "PEKF_LIB=ab/wbasis.so timeout -k 10 300 $B > gpurun_out/r1zp/wbasis_1.json" \
 "PEKF_LIB=ab/v354.so timeout -k 10 300 $B > gpurun_out/r1zp/v354_2.json" \
 "PEKF_LIB=ab/wbasis.so timeout -k 10 300 $B > gpurun_out/r1zp/wbasis_2.json"
