#!/usr/bin/env bash
# no near-identity test in the reference-frame path (333 VALU per record): parity, A/B against HEAD
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zw \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/head.so timeout -k 10 300 $B > gpurun_out/r1zw/head_1.json" \
 "PEKF_LIB=ab/noid.so timeout -k 10 300 $B > gpurun_out/r1zw/noid_1.json" \
 "PEKF_LIB=ab/head.so timeout -k 10 300 $B > gpurun_out/r1zw/head_2.json" \
 "PEKF_LIB=ab/noid.so timeout -k 10 300 $B > gpurun_out/r1zw/noid_2.json"
