#!/usr/bin/env bash
# e = v sc - z as a three-address v_fma_f64 (inline asm; 13 fewer VALU per record): parity, A/B against HEAD
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zu \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/head.so timeout -k 10 300 $B > gpurun_out/r1zu/head_1.json" \
 "PEKF_LIB=ab/fmasub.so timeout -k 10 300 $B > gpurun_out/r1zu/fmasub_1.json" \
 "PEKF_LIB=ab/head.so timeout -k 10 300 $B > gpurun_out/r1zu/head_2.json" \
 "PEKF_LIB=ab/fmasub.so timeout -k 10 300 $B > gpurun_out/r1zu/fmasub_2.json"
