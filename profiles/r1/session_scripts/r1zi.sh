#!/usr/bin/env bash
# 3-deep record ring (two rows in flight) against the 2-deep ping-pong of the 360-VALU build, C2 and C3
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zi \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zi/v360_c2_1.json" \
 "PEKF_LIB=ab/ring3.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zi/ring3_c2_1.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zi/v360_c3_1.json" \
 "PEKF_LIB=ab/ring3.so timeout -k 10 300 $B > gpurun_out/r1zi/ring3_c3_1.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zi/v360_c2_2.json" \
 "PEKF_LIB=ab/ring3.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zi/ring3_c2_2.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zi/v360_c3_2.json" \
 "PEKF_LIB=ab/ring3.so timeout -k 10 300 $B > gpurun_out/r1zi/ring3_c3_2.json"
