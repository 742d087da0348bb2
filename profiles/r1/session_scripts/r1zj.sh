#!/usr/bin/env bash
# row offset advanced by an add (no 64-bit multiply per step), 32-bit step counter: C2 / C3 against the 360-VALU build
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zj \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zj/v360_c2_1.json" \
 "PEKF_LIB=ab/off8.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zj/off8_c2_1.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zj/v360_c3_1.json" \
 "PEKF_LIB=ab/off8.so timeout -k 10 300 $B > gpurun_out/r1zj/off8_c3_1.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zj/v360_c2_2.json" \
 "PEKF_LIB=ab/off8.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zj/off8_c2_2.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zj/v360_c3_2.json" \
 "PEKF_LIB=ab/off8.so timeout -k 10 300 $B > gpurun_out/r1zj/off8_c3_2.json"
