#!/usr/bin/env bash
# cost of the Q4 z fallback branch: the 360-VALU build against the same kernel with the branch compiled out
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zh2 \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zh2/v360_1.json" \
 "PEKF_LIB=ab/nofb.so timeout -k 10 300 $B > gpurun_out/r1zh2/nofb_1.json" \
 "PEKF_LIB=ab/v360.so timeout -k 10 300 $B > gpurun_out/r1zh2/v360_2.json" \
 "PEKF_LIB=ab/nofb.so timeout -k 10 300 $B > gpurun_out/r1zh2/nofb_2.json"
