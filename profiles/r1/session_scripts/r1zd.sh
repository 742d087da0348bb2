#!/usr/bin/env bash
# same-box A/B of the fused kernel: 3276dda (402 VALU/step) vs the current build (360)
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zd \
 "PEKF_LIB=ab/base.so timeout -k 10 300 $B > gpurun_out/r1zd/base1.json" \
 "PEKF_LIB=ab/new.so timeout -k 10 300 $B > gpurun_out/r1zd/new1.json" \
 "PEKF_LIB=ab/base.so timeout -k 10 300 $B > gpurun_out/r1zd/base2.json" \
 "PEKF_LIB=ab/new.so timeout -k 10 300 $B > gpurun_out/r1zd/new2.json" \
 "PEKF_LIB=ab/base.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zd/base_c2.json" \
 "PEKF_LIB=ab/new.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zd/new_c2.json"
