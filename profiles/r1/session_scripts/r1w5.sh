#!/usr/bin/env bash
# 5 waves per SIMD forced on k_run (96 VGPRs + scratch reloads of loop constants) vs 4 (114 VGPRs)
B="python bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1w5
exec scripts/gpu_session.sh r1w5 \
 "PEKF_LIB=ab/w5.so timeout -k 10 300 $B > $O/w5_c3_1.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B > $O/lz_c3_1.json" \
 "PEKF_LIB=ab/w5.so timeout -k 10 300 $B > $O/w5_c3_2.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B > $O/lz_c3_2.json" \
 "PEKF_LIB=ab/w5.so timeout -k 10 300 $B --batch 65536 > $O/w5_c2_1.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B --batch 65536 > $O/lz_c2_1.json"
