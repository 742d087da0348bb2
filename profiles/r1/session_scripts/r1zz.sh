#!/usr/bin/env bash
# S^-1 pinned in front of the Wahba fallback branch (interleaves with the Wahba chain; +8 VALU) vs current, C2 and C3
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zz \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zz/cur_c2_1.json" \
 "PEKF_LIB=ab/pin.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zz/pin_c2_1.json" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B > gpurun_out/r1zz/cur_c3_1.json" \
 "PEKF_LIB=ab/pin.so timeout -k 10 300 $B > gpurun_out/r1zz/pin_c3_1.json" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zz/cur_c2_2.json" \
 "PEKF_LIB=ab/pin.so timeout -k 10 300 $B --batch 65536 > gpurun_out/r1zz/pin_c2_2.json" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B > gpurun_out/r1zz/cur_c3_2.json" \
 "PEKF_LIB=ab/pin.so timeout -k 10 300 $B > gpurun_out/r1zz/pin_c3_2.json"
