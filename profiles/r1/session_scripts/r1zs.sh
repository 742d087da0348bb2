#!/usr/bin/env bash
# record loads with the non-temporal cache policy (aux 2 = nt, aux 3 = sc0 nt) against the default policy
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zs \
 "PEKF_LIB=ab/wb.so timeout -k 10 300 $B > gpurun_out/r1zs/def_1.json" \
 "PEKF_LIB=ab/aux2.so timeout -k 10 300 $B > gpurun_out/r1zs/nt_1.json" \
 "PEKF_LIB=ab/aux3.so timeout -k 10 300 $B > gpurun_out/r1zs/sc0nt_1.json" \
 "PEKF_LIB=ab/wb.so timeout -k 10 300 $B > gpurun_out/r1zs/def_2.json" \
 "PEKF_LIB=ab/aux2.so timeout -k 10 300 $B > gpurun_out/r1zs/nt_2.json" \
 "PEKF_LIB=ab/aux3.so timeout -k 10 300 $B > gpurun_out/r1zs/sc0nt_2.json"
