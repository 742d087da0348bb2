#!/usr/bin/env bash
# |X|^2 snapped to 1 and carried as a constant after a launch's first record (354 VALU): parity, A/B against the committed 360 build
B="python bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1zm \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/off8.so timeout -k 10 300 $B > gpurun_out/r1zm/v360_1.json" \
 "PEKF_LIB=ab/n2snap.so timeout -k 10 300 $B > gpurun_out/r1zm/v354_1.json" \
 "PEKF_LIB=ab/off8.so timeout -k 10 300 $B > gpurun_out/r1zm/v360_2.json" \
 "PEKF_LIB=ab/n2snap.so timeout -k 10 300 $B > gpurun_out/r1zm/v354_2.json"
