#!/usr/bin/env bash
# 2S innovation covariance (323 VALU per record without missing magnetometer samples) vs current (333):
# GPU tests on the new build, bitwise state digests of both builds, C3 / C5 benches alternating
B="python bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1s2
exec scripts/gpu_session.sh r1s2 \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 python scripts/state_digest.py $O/cur.npz" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 python scripts/state_digest.py $O/s2.npz" \
 "python scripts/cmp_digest.py $O/cur.npz $O/s2.npz > $O/cmp.txt" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B > $O/cur_c3_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_1.json" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B --missing > $O/cur_c5_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B --missing > $O/s2_c5_1.json" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B > $O/cur_c3_2.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_2.json" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 $B --batch 65536 > $O/cur_c2_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B --batch 65536 > $O/s2_c2_1.json"
