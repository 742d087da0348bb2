#!/usr/bin/env bash
# covariance carried as N (P = rI + beta D N D, 317 VALU per record) vs the 2S build (323) vs 333:
# GPU tests on the new build, state digests of the three builds (333 vs 2S must be bit-identical),
# C3 / C5 / C2 benches alternating
B="python bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1nc
exec scripts/gpu_session.sh r1nc \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 python scripts/state_digest.py $O/v333.npz" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 python scripts/state_digest.py $O/s2.npz" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 python scripts/state_digest.py $O/nc.npz" \
 "python scripts/cmp_digest.py $O/v333.npz $O/s2.npz > $O/cmp_v333_s2.txt" \
 "python scripts/cmp_digest.py $O/s2.npz $O/nc.npz > $O/cmp_s2_nc.txt" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B --missing > $O/s2_c5_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B --missing > $O/nc_c5_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_2.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_2.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B --batch 65536 > $O/s2_c2_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B --batch 65536 > $O/nc_c2_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B --precision mixed > $O/s2_mixed_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B --precision mixed > $O/nc_mixed_1.json"
