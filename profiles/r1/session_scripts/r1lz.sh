#!/usr/bin/env bash
# X left unnormalised between records + q_W recomputed where needed (RefWLazy; 312 VALU, 114 VGPRs)
# vs the N-carry build (317, 126 VGPRs): GPU tests on the new build, digests, C3 x4 / C5 / mixed / C2
B="python bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1lz
exec scripts/gpu_session.sh r1lz \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 python scripts/state_digest.py /tmp/nc.npz" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 python scripts/state_digest.py /tmp/lz.npz" \
 "python scripts/cmp_digest.py /tmp/nc.npz /tmp/lz.npz > $O/cmp_nc_lz.txt" \
 "rm -f /tmp/nc.npz /tmp/lz.npz" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B > $O/lz_c3_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_1.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B > $O/lz_c3_2.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_2.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B > $O/lz_c3_3.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_3.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B --missing > $O/lz_c5_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B --missing > $O/nc_c5_1.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B --precision mixed > $O/lz_mixed_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B --precision mixed > $O/nc_mixed_1.json" \
 "PEKF_LIB=ab/lz.so timeout -k 10 300 $B --batch 65536 > $O/lz_c2_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B --batch 65536 > $O/nc_c2_1.json"
