#!/usr/bin/env bash
# second same-box A/B of the N-carry build (nc) against the 2S build (s2): digests compared on the
# box (the .npz files stay in /tmp), C3 four times each, alternating
B="python bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1nc2
exec scripts/gpu_session.sh r1nc2 \
 "PEKF_LIB=ab/cur.so timeout -k 10 300 python scripts/state_digest.py /tmp/v333.npz" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 python scripts/state_digest.py /tmp/s2.npz" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 python scripts/state_digest.py /tmp/nc.npz" \
 "python scripts/cmp_digest.py /tmp/v333.npz /tmp/s2.npz > $O/cmp_v333_s2.txt" \
 "python scripts/cmp_digest.py /tmp/s2.npz /tmp/nc.npz > $O/cmp_s2_nc.txt" \
 "rm -f /tmp/v333.npz /tmp/s2.npz /tmp/nc.npz" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_1.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_1.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_2.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_2.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_3.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_3.json" \
 "PEKF_LIB=ab/nc.so timeout -k 10 300 $B > $O/nc_c3_4.json" \
 "PEKF_LIB=ab/s2.so timeout -k 10 300 $B > $O/s2_c3_4.json"
