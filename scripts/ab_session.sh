#!/usr/bin/env bash
# Same-box A/B of two libpekf.so builds: state digests (bit-for-bit comparison, files kept in /tmp),
# the GPU test suite on the working-tree build, then config-3 and config-2 timings alternating.
# usage: scripts/ab_session.sh <tag> <base.so> <new.so>
set -u
tag=$1; base=$2; new=$3
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2"
scripts/gpu_session.sh "$tag" \
 "PEKF_LIB=$new timeout -k 10 120 python3 scripts/state_digest.py /tmp/${tag}_new.npz" \
 "PEKF_LIB=$base timeout -k 10 120 python3 scripts/state_digest.py /tmp/${tag}_base.npz" \
 "python3 scripts/cmp_digest.py /tmp/${tag}_base.npz /tmp/${tag}_new.npz" \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "scripts/ab_libs.sh $base $new" \
 "AB_ARGS='--batch 65536' scripts/ab_libs.sh $base $new"
