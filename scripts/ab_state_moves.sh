#!/usr/bin/env bash
# Round 6: the phase-3 state machine with masked moves for f32 events too, and f32 samples held as an
# aligned (x, y) pair + z (pekf_phase3.hpp), against the build before it (ab/base.so, the previous
# commit's libpekf.so).  On one box: the two builds' front-end outputs compared bit for bit
# (scripts/frontend_digest.py), the front-end GPU tests and a fused-vs-split fuzz run on the new build,
# then ABBA (two rounds) of k_live (FP64 records, the default), k_live with f32 records and k_frontend on
# the bench_aux workload (1,048,576 filters x 1,024 events).
# usage: scripts/ab_state_moves.sh check|abba <out dir>   (two gpurun calls: each fits one call's limit)
set -eu
PHASE=$1
OUT=${2:-gpurun_out/moves}
mkdir -p "$OUT"
BASE=ab/base.so
NEW=poseestimationkf_amd/libpekf.so
export PEKF_EV64_CACHE=/tmp/pekf_probe_streams.npz
if [ "$PHASE" = check ]; then
PEKF_LIB=$BASE timeout -k 10 300 python3 -u scripts/frontend_digest.py /tmp/digest_base.npz
PEKF_LIB=$NEW timeout -k 10 300 python3 -u scripts/frontend_digest.py /tmp/digest_new.npz
python3 scripts/frontend_digest.py --compare /tmp/digest_base.npz /tmp/digest_new.npz > "$OUT/digest_compare.txt"
timeout -k 10 600 python3 -u -m pytest tests/test_live.py tests/test_frontend.py tests/test_long_gaps.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
timeout -k 10 600 python3 -u scripts/fuzz_live.py --cases 200 --seed 71 > "$OUT/fuzz_seed71.log" 2>&1
fi
[ "$PHASE" = abba ] || { echo done; exit 0; }
# LIBS: the builds to alternate (default: the base and the new one), in order then reversed, two rounds;
# REPS launches each (the first few run while the clock ramps: compare the last ones)
LIBS=${LIBS:-"$BASE $NEW"}
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for r in 1 2; do
  for lib in $LIBS $REV; do
    for mode in "--live" "--live --f32" ""; do
      echo "== $lib round $r mode '$mode'"
      PEKF_LIB=$lib timeout -k 10 200 python3 scripts/frontend_probe.py ${REPS:-8} $mode
    done
  done
done > "$OUT/abba.log" 2>&1
echo done
