#!/usr/bin/env bash
# A/B of the fused front-end + filter kernel with and without the PIN schedule of ekf_record_step
# (ab/live_off.so, ab/live_on.so), order-balanced, the "live" line of scripts/bench_aux.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/livepin; mkdir -p $O
timeout -k 10 300 env PEKF_LIB=ab/live_on.so python -u -m pytest tests/test_live.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_on.log 2>&1 || { tail -20 $O/tests_on.log; exit 1; }
tail -1 $O/tests_on.log
for lib in live_off live_on live_on live_off; do
  PEKF_AUX_ONLY=live PEKF_LIB=ab/$lib.so timeout -k 10 200 python3 scripts/bench_aux.py > $O/aux_$lib.json 2> $O/aux_$lib.err || exit $?
  echo "$lib $(grep -o 'fused front-end + filter: .*' $O/aux_$lib.err)"
done
