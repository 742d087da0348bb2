set -o pipefail
O=gpurun_out/r6e; mkdir -p $O
export PEKF_EV64_CACHE=/tmp/ev64_cache.npz
timeout -k 10 400 python3 -u -m pytest tests/test_live.py tests/test_frontend.py -x -q -s --timeout 200 --timeout-method thread -k "fp64 or session or zero_time" > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|vs the|events" $O/tests.log | tail -20; [ $rc -le 1 ] || exit $rc
for v in default ab/live_lean_w2.so ab/live_lean_w2q3.so ab/live_lean_w1q8.so ab/live_lean_w2.so default; do
  if [ $v = default ]; then unset PEKF_LIB; else export PEKF_LIB=$PWD/$v; fi
  n=$(basename $v .so)
  PEKF_EV64_ONLY=live timeout -k 10 300 python3 scripts/bench_ev64.py > $O/ev64_$n.json 2> $O/ev64_$n.log || exit $?
  tail -3 $O/ev64_$n.log
done
