set -o pipefail
O=gpurun_out/r6b; mkdir -p $O
export PEKF_EV64_CACHE=/tmp/ev64_cache.npz
timeout -k 10 400 python3 -u -m pytest tests/test_live.py tests/test_frontend.py tests/test_wire.py -x -q --timeout 200 --timeout-method thread -k "fp64 or wire or session" > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -le 1 ] || exit $rc
for v in default ab/live_w2q4.so ab/live_w1q8.so ab/live_w1q6.so ab/frontend_base.so ab/frontend_r6.so ab/frontend_p64.so default; do
  if [ $v = default ]; then unset PEKF_LIB; else export PEKF_LIB=$PWD/$v; fi
  n=$(basename $v .so)
  timeout -k 10 300 python3 scripts/bench_ev64.py > $O/ev64_$n.json 2> $O/ev64_$n.log || exit $?
  tail -12 $O/ev64_$n.log
done
