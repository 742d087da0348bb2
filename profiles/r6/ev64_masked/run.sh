set -o pipefail
O=gpurun_out/r6h; mkdir -p $O
export PEKF_EV64_CACHE=/tmp/ev64_cache.npz TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_live.py tests/test_frontend.py -x -q -s --timeout 200 --timeout-method thread -k "fp64 or session or zero_time" > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|vs the|events" $O/tests.log | tail -20; [ $rc -le 1 ] || exit $rc
for v in default ab/live_sel.so default ab/live_sel.so; do
  if [ $v = default ]; then unset PEKF_LIB; else export PEKF_LIB=$PWD/$v; fi
  n=$(basename $v .so)
  PEKF_EV64_ONLY=live timeout -k 10 300 python3 scripts/bench_ev64.py > $O/ev64_$n.json 2> $O/ev64_$n.log || exit $?
  grep -E "live" $O/ev64_$n.log | tr '\n' ' '; echo
done
bash scripts/pmc_live_variant.sh $O/pmc_ev64 $PWD/poseestimationkf_amd/libpekf.so --ev64 > /dev/null || exit $?
python3 -c "import json; d=json.load(open('$O/pmc_ev64/summary.json')); print({k: d[k] for k in ('valu_insts_per_wave','valu_busy','effective_clock_ghz','traffic_over_algorithmic','kernel_ns_sq_pass')})"
