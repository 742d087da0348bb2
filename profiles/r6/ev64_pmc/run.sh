set -o pipefail
O=gpurun_out/r6f; mkdir -p $O
export PEKF_EV64_CACHE=/tmp/ev64_cache.npz TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_live.py tests/test_frontend.py -x -q -s --timeout 200 --timeout-method thread -k "fp64 or session or zero_time" > $O/tests.log 2>&1; rc=$?; grep -E "passed|failed|vs the|events" $O/tests.log | tail -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_ev64.py > $O/ev64.json 2> $O/ev64.log || exit $?
tail -12 $O/ev64.log
bash scripts/pmc_live_variant.sh $O/pmc_ev64 $PWD/poseestimationkf_amd/libpekf.so --ev64 || exit $?
bash scripts/pmc_live_variant.sh $O/pmc_f32 $PWD/poseestimationkf_amd/libpekf.so || exit $?
