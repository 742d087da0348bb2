# k_frontend's pooled record queue (PEKF_FE_POOL slots per 8-lane group) against the kept per-lane
# 10-row queue (g8s10): for each variant library (ab/frontend_<name>.so, SRC=pekf_frontend
# scripts/build_live_variants.sh), the randomised split-vs-fused sweep (bit-identical records), one
# WRITE_SIZE pass of the probe; then a same-box timing round robin.  Repo root.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r5pool}; mkdir -p $O
V="${V:-g8s10 p78 p74r32 p64 p56}"
for v in $V; do
  PEKF_LIB=ab/frontend_$v.so timeout -k 10 300 python3 -u scripts/fuzz_live.py --cases 200 --seed 61 > $O/fuzz_$v.log 2>&1 || { tail -n 20 $O/fuzz_$v.log; exit 1; }
  tail -n 1 $O/fuzz_$v.log
  PEKF_LIB=ab/frontend_$v.so timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_frontend.py tests/test_long_gaps.py > $O/tests_$v.log 2>&1 || { tail -n 30 $O/tests_$v.log; exit 1; }
  tail -n 1 $O/tests_$v.log
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_$v.log 2>&1 || exit $?
  grep k_frontend $O/w_$v/run_counter_collection.csv | tail -n 1 | awk -F, '{print "'$v' WRITE_SIZE KiB", $(NF-2)}'
done
for round in $(seq ${ROUNDS:-2}); do
  for v in $V; do
    echo "== $v round $round"
    PEKF_LIB=ab/frontend_$v.so timeout -k 10 120 python3 scripts/frontend_probe.py 5 || exit $?
  done
done
