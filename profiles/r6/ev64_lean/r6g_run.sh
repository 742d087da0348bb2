set -o pipefail
O=gpurun_out/r6g; mkdir -p $O
export PEKF_EV64_CACHE=/tmp/ev64_cache.npz TMPDIR=/tmp
timeout -k 10 200 python3 scripts/debug_split64b.py > $O/split.log 2>&1 || exit $?
cat $O/split.log
for v in default ab/frontend_prelean.so default ab/frontend_prelean.so; do
  if [ $v = default ]; then unset PEKF_LIB; else export PEKF_LIB=$PWD/$v; fi
  n=$(basename $v .so)
  timeout -k 10 300 python3 scripts/bench_ev64.py > $O/ev64_$n.json 2> $O/ev64_$n.log || exit $?
  grep -E "live|frontend|run64|init" $O/ev64_$n.log | tr '\n' ' '; echo
done
