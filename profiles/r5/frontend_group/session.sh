# k_frontend with per-lane-group queue bases (PEKF_FE_GROUP) and deeper queues: for each variant
# library (ab/frontend_<name>.so, SRC=pekf_frontend scripts/build_live_variants.sh), the randomised
# split-vs-fused sweep (the split pipeline's records come from k_frontend: bit-identical records), one
# WRITE_SIZE pass of the probe; then a same-box timing round robin over all of them.  Repo root.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5fe; mkdir -p $O
V="g64s10 g8s10 g8s12 g8s14 g8s16 g16s14"
for v in $V; do
  PEKF_LIB=ab/frontend_$v.so timeout -k 10 300 python3 -u scripts/fuzz_live.py --cases 200 --seed 61 > $O/fuzz_$v.log 2>&1 || { tail -n 20 $O/fuzz_$v.log; exit 1; }
  tail -n 1 $O/fuzz_$v.log
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_$v.log 2>&1 || exit $?
  grep k_frontend $O/w_$v/run_counter_collection.csv | tail -n 1 | awk -F, '{print "'$v' WRITE_SIZE KiB", $(NF-2)}'
done
for round in 1 2; do
  for v in $V; do
    echo "== $v round $round"
    PEKF_LIB=ab/frontend_$v.so timeout -k 10 120 python3 scripts/frontend_probe.py 5 || exit $?
  done
done
