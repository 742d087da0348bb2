# PMC passes of k_live with FP64 records (the default) and f32 records (PEKF_EV_F32_RECORDS), the
# frontend_probe --live workload (1,048,576 filters x 1,024 events).  Repo root.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5livepmc; mkdir -p $O
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for m in f64 f32; do
  flag=""; [ $m = f32 ] && flag=--f32
  timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/sq_$m -o run --output-format csv -- python3 scripts/frontend_probe.py 3 --live $flag > $O/sq_$m.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$m -o run --output-format csv -- python3 scripts/frontend_probe.py 3 --live $flag > $O/f_$m.log 2>&1 || exit $?
  python3 scripts/pmc_live_summary.py $O/sq_$m/run_counter_collection.csv $O/f_$m/run_counter_collection.csv > $O/pmc_$m.json || exit $?
  echo "== $m"; cat $O/pmc_$m.json
done
