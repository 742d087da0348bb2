# The committed k_frontend (10-row LDS queue): randomised split-vs-fused sweep (scripts/fuzz_live.py,
# two seeds; the split pipeline's records come from k_frontend), then one WRITE_SIZE and one FETCH_SIZE
# pass and an SQ pass of the probe.  Repo root.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4fe_final; mkdir -p $O
for s in 51 52; do
  timeout -k 10 300 python3 -u scripts/fuzz_live.py --cases 600 --seed $s > $O/fuzz_seed$s.log 2>&1 || { tail -n 20 $O/fuzz_seed$s.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/f.log 2>&1 || exit $?
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/sq -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/sq.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/frontend_probe.py 6 > $O/probe.log 2>&1 || exit $?
tail -n 1 $O/fuzz_seed*.log
cat $O/probe.log
