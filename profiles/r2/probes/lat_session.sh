set -u
O=gpurun_out/lat; mkdir -p $O
timeout -k 10 60 build/probe_latency > $O/probe_latency.txt 2>&1 || exit $?
cat $O/probe_latency.txt
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
B="python3 bench.py --cpu-baseline none --parity-samples 0 --batch 65536"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 0 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/pmc_sq -o run --output-format csv -- $B --steps 1 --warmup 0 > $O/sq.log 2>&1 || exit $?
python3 scripts/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_sq/run_counter_collection.csv 65536 10000 $O/pmc_summary_c2.json && cat $O/pmc_summary_c2.json
