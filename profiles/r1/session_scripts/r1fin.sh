#!/usr/bin/env bash
# profile refresh (312-VALU build): parity suite, smoke, kernel trace, PMC passes,
# bench lines (C3 with the CPU baseline, C2, C5, mixed), the RCCL path at world size 1, aux kernels
B="python3 bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1fin
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
exec scripts/gpu_session.sh r1fin \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B --steps 3 --warmup 1" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 0" \
 "timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/pmc_sq -o run --output-format csv -- $B --steps 1 --warmup 0" \
 "python3 scripts/pmc_summary.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_sq/run_counter_collection.csv 1048576 10000 profiles/r1/pmc_summary_c3.json && cp profiles/r1/pmc_summary_c3.json $O/" \
 "timeout -k 10 400 python bench.py > $O/bench_c3_f64.json" \
 "timeout -k 10 300 python bench.py --batch 65536 --cpu-baseline none > $O/bench_c2_f64.json" \
 "timeout -k 10 300 python bench.py --missing --cpu-baseline none > $O/bench_c5_f64.json" \
 "timeout -k 10 300 python bench.py --precision mixed --cpu-baseline none > $O/bench_c3_mixed.json" \
 "timeout -k 10 300 python bench.py --dist --cpu-baseline none --steps 2 > $O/bench_dist1.json" \
 "timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/auxtrace -o aux --output-format csv -- python3 scripts/bench_aux.py > $O/aux_bench.json"
