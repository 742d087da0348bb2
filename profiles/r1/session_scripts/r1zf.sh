#!/usr/bin/env bash
# profile refresh for the 360-VALU fused kernel: bench lines, kernel trace, PMC passes
B="python3 bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/r1zf
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
exec scripts/gpu_session.sh r1zf \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B --steps 3 --warmup 1" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 0" \
 "timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/pmc_sq -o run --output-format csv -- $B --steps 1 --warmup 0" \
 "timeout -k 10 400 python bench.py > $O/bench_c3_f64.json" \
 "timeout -k 10 300 python bench.py --batch 65536 --cpu-baseline none > $O/bench_c2_f64.json" \
 "timeout -k 10 300 python bench.py --missing --cpu-baseline none > $O/bench_c5_f64.json" \
 "timeout -k 10 300 python bench.py --precision mixed --cpu-baseline none > $O/bench_c3_mixed.json"
