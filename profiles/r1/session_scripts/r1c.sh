#!/usr/bin/env bash
# round-1 measurement session: parity tests, configs 3/5/2, rocprofv3 kernel trace + PMC passes
B="python3 bench.py --cpu-baseline none --parity-samples 0"
exec scripts/gpu_session.sh r1c \
 "timeout -k 10 400 python -m pytest tests -m gpu -q -s -p no:cacheprovider" \
 "timeout -k 10 400 python bench.py --steps 3 --warmup 1" \
 "timeout -k 10 300 python bench.py --steps 3 --warmup 1 --missing --cpu-baseline none" \
 "timeout -k 10 300 python bench.py --steps 3 --warmup 1 --batch 65536 --cpu-baseline none" \
 "timeout -k 10 120 rocprofv3 -L > gpurun_out/r1c/counters.txt 2>&1; grep -c . gpurun_out/r1c/counters.txt" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r1c/trace -o run --output-format csv -- $B --steps 3 --warmup 1" \
 "timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r1c/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 0" \
 "timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/r1c/pmc_sq -o run --output-format csv -- $B --steps 1 --warmup 0"
