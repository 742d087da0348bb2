#!/usr/bin/env bash
# SQ counters of the fused kernel, 3276dda vs the current build, same box
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 1 --warmup 0"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
export PEKF_LIB
exec scripts/gpu_session.sh r1ze \
 "PEKF_LIB=ab/base.so timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r1ze/sq_base -o run --output-format csv -- $B" \
 "PEKF_LIB=ab/new.so timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r1ze/sq_new -o run --output-format csv -- $B" \
 "PEKF_LIB=ab/new.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r1ze/fetch_new -o run --output-format csv -- $B"
