#!/usr/bin/env bash
# does HBM traffic cost clock? the same launch with the records resident in the Infinity Cache (window 2)
B="python3 bench.py --cpu-baseline none --parity-samples 0"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
exec scripts/gpu_session.sh r1zk \
 "timeout -k 10 300 $B > gpurun_out/r1zk/w1024.json" \
 "timeout -k 10 300 $B --window 2 > gpurun_out/r1zk/w2.json" \
 "timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/r1zk/sq_w2 -o run --output-format csv -- $B --window 2 --steps 1 --warmup 0" \
 "timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r1zk/fetch_w2 -o run --output-format csv -- $B --window 2 --steps 1 --warmup 0"
