#!/usr/bin/env bash
# PMC of the fused front-end + filter kernel in steady state for one libpekf build (PEKF_LIB): 10
# launches of frontend_probe.py --live, one SQ pass and one FETCH_SIZE pass, summary of the last
# launch (scripts/pmc_live_summary.py).  usage: scripts/pmc_live_variant.sh <out dir> <lib.so> [--ev64]
set -u
O=$1; LIB=$2; EV=${3:-}; mkdir -p $O
EVB=16; [ "$EV" = "--ev64" ] && EVB=32
export TMPDIR=/tmp PEKF_LIB=$LIB
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 180 rocprofv3 --pmc $SQ -d $O/sq -o run --output-format csv -- python3 scripts/frontend_probe.py 10 --live $EV > $O/sq.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 scripts/frontend_probe.py 10 --live $EV > $O/fetch.log 2>&1 || exit $?
python3 scripts/pmc_live_summary.py $O/sq/run_counter_collection.csv $O/fetch/run_counter_collection.csv $EVB > $O/summary.json
cat $O/summary.json
