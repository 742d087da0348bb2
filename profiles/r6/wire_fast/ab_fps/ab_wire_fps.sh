#!/usr/bin/env bash
# One or two frame indices per step of k_wire_events (PEKF_WIRE_FPS) by batch, same box: the wire GPU tests
# and scripts/fuzz_wire.py under each form, then scripts/wire_probe.py at 65,536 / 131,072 / 262,144 phones
# and the session probe under each (and the library $BASE, one frame per step, beside them).
# usage: LIB=ab/new.so BASE=ab/old.so scripts/ab_wire_fps.sh <out dir>
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/wirefps}
mkdir -p "$O"
for fps in 1 2; do
  PEKF_WIRE_FPS=$fps PEKF_LIB=$LIB timeout -k 10 300 python3 -u -m pytest tests/test_wire_dev.py -m gpu -x -q \
      --timeout 200 --timeout-method thread > "$O/tests_fps$fps.log" 2>&1 || exit 1
  PEKF_WIRE_FPS=$fps PEKF_LIB=$LIB timeout -k 10 300 python3 -u scripts/fuzz_wire.py --cases 30 --seed 74$fps \
      > "$O/fuzz_fps$fps.log" 2>&1 || exit 1
done
for rep in 1 2; do
  for tile in 64 128 256; do
    PEKF_LIB=$BASE timeout -k 10 300 python3 scripts/wire_probe.py 5 --tile $tile >> "$O/probe_base_t$tile.jsonl" 2>> "$O/stderr.log" || exit 1
    for fps in 1 2; do
      PEKF_WIRE_FPS=$fps PEKF_LIB=$LIB timeout -k 10 300 python3 scripts/wire_probe.py 5 --tile $tile \
          >> "$O/probe_fps${fps}_t$tile.jsonl" 2>> "$O/stderr.log" || exit 1
    done
  done
  PEKF_LIB=$BASE timeout -k 10 300 python3 scripts/wire_probe.py 5 --session >> "$O/session_base.jsonl" 2>> "$O/stderr.log" || exit 1
  for fps in 1 2; do
    PEKF_WIRE_FPS=$fps PEKF_LIB=$LIB timeout -k 10 300 python3 scripts/wire_probe.py 5 --session \
        >> "$O/session_fps$fps.jsonl" 2>> "$O/stderr.log" || exit 1
  done
done
echo done
