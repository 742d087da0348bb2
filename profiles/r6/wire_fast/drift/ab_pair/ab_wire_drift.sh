#!/usr/bin/env bash
# Same-box comparison of wire-parser builds on aligned and drifted rows (scripts/wire_probe.py --drift):
# each build's wire GPU tests, then the probe at drift 0, 8 and 64 for each build, in order and reversed.
# usage: LIBS="ab/a.so ab/b.so" scripts/ab_wire_drift.sh <out dir>
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/wiredrift}
mkdir -p "$O"
for lib in $LIBS; do
  n=$(basename "$lib" .so)
  PEKF_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_wire_dev.py -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$O/tests_$n.log" 2>&1 || exit 1
done
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for d in 0 8 64; do
  for lib in $LIBS $REV; do
    n=$(basename "$lib" .so)
    PEKF_LIB=$lib timeout -k 10 300 python3 scripts/wire_probe.py 5 --drift $d >> "$O/probe_${n}_d$d.jsonl" \
        2>> "$O/stderr.log" || exit 1
  done
done
echo done
