#!/usr/bin/env bash
# Same-box comparison of builds of the device wire parser (pekf_wire_dev.hip): the wire GPU tests on each
# build, then scripts/wire_probe.py (262,144 phones x 1,024 frames) on each, in order and reversed, and
# with SESSION=1 the session probe (65,536 phones, one wave per SIMD) on each.
# usage: LIBS="ab/a.so ab/b.so" [SESSION=1] scripts/ab_wire.sh <out dir>
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/wireab}
mkdir -p "$O"
LIBS=${LIBS:-poseestimationkf_amd/libpekf.so}
for lib in $LIBS; do
  n=$(basename "$lib" .so)
  PEKF_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_wire_dev.py -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$O/tests_$n.log" 2>&1 || exit 1
done
REV=$(echo $LIBS | tr ' ' '\n' | tac | tr '\n' ' ')
for lib in $LIBS $REV; do
  n=$(basename "$lib" .so)
  PEKF_LIB=$lib timeout -k 10 300 python3 scripts/wire_probe.py 5 >> "$O/probe_$n.jsonl" 2>> "$O/stderr.log" || exit 1
done
if [ "${SESSION:-0}" = 1 ]; then
  for lib in $LIBS $REV; do
    n=$(basename "$lib" .so)
    PEKF_LIB=$lib timeout -k 10 300 python3 scripts/wire_probe.py 5 --session >> "$O/session_$n.jsonl" \
        2>> "$O/stderr.log" || exit 1
  done
fi
echo done
