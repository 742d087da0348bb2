#!/usr/bin/env bash
# Order-balanced (ABBA, two rounds) same-box A/B of two libpekf.so builds on the config-3 bench
# (kernel ms by HIP events).  usage: scripts/ab_abba.sh ab/a.so ab/b.so [extra bench args]
set -u
A=$1; Bl=$2; shift 2
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2 $*"
for r in 1 2; do
  for lib in $A $Bl $Bl $A; do
    echo "== $lib round $r"
    PEKF_LIB=$lib timeout -k 10 200 $B 2>&1 >/dev/null | grep "timed:" || exit $?
  done
done
