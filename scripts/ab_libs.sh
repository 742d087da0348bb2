#!/usr/bin/env bash
# Same-box A/B of libpekf.so builds on the config-3 bench (kernel ms by HIP events), alternating
# the libraries given as arguments, two rounds.  usage: scripts/ab_libs.sh ab/x.so ab/y.so ...
set -u
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2 ${AB_ARGS:-}"
for round in 1 2; do
  for lib in "$@"; do
    echo "== $lib round $round"
    PEKF_LIB=$lib timeout -k 10 200 $B 2>&1 >/dev/null | grep "timed:" || exit $?
  done
done
