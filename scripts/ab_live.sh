#!/usr/bin/env bash
# Same-box A/B of libpekf.so builds on the fused front-end + filter kernel (1,048,576 filters x 1,024
# events, HIP-event ms of pekf_live_dev), alternating the libraries given, two rounds.
# usage: scripts/ab_live.sh ab/live_x.so ab/live_y.so ...
set -u
for round in 1 2; do
  for lib in "$@"; do
    echo "== $lib round $round"
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py ${REPS:-4} --live || exit $?
  done
done
