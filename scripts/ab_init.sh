#!/usr/bin/env bash
# Same-box A/B of libpekf.so builds on phase 2 (pekf_frontend_init_dev, 1,048,576 filters x 1,024 events,
# HIP-event ms; the stats digest must agree between builds), alternating, two rounds.
# usage: [INIT_MODE=--init-means] scripts/ab_init.sh ab/x.so ab/y.so ...
set -u
for round in 1 2; do
  for lib in "$@"; do
    echo "== $lib round $round"
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 6 ${INIT_MODE:---init} || exit $?
  done
done
