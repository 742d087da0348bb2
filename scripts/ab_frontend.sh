#!/usr/bin/env bash
# Same-box A/B of front-end builds (ab/fe*.so): the k_frontend workload of scripts/frontend_probe.py
# under each library, alternating, two rounds.
set -u
for round in 1 2; do
  for lib in "$@"; do
    echo "== $lib round $round"
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 5 || exit $?
  done
done
