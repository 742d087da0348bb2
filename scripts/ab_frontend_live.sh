#!/usr/bin/env bash
# Same-box A/B of libpekf.so builds on the front-end kernel and the fused front-end + filter kernel
# (scripts/frontend_probe.py, with and without --live), alternating the libraries, two rounds.
# usage: scripts/ab_frontend_live.sh ab/x.so ab/y.so ...
set -u
for round in 1 2; do
  for lib in "$@"; do
    echo "== $lib round $round"
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 4 || exit $?
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 4 --live || exit $?
  done
done
