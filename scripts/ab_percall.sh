#!/usr/bin/env bash
# Same-box A/B of the n = 1 per-call latency (scripts/percall_latency.cpp, C entry points, resident
# service) between two libpekf.so builds, alternated A B B A twice.  The probe finds libpekf.so through
# its RUNPATH, so LD_LIBRARY_PATH selects the build.  usage: scripts/ab_percall.sh <dirA> <dirB>
set -u
for r in 1 2; do
  for d in $1 $2 $2 $1; do
    echo "== $d round $r"
    LD_LIBRARY_PATH=$d timeout -k 5 60 build/percall_latency || exit $?
  done
done
# config 1's drop-in loop (main_file.py:38-46 over the committed log, scripts/bench_aux.py c1_loop)
# with each build: LD_LIBRARY_PATH makes _fastcall.so bind the same libpekf.so that PEKF_LIB loads
for r in 1 2; do
  for d in $1 $2 $2 $1; do
    echo "== c1 loop $d round $r"
    PEKF_LIB=$d/libpekf.so LD_LIBRARY_PATH=$d timeout -k 5 120 python3 -c \
      "import sys; sys.path.insert(0, 'scripts'); import bench_aux; print(bench_aux.c1_loop())" || exit $?
  done
done
