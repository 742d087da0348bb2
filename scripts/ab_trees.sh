#!/usr/bin/env bash
# Same-box A/B of two whole checkouts (their own bench.py, Python layer and libraries), e.g. the
# round's starting tree copied under ab/ against the working tree; config 3, 2 and 5, alternating.
# usage: scripts/ab_trees.sh <other-tree-dir>
set -u
other=$1
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2"
for args in "" "--batch 65536" "--missing"; do
  for round in 1 2; do
    for tree in "$other" .; do
      echo "== $tree $args round $round"
      (cd "$tree" && timeout -k 10 200 $B $args 2>&1 >/dev/null | grep "timed:") || exit $?
    done
  done
done
