#!/usr/bin/env bash
# Config 4's eight per-rank workloads (filters r*2^20 ... (r+1)*2^20 - 1 of the 8,388,608-filter job,
# 10,000 records each) run one after another on ONE GPU through bench.py --shard-of r/8: the per-GPU
# kernel time and parity of every shard at its global filter ids.  Not an 8-GPU measurement (the
# driver runs that); a rehearsal of every rank's workload.  usage: scripts/c4_shards.sh <out-dir>
set -u
out=$1
mkdir -p "$out"
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 200 python3 bench.py --shard-of $r/8 --cpu-baseline none --steps 3 --warmup 1 \
      --parity-samples 32 > "$out/shard_$r.json" 2> "$out/shard_$r.log" || exit $?
  grep -h "timed:\|parity:" "$out/shard_$r.log"
done
