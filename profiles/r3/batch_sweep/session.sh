#!/usr/bin/env bash
# Headline kernel rate against the batch (filters per GPU): 64K (config 2, one wave per SIMD) up to 4M
# (172 GB of resident window), 10,000 records per launch; one bench line per batch into $1/.
set -u
out=${1:-gpurun_out/sweep}; mkdir -p "$out"
for b in 65536 131072 196608 262144 524288 786432 1048576 2097152 4194304; do
  timeout -k 10 300 python3 bench.py --batch $b --steps 2 --warmup 1 --cpu-baseline none --parity-samples 4 \
      > "$out/b$b.json" 2> "$out/b$b.err" || exit $?
  python3 -c "import json,sys; d=json.load(open('$out/b$b.json')); print('$b', round(d['roofline']['kernel_ms'],3), '%.3e' % d['value'], round(d['valu_roofline']['frac'],3), d['parity']['max_abs_err_vs_oracle'])"
done
