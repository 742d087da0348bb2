#!/usr/bin/env bash
# Same-box ABBA of k_run's HOIST schedule (PEKF_RUN_HOIST=0 / 1, one library) at config 2 (65,536
# filters: one wave per SIMD) and config 3 (1,048,576), kernel ms by HIP events; then the state
# digests of both schedules, which must be bit-identical.
set -u
out=${1:-gpurun_out/ab_hoist}
mkdir -p "$out"
B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2"
for cfg in c2 c3; do
  args=""; [ $cfg = c2 ] && args="--batch 65536"
  for r in 1 2; do
    for h in 0 1 1 0; do
      echo "== $cfg hoist=$h round $r"
      PEKF_RUN_HOIST=$h timeout -k 10 200 $B $args 2>&1 >/dev/null | grep "timed:" || exit $?
    done
  done
done
for h in 0 1; do
  PEKF_RUN_HOIST=$h timeout -k 10 200 python3 scripts/state_digest.py "/tmp/digest_h$h.npz" || exit $?
done
python3 scripts/cmp_digest.py /tmp/digest_h0.npz /tmp/digest_h1.npz   # (~40 MB each: not in gpurun_out)
