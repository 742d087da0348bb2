#!/usr/bin/env bash
# Same-box ABBA of k_live's record precision: f32 stream records vs FP64 low-pass acc / mag
# (the default; PEKF_EV_F32_RECORDS gives f32), 1,048,576 filters x 1,024 events, HIP-event ms of pekf_live_ext_dev.
set -u
for mode in f32 f64 f64 f32 f32 f64; do
  echo "== $mode"
  flag=""; [ "$mode" = f32 ] && flag=--f32
  timeout -k 10 120 python3 scripts/frontend_probe.py ${REPS:-5} --live $flag || exit $?
done
