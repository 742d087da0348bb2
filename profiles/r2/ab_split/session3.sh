#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/split3
timeout -k 10 60 scripts/wave_simd_probe > gpurun_out/split3/wave_simd_probe.txt 2>&1 || exit $?
cat gpurun_out/split3/wave_simd_probe.txt
AB_ARGS="--batch 65536" timeout -k 10 500 scripts/ab_libs.sh ab/base.so ab/split8.so ab/split_alt.so 2>&1 | tee gpurun_out/split3/ab_c2.txt
