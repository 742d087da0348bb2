#!/usr/bin/env bash
exec scripts/gpu_session.sh r1d \
 "timeout -k 10 400 python -m pytest tests -m gpu -q -s -p no:cacheprovider" \
 "timeout -k 10 120 build/probe_fp64" \
 "timeout -k 10 400 python bench.py --steps 3 --warmup 1" \
 "timeout -k 10 300 python bench.py --steps 3 --warmup 1 --precision mixed --cpu-baseline none" \
 "timeout -k 10 300 python bench.py --steps 3 --warmup 1 --dist --cpu-baseline none --parity-samples 4"
