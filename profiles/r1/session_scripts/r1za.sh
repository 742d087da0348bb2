#!/usr/bin/env bash
# re-entry check of the restored tree: GPU parity suite, smoke, default bench line
exec scripts/gpu_session.sh r1za \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "timeout -k 10 500 python bench.py > gpurun_out/r1za/bench_default.json"
