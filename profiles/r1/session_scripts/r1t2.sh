#!/usr/bin/env bash
# GPU test suite on the final build (adds the chunked non-trajectory run at other noise scales)
exec scripts/gpu_session.sh r1t2 \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
