#!/usr/bin/env bash
# GPU parity suite (adds arbitrary reference frames)
exec scripts/gpu_session.sh r1zy \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
