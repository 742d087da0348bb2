#!/usr/bin/env bash
exec scripts/gpu_session.sh r1s \
 "timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider -x"
