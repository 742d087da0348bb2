#!/usr/bin/env bash
# A/B of the small-batch split kernel (pekf_run_split.hip) against the one-lane kernel at config 2
tag=${1:-split2}
B="python3 bench.py --cpu-baseline none --parity-samples 0"
O=gpurun_out/$tag
exec scripts/gpu_session.sh $tag \
 "timeout -k 10 300 python -u -m pytest tests/test_split_kernel.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_RUN_SPLIT=0 timeout -k 10 300 $B --batch 65536 > $O/c2_onelane_a.json" \
 "PEKF_RUN_SPLIT=1 timeout -k 10 300 $B --batch 65536 > $O/c2_split_a.json" \
 "PEKF_RUN_SPLIT=0 timeout -k 10 300 $B --batch 65536 > $O/c2_onelane_b.json" \
 "PEKF_RUN_SPLIT=1 timeout -k 10 300 $B --batch 65536 > $O/c2_split_b.json" \
 "PEKF_RUN_SPLIT=1 timeout -k 10 300 $B --batch 262144 > $O/b256k_split.json" \
 "PEKF_RUN_SPLIT=0 timeout -k 10 300 $B --batch 262144 > $O/b256k_onelane.json"
