set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -8 $O/tests.log; exit $rc
