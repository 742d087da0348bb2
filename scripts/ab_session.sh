B="python3 bench.py --cpu-baseline none --parity-samples 0 --steps 5 --warmup 2"
scripts/gpu_session.sh ab_omod \
 "timeout -k 10 120 python3 scripts/state_digest.py gpurun_out/ab_omod/new.npz" \
 "PEKF_LIB=ab/base.so timeout -k 10 120 python3 scripts/state_digest.py gpurun_out/ab_omod/base.npz" \
 "python3 scripts/cmp_digest.py gpurun_out/ab_omod/base.npz gpurun_out/ab_omod/new.npz" \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
 "PEKF_LIB=ab/base.so timeout -k 10 200 $B > gpurun_out/ab_omod/base1.json" \
 "timeout -k 10 200 $B > gpurun_out/ab_omod/new1.json" \
 "PEKF_LIB=ab/base.so timeout -k 10 200 $B > gpurun_out/ab_omod/base2.json" \
 "timeout -k 10 200 $B > gpurun_out/ab_omod/new2.json"
