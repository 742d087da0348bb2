#!/usr/bin/env bash
# Same-box A/B of two libpekf.so builds on the kernels beside the headline (scripts/bench_aux.py).
set -u
for r in 1 2; do for lib in "$@"; do echo "== $lib"; PEKF_LIB=$lib timeout -k 10 200 python3 scripts/bench_aux.py 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(' '.join('%s=%.4f' % (k, d[k]['kernel_ms']) for k in ('frontend','gyro_chain','wahba_stream','online_step_aos','online_step_soa','handle_update_aos','handle_update_soa','predict_dev','correct_dev')))" || exit 1; done; done
