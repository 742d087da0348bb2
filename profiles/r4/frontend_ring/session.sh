set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fering; mkdir -p $O
for r in 1 2; do
  for lib in ab/frontend_base.so ab/frontend_r12.so ab/frontend_r18.so ab/frontend_r24.so ab/frontend_r24.so ab/frontend_r18.so ab/frontend_r12.so ab/frontend_base.so; do
    echo "== $lib round $r"
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 10 || exit 1
  done
done > $O/ab.log 2>&1
python3 scripts/ab_summary.py $O/ab.log 5
