# k_frontend with the per-wave LDS row queue (PEKF_FE_STAGE rows, THR): parity of two builds on the
# front-end tests, same-box A/B against the direct-store build, WRITE_SIZE per build.  Repo root.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4fe_stage; mkdir -p $O
for v in s16t60 s8t56; do
  PEKF_LIB=ab/frontend_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_frontend.py tests/test_live.py tests/test_long_gaps.py > $O/parity_$v.log 2>&1 || { cat $O/parity_$v.log | tail -30; exit 1; }
done
timeout -k 10 600 scripts/ab_frontend.sh ab/frontend_base.so ab/frontend_s16t60.so ab/frontend_s16t56.so ab/frontend_s12t56.so ab/frontend_s8t56.so > $O/ab.log 2>&1 || exit $?
for v in base s16t60 s12t56 s8t56; do
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_$v.log 2>&1 || exit $?
done
tail -2 $O/parity_*.log
cat $O/ab.log
