set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3fe; mkdir -p $O
timeout -k 10 300 scripts/ab_frontend.sh ab/fe_base.so ab/fe_fm.so > $O/ab.log 2>&1 || exit $?
for v in base fm; do
  PEKF_LIB=ab/fe_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_$v.log 2>&1 || exit $?
done
cat $O/ab.log
