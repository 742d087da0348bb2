# Same-box A/B of k_frontend record stores / event loads with the non-temporal hint, then one
# WRITE_SIZE and one FETCH_SIZE pass per build.  Run from the repo root on the box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4fe_nt; mkdir -p $O
REPS=8 timeout -k 10 400 scripts/ab_frontend.sh ab/frontend_base.so ab/frontend_nt.so ab/frontend_ntl.so > $O/ab.log 2>&1 || exit $?
for v in base nt ntl; do
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_$v.log 2>&1 || exit $?
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/f_$v.log 2>&1 || exit $?
done
cat $O/ab.log
