# Sweep of the queue depth (rows), write threshold and check period of k_frontend's LDS row queue:
# same-box A/B against the direct-store build (base), then WRITE_SIZE of the chosen setting.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4fe_sweep2; mkdir -p $O
timeout -k 10 900 scripts/ab_frontend.sh ab/frontend_base.so ab/frontend_s10t56.so ab/frontend_s10t52.so ab/frontend_s10t58.so ab/frontend_s9t56.so ab/frontend_s11t56.so ab/frontend_s10t56e3.so > $O/ab.log 2>&1 || exit $?
PEKF_LIB=ab/frontend_s10t56.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_s10t56 -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_s10t56.log 2>&1 || exit $?
cat $O/ab.log
