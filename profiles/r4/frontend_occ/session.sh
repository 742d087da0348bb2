# k_frontend: what do the record stores cost (records formed, stores skipped), and does capping the
# waves per CU (dynamic LDS) let L2 merge more of the scattered record stores?  Same-box A/B, then
# WRITE_SIZE per build and one SQ pass of the base build.  Run from the repo root on the box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4fe_occ; mkdir -p $O
timeout -k 10 400 scripts/ab_frontend.sh ab/frontend_base.so ab/frontend_nostore.so ab/frontend_occ2.so > $O/ab.log 2>&1 || exit $?
for v in base occ2; do
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/w_$v.log 2>&1 || exit $?
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for v in base nostore; do
  PEKF_LIB=ab/frontend_$v.so timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/sq_$v -o run --output-format csv -- python3 scripts/frontend_probe.py 2 > $O/sq_$v.log 2>&1 || exit $?
done
PEKF_LIB=ab/frontend_occ1.so timeout -k 10 120 python3 scripts/frontend_probe.py 5 > $O/occ1.log 2>&1
echo "occ1 rc=$?" >> $O/occ1.log
cat $O/ab.log $O/occ1.log
