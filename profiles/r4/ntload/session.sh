# Non-temporal event loads (every event is read once) in k_frontend, k_live and phase 2: order-balanced
# (ABBA, two rounds) same-box A/B, 12 launches each (the first ones run while the clock ramps).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ntload; mkdir -p $O
abba() {  # abba <mode flag or ""> <a.so> <b.so>
  for r in 1 2; do
    for lib in $2 $3 $3 $2; do
      echo "== $lib round $r"
      PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 12 $1 || return 1
    done
  done
}
abba "" ab/frontend_base.so ab/frontend_ntl.so > $O/frontend.log 2>&1 || exit 1
abba --live ab/live_base.so ab/live_ntl.so > $O/live.log 2>&1 || exit 1
abba --init-means ab/frontend_p2base.so ab/frontend_base.so > $O/init_means.log 2>&1 || exit 1
for f in frontend live init_means; do echo "-- $f"; python3 scripts/ab_summary.py $O/$f.log 6; done
