set -u
for round in 1 2; do
  for lib in ab/live_q4.so ab/live_q5.so ab/live_q5.so ab/live_q4.so; do
    echo "== $lib round $round"
    PEKF_LIB=$lib timeout -k 10 120 python3 scripts/frontend_probe.py 5 --live || exit $?
  done
done
