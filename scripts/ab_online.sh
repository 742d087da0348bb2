set -u
for r in 1 2 3; do for lib in ab/prev.so ab/one.so; do echo "== $lib"; PEKF_LIB=$lib timeout -k 10 120 python3 scripts/online_probe.py 50 || exit $?; done; done
