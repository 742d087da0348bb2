set -u
mkdir -p gpurun_out/r4_probe
{
echo "== nproc $(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'
echo "== OMP $OMP_NUM_THREADS"
echo "== /proc/self/cgroup"; cat /proc/self/cgroup
echo "== mounts"; grep cgroup /proc/mounts
for f in cpu.max cpuset.cpus.effective cpu.weight cgroup.controllers; do echo "== /sys/fs/cgroup/$f"; cat /sys/fs/cgroup/$f 2>&1; done
p=$(sed -n 's/^0:://p' /proc/self/cgroup); echo "== own path $p"
d=/sys/fs/cgroup$p; while [ "$d" != "/sys/fs" ] && [ -n "$d" ]; do echo "-- $d"; cat $d/cpu.max $d/cpuset.cpus.effective 2>&1; d=$(dirname $d); done
ls /sys/fs/cgroup/ | head -50
} > gpurun_out/r4_probe/cgroup.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_probe/gputests.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r4_probe/gputests.log
