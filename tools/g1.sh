set -o pipefail
O=gpurun_out/g1; mkdir -p $O
(nproc; python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max; grep -m1 'model name' /proc/cpuinfo) > $O/host.txt 2>&1
timeout -k 10 300 python3 tools/gpu_quick.py > $O/quick.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1
echo exit $?
