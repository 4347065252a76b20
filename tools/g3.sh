set -o pipefail
O=gpurun_out/g3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline > $O/bench.json 2> $O/bench.err &&
bash tools/pmc_run.sh $O/pmc_cornell_f64 cornell f64
echo exit $?
