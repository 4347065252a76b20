set -o pipefail
O=gpurun_out/g6; mkdir -p $O; export TMPDIR=/tmp
for cfg in cornell readme demo1 bunny_cornell pawn_fog; do
  for p in f64 f32; do
    bash tools/pmc_run.sh $O/pmc_${cfg}_$p $cfg $p || exit 1
    echo "pmc $cfg $p done"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --steps 10 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err
echo exit $?
