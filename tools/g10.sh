set -o pipefail
O=gpurun_out/g10; mkdir -p $O; export TMPDIR=/tmp
export RT_AMD_LIB=$PWD/raytrace_amd/_lib/exp/librt_amd_prof.so
for c in bunny_cornell demo1; do for p in f32; do
  timeout -k 10 120 python3 -u tools/phase_prof.py $c $p 3 >> $O/phase.jsonl 2>> $O/phase.err || exit 1
done; done
echo done
