set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/phase; mkdir -p $O
for c in "bunny_cornell f32" "bunny_cornell f64" "pawn_fog f64" "pawn_fog f32"; do
  RT_AMD_LIB=$PWD/raytrace_amd/_lib/exp/librt_amd_prof.so timeout -k 10 300 python3 tools/phase_prof.py $c 2 >> $O/phase.jsonl 2>> $O/phase.err || { echo "phase $c failed"; tail -5 $O/phase.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/phase.jsonl'):
    d=json.loads(l); r=dict(d); r.pop('raw'); print(json.dumps(r))"
for c in "bunny_cornell f32" "bunny_cornell f64"; do set -- $c
  bash tools/pmc_run.sh $O/pmc_$1_$2 $1 $2 || exit 1
  cat $O/pmc_$1_$2/summary.txt | tail -6
done
