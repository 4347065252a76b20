#!/bin/bash
# One GPU session, every measurement the rounds take as a named step (replaces the one-off session
# scripts of rounds 2-3).  From the repo root, on the GPU box:
#   bash tools/gpu_round.sh <tag> [step ...]        (default steps: tests bench prof)
# Steps:
#   tests      every -m gpu test (one process)
#   bench      the headline bench line (binary64 + FP32 record), 20 frames
#   benchall   a bench line for every other config (CONFIGS), 5 frames
#   summary    one line per bench_*.json of this tag: Msamples/s, ms per frame, f32 record
#   prof       rocprofv3 --kernel-trace --stats of the headline, default two streams
#   prof1      the same on one stream (per-launch durations without overlap)
#   traffic    FETCH_SIZE / WRITE_SIZE passes of their own (one stream) for CPS="<config>:<prec> ..."
#              with the in-tree build and each raytrace_amd/_lib/exp/*.so
#   pmcvalu    tools/pmc_run.sh passes (mix, wave states, traffic) for CONFIGS x PRECS, folded into
#              profiles/pmc_valu.json
#   ab         tools/ab_libs.sh over AB_CFGS ("<config>:<sim-shards> ...") in PRECS, REPS repetitions
#   image      tools/image_ab.py: images of each exp lib against the in-tree build, bit for bit
#   phase      phase profile (needs raytrace_amd/_lib/diag/librt_amd_prof.so, -DRT_PHASE_PROF)
#   microbench VALU rate / binary64 math microbenchmarks, built from source here
#   rehearse   bench.py --gpus 2 / 3 on one GPU, frames bit-identical to N = 1
#   shards     tools/shard_share_sweep.sh: one rank's share of an N-GPU frame, N = 1, 2, 4, 8
#   abiprobe   tools/abi_probe.py: the C-ABI device lists [0] x 1..3 in a process of their own
#   abiprobe2  tools/abi_probe2.py: [0, 0] after torch / distributed set-up / under torchrun
#   demo2fit   tools/demo2_fit.py: demo2 at 800 x 800 against the published demo2.png (depth sweep,
#              renders for the spp estimate)
# Env: CONFIGS, PRECS, CPS, AB_CFGS, REPS, PROF_STEPS, PYTEST_K, ROUND.  Each GPU step runs under
# a timeout of its own and the session stops at the first failing step.
export RT_AMD_EXPERIMENTS=1  # the library reads RT_AMD_* knobs / RT_AMD_LIB only with this set
set -o pipefail
TAG=${1:-r3}
shift
STEPS=${*:-"tests bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ALL_CONFIGS="readme demo1 demo1_1200x800 bunny_cornell pawn_fog"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -20; exit 1; }
      tail -1 "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_cornell.json" 2> "$OUT/bench_cornell.err" || { echo "bench failed"; tail -5 "$OUT/bench_cornell.err"; exit 1; } ;;
    benchall)
      for c in ${CONFIGS:-$ALL_CONFIGS}; do
        timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_$c.json" 2>> "$OUT/bench_other.err" || { echo "bench $c failed"; exit 1; }
      done ;;
    summary)
      for f in "$OUT"/bench_*.json; do python3 - "$f" <<'PY'
import json, os, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); f = d.get("f32_fast_path", {})
print(os.path.basename(sys.argv[1])[6:-5], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], "f32", f.get("value"), f.get("ms_per_step"))
PY
      done ;;
    prof|prof1)
      extra=""; [ $s = prof1 ] && extra="--streams 1"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$s" -o run -- \
        python3 bench.py --steps ${PROF_STEPS:-20} --warmup 5 --no-cpu-baseline $extra > "$OUT/${s}_bench.json" 2> "$OUT/$s.err" || { echo "rocprof $s failed"; tail -20 "$OUT/$s.err"; exit 1; }
      grep -h "render_kernel\|resolve" "$OUT"/$s/*kernel_stats.csv | cut -c1-160 ;;
    traffic)
      for cp in ${CPS:-cornell:f64}; do
        c=${cp%%:*}; p=${cp#*:}
        for lib in "" raytrace_amd/_lib/exp/*.so; do
          if [ -n "$lib" ]; then [ -e "$lib" ] || continue; export RT_AMD_LIB=$PWD/$lib; nm=$(basename $lib .so); else unset RT_AMD_LIB; nm=intree; fi
          for ctr in FETCH_SIZE WRITE_SIZE; do
            d=$OUT/${c}_${p}_${nm}_$ctr
            timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $d -o run -- \
              python3 bench.py --config $c --precision $p --no-f32 --steps 3 --warmup 1 --warmup-s 0 --no-cpu-baseline --streams 1 --plan overlapped \
              > $d.json 2> $d.err || { echo "pass $c $p $nm $ctr failed"; tail -3 $d.err; exit 1; }
            python3 - "$d" "$c $p $nm $ctr" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "rt_render_kernel" in r["Kernel_Name"]]
print(sys.argv[2], "per launch (KB as reported):", sum(v) / max(1, len(v)), "launches", len(v))
PY
          done
        done
      done
      unset RT_AMD_LIB ;;
    pmcvalu)
      for c in ${CONFIGS:-cornell}; do
        for p in ${PRECS:-f64 f32}; do
          bash tools/pmc_run.sh "$OUT/pmc_${c}_$p" $c $p || exit 1
          python3 tools/pmc_fold.py "$OUT/pmc_${c}_$p" $c $p ${ROUND:-r3} || exit 1
        done
      done
      cp profiles/pmc_valu.json "$OUT/pmc_valu.json" ;;
    ab)
      for p in ${PRECS:-f64 f32}; do
        PREC=$p REPS=${REPS:-2} bash tools/ab_libs.sh "$TAG/ab_$p" "${AB_CFGS:-bunny_cornell:1 demo1:1 pawn_fog:1}" ${AB_STEPS:-4} || exit 1
      done ;;
    image)
      for lib in raytrace_amd/_lib/exp/*.so; do
        [ -e "$lib" ] || continue
        nm=$(basename $lib .so)
        timeout -k 10 400 python3 tools/image_ab.py $lib $OUT/image_ab_$nm.json > $OUT/image_ab_$nm.log 2>&1 || { echo "image_ab $nm failed"; tail -20 $OUT/image_ab_$nm.log; exit 1; }
        echo "$nm: $(grep -c "'bit_identical': True" $OUT/image_ab_$nm.log) bit-identical of $(grep -c bit_identical $OUT/image_ab_$nm.log)"
      done ;;
    stamps)  # needs raytrace_amd/_lib/diag/librt_amd_stamps.so (-DRT_WAVE_STAMPS)
      for c in ${STAMP_CPS:-cornell:f64 cornell:f32}; do
        RT_AMD_LIB=$PWD/raytrace_amd/_lib/diag/librt_amd_stamps.so timeout -k 10 200 python3 tools/wave_stamps.py ${c%%:*} ${c#*:} 5 >> $OUT/stamps.jsonl 2>> $OUT/stamps.err || { echo "stamps $c failed"; tail -5 $OUT/stamps.err; exit 1; }
      done
      python3 -c "import json,sys; [print(d['config'], d['precision'], d['median'], d['per_frame'][0]['ramp_ms'], d['per_frame'][0]['end_ms'], d['per_frame'][0]['alive_by_tenth']) for d in map(json.loads, open(sys.argv[1]))]" $OUT/stamps.jsonl ;;
    phase)
      for c in ${PHASE_CPS:-bunny_cornell:f32 bunny_cornell:f64 pawn_fog:f64 pawn_fog:f32}; do
        RT_AMD_LIB=$PWD/raytrace_amd/_lib/diag/librt_amd_prof.so timeout -k 10 300 python3 tools/phase_prof.py ${c%%:*} ${c#*:} 2 >> $OUT/phase.jsonl 2>> $OUT/phase.err || { echo "phase $c failed"; tail -5 $OUT/phase.err; exit 1; }
      done ;;
    microbench)  # built from source here, never a committed binary
      make -C tools/microbench all > "$OUT/microbench_build.log" 2>&1 || { echo "microbench build failed"; exit 1; }
      timeout -k 10 120 tools/microbench/valu_rates > "$OUT/valu_rates.json" || exit 1
      timeout -k 10 120 tools/microbench/f64_math_check > "$OUT/f64_math_check.json" || exit 1 ;;
    rehearse)
      bash tools/rehearse_dist.sh "$TAG/rehearse" || exit 1 ;;
    shards)
      bash tools/shard_share_sweep.sh "$TAG/shards" > "$OUT/shards.log" 2>&1 || { echo "shard sweep failed"; tail -5 "$OUT/shards.log"; exit 1; }
      cat "$OUT/shards.log" ;;
    abiprobe)
      timeout -k 10 300 python3 -u tools/abi_probe.py ${ABI_CFG:-cornell} 20 > "$OUT/abi_probe.jsonl" 2> "$OUT/abi_probe.err" || { echo "abi_probe failed"; tail -20 "$OUT/abi_probe.err"; exit 1; }
      python3 -c "import json,sys; [print(d['devices'], d['ms_per_frame'], d['kernel_ms_max_device'], d['sha16'], d['calls'][-1]) for d in map(json.loads, open(sys.argv[1]))]" "$OUT/abi_probe.jsonl" ;;
    abiprobe2)
      for m in ${ABI_MODES:-plain torch torch_tensors dist}; do
        timeout -k 10 200 python3 -u tools/abi_probe2.py $m >> "$OUT/abi_probe2.jsonl" 2>> "$OUT/abi_probe2.err" || { echo "abi_probe2 $m failed"; tail -5 "$OUT/abi_probe2.err"; exit 1; }
      done
      timeout -k 10 200 python3 -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 tools/abi_probe2.py plain \
        | sed 's/"plain"/"torchrun_plain"/' >> "$OUT/abi_probe2.jsonl" 2>> "$OUT/abi_probe2.err" || { echo "abi_probe2 torchrun failed"; tail -5 "$OUT/abi_probe2.err"; exit 1; }
      cat "$OUT/abi_probe2.jsonl" ;;
    demo2fit)
      timeout -k 10 600 python3 -u tools/demo2_fit.py "$OUT/demo2_fit.jsonl" > "$OUT/demo2_fit.log" 2>&1 || { echo "demo2_fit failed"; tail -20 "$OUT/demo2_fit.log"; exit 1; } ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
