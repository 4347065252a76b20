#!/bin/bash
# PMC passes of the render kernel for one (config, precision): instruction mix, wave states,
# lane utilisation, and HBM traffic (FETCH_SIZE / WRITE_SIZE in passes of their own), each pass
# `rocprofv3 --pmc ... --kernel-trace` only, one stream, 3 timed frames.
# usage: bash tools/pmc_run.sh <outdir> <config> <precision>     env: PASSES="1 2 3" (a subset of
# the six passes below; default all), RT_AMD_LIB + RT_AMD_EXPERIMENTS=1 for an experiment build
set -o pipefail
OUT=$1; CFG=${2:-cornell}; PREC=${3:-f64}
mkdir -p "$OUT"; export TMPDIR=/tmp
ARGS="--config $CFG --precision $PREC --no-f32 --steps 3 --warmup 1 --warmup-s 0 --no-cpu-baseline --streams 1 --plan overlapped"
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4 5 6} " in *" $i "*) ;; *) continue ;; esac
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pmc pass $i failed"; tail -3 "$OUT/p$i.err"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
