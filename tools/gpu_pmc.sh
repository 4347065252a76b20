#!/bin/bash
# PMC passes (one counter group per pass, --kernel-trace only) for the render kernel.
# usage: bash tools/gpu_pmc.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift
ARGS=${*:-"--steps 3 --warmup 1 --warmup-s 0 --no-cpu-baseline"}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -n "$LIST" ]; then rocprofv3 -L > "$OUT/counters_list.txt" 2>&1; fi
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_FLAT SQ_INSTS_GDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_IFETCH SQ_WAIT_INST_VMEM SQ_INSTS_SMEM_NORM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pass $i failed"; tail -5 "$OUT/p$i.err"; }
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/summary.txt"
