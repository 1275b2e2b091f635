#!/bin/bash
# PMC passes over a short bench run (one pass per counter group; each pass under its own time limit).
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
CMD=${PMC_CMD:-"python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train"}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" \
           "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python tools/pmc_summary.py $OUT/p*/run_counter_collection.csv > "$OUT/summary.txt"
cat "$OUT/summary.txt"
