#!/bin/bash
# Round 5: memory-path counters of the headline step (TA busy / stalls, VMEM and LDS instruction counts, LDS FIFO and
# bank stalls, L1->L2 read latency), one rocprofv3 --pmc pass per group, each under its own limit
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5ah; mkdir -p $OUT
CMD="python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-bf16-leg --no-padded-leg --no-cpu-config1"
cd /tmp
i=0
for grp in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 $R/tools/pmc_summary.py $OUT/p*/run_counter_collection.csv > "$OUT/summary.txt"
rm -f $OUT/p*/run_counter_collection.csv.bak
cat "$OUT/summary.txt" | cut -c1-600
