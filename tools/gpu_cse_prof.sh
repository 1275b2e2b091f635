#!/bin/bash
# CSE layer (java dims, B=64) profile with the in-order backward schedule: kernel stats + PMC passes.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/cse_prof}
mkdir -p "$OUT"
export CSA_BWD_CONCUR=0
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python tools/cse_bench.py 64 20 > "$OUT/trace.log" 2>&1 || exit $?
grep "CSE rel_attn" "$OUT/trace.log"
python3 - $OUT/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
PMC_CMD="python tools/cse_bench.py 64 3" EXTRA_PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS" bash tools/gpu_pmc.sh "$OUT/pmc" | grep -E "k_rel_(bwd|fwd)"
