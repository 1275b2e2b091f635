#!/bin/bash
# Round 5, final tree: BASELINE configs 4 and 5 (tools/config_sweep.sh: headline, dense, N = 1024 at k = 16..128) and
# the bf16 mode's kernel stats, for the round-5 tables
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5al; mkdir -p $OUT
cd $R
bash tools/config_sweep.sh $OUT/sweep > $OUT/sweep.log 2>&1 || { tail -5 $OUT/sweep.log; exit 1; }
cut -c1-160 $OUT/sweep/sweep.jsonl
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bf16 -o run -- python3 $R/bench.py --precision bf16 --steps 20 --warmup 3 --no-padded-leg --no-cpu-baseline --no-train --no-cpu-config1 > $OUT/bf16.log 2>&1 || exit 1
rm -f $OUT/*/run_kernel_trace.csv
python3 - $OUT/bf16/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
