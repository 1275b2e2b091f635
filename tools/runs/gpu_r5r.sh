#!/bin/bash
# Round 5: CSE layer kernel stats on the current tree (tools/cse_bench.py 64, in order)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5r; mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/cse_bench.py 64 20 in_order > $O/trace.log 2>&1 || exit 1
grep CSE $O/trace.log
python3 - $O/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
rm -f $O/trace/run_kernel_trace.csv
