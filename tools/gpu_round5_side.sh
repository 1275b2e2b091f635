#!/bin/bash
# Round-5 side captures (one box): the dense FullAttention ablation (config 4: bench line, kernel stats, SQ / traffic
# counter passes), the bf16 mode (bench line, kernel stats), the CSE layer and the java train step kernel stats.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5side
mkdir -p $OUT
cd $R
NB="--no-cpu-baseline --no-train --no-cpu-config1"
timeout -k 10 300 python bench.py --dense $NB > $OUT/bench_dense.json 2> $OUT/bench_dense.err || { tail -5 $OUT/bench_dense.err; exit 1; }
tail -c 600 $OUT/bench_dense.json; echo
timeout -k 10 300 python bench.py --precision bf16 $NB > $OUT/bench_bf16.json 2> $OUT/bench_bf16.err || { tail -5 $OUT/bench_bf16.err; exit 1; }
tail -c 300 $OUT/bench_bf16.json; echo
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dense -o run -- python3 $R/bench.py --dense --steps 20 --warmup 3 $NB > $OUT/dense.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bf16 -o run -- python3 $R/bench.py --precision bf16 --steps 20 --warmup 3 --no-padded-leg $NB > $OUT/bf16.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/train -o run -- python3 $R/tools/prof_train.py 5 > $OUT/train.log 2>&1 || exit 1
cd $R
PMC_CMD="python3 $R/bench.py --dense --steps 2 --warmup 1 $NB" bash tools/gpu_pmc.sh $OUT/pmc_dense > /dev/null || exit 1
rm -f $OUT/*/run_kernel_trace.csv
for d in dense bf16; do echo "== $d"; python3 - $OUT/$d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
grep -E "k_attn" $OUT/pmc_dense/summary.txt | cut -c1-300
