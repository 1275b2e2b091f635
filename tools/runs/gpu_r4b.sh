#!/bin/bash
# Round 4: full GPU test suite + headline bench (layer only) + rocprof kernel stats of the layer bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_all.log 2>&1; rc=$?
tail -5 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_l$i.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_l$i.json')); print(d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], d['stage_ms'], d['bf16_mode']['ms_per_step'])"
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg > /dev/null 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/prof_b -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $GRAFT_REPO_ROOT/gpurun_out/kstats_b.csv
head -12 $GRAFT_REPO_ROOT/gpurun_out/kstats_b.csv | cut -d, -f1-4
