#!/bin/bash
# Round 4: SBM/bf16/model GPU tests + layer bench x2 + kernel trace.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_e.log 2>&1; rc=$?; tail -2 gpurun_out/pt_e.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_e$i.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_e$i.json')); print(d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], d['stage_ms'], d['bf16_mode']['ms_per_step'])"
done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg > $R/gpurun_out/prof_e.log 2>&1 || exit $?
