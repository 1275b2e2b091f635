#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_f.log 2>&1; rc=$?; tail -2 gpurun_out/pt_f.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_f$i.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_f$i.json')); print(d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], d['stage_ms'], d['bf16_mode']['ms_per_step'])"
done
bash tools/gpu_capture.sh f
