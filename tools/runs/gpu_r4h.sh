#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_h.log 2>&1; rc=$?; tail -2 gpurun_out/pt_h.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for sch in auto in_order; do
    CSA_BWD_CONCUR=$([ $sch = auto ] && echo "" || echo 0) timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_h.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/bench_h.json')); print('$sch', d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], {k: round(v,4) for k,v in d['stage_ms'].items()}, d['bf16_mode']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
done
