#!/bin/bash
# Round 4: GPU tests on the single-launch in-order projection backward, two bench runs, the headline
# evidence capture (stats + FETCH + WRITE -> pmc table), and the SQ counter passes of the layer bench.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_j.log 2>&1; rc=$?; tail -2 gpurun_out/pt_j.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_j$i.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_j$i.json')); print(d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], {k: round(v,4) for k,v in d['stage_ms'].items()}, d['bf16_mode']['ms_per_step'], d['bwd_schedule'][:40])"
done
bash tools/gpu_capture.sh j || exit $?
PMC_CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-bf16-leg" bash tools/gpu_pmc.sh gpurun_out/pmc_j > /dev/null || exit $?
