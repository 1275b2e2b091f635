#!/bin/bash
# Round 4: GPU tests; same-box A/B of the concurrent projection backward (auto vs in_order) and of the 24-bit
# RNG cost (RNG24C: two extra Philox calls per attention tile, half a call per 8 proj-dropout draws);
# the one-GPU two-rank DDP semantics check.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_i.log 2>&1; rc=$?; tail -2 gpurun_out/pt_i.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib concur
  CSA_HIP_LIB=$2 CSA_BWD_CONCUR=$3 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 > gpurun_out/bench_i.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bench_i.json')); print('$1', d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], {k: round(v,4) for k,v in d['stage_ms'].items()}, d['bf16_mode']['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['bwd_schedule'][:40])"
}
for i in 1 2; do
  run auto $LIB/libcsa_hip.so "" || exit 1
  run in_order $LIB/libcsa_hip.so 0 || exit 1
  run rng24c $LIB/libcsa_RNG24C.so "" || exit 1
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/ddp_one_gpu.py 8 > gpurun_out/ddp_one_gpu.log 2>&1; rc=$?; grep '^{' gpurun_out/ddp_one_gpu.log; echo "ddp rc=$rc"
# CSE: the g-tile handoff vs the recomputing query kernel (java layer shape, B=64), same box, alternating
for i in 1 2 3; do
  for v in hip RELRECOMP; do
    echo -n "cse $v: "; CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python tools/cse_bench.py 64 20 2>&1 | tail -1 || exit 1
  done
done
