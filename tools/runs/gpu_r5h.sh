#!/bin/bash
# Round 5: static persistent forward (k_attn_fwd_s: 8 independent waves per workgroup, 5 items each) with start
# staggers 0 / 3 / 5 x s_sleep(127) for waves 4..7, same box, against OLD and R4.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5h; mkdir -p $O
CSA_HIP_LIB=$LIB/libcsa_S5.so timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_S5.log 2>&1; rc=$?; tail -2 $O/pytest_S5.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2 3; do
  for v in OLD S0 S3 S5; do run $v $LIB/libcsa_$v.so || exit 1; done
done
