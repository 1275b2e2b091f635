#!/bin/bash
# Round 5: persistent k_attn_fwd_p with deferred queue claims and counted transition waits: SBM GPU tests, same-box
# A/B vs PO (k_attn_fwd) and PP (priority); s_memtime phase stamps of k_attn_fwd (ST) and of its MFMA skeleton
# (STD); MFMA / VALU probe with the s_memtime clock calibration.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5c; mkdir -p $O
timeout -k 10 60 ./tools/mfma_valu_probe > $O/probe.txt 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_property_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2; do
  run tree $LIB/libcsa_hip.so || exit 1
  for v in PO PP; do run $v $LIB/libcsa_$v.so || exit 1; done
done
for v in ST STD; do
  CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/stamps_$v.txt 2>&1 || exit 1
done
grep -c FST $O/stamps_ST.txt
