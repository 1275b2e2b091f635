#!/bin/bash
# Round 5 first probe: full GPU test suite on the ABI v8 tree; MFMA/VALU overlap probe; removal experiments of
# k_attn_fwd (no Philox / no bit packing / no elementwise / no in-loop DMA / MFMA skeleton) and k_attn_bwd_kv.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
O=$R/gpurun_out/r5a; mkdir -p $O
timeout -k 10 60 ./tools/mfma_valu_probe > $O/probe.txt 2>&1; rc=$?; cat $O/probe.txt | head -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag lib
  CSA_HIP_LIB=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-bf16-leg > $O/bench_$1.json || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$1.json')); print('$1', d['ms_per_step'], {k: round(v,4) for k,v in d['stage_ms'].items()})"
}
for i in 1 2; do
  run base $LIB/libcsa_hip.so || exit 1
  for v in FA FB FC FD FE; do run $v $LIB/libcsa_$v.so || exit 1; done
done
