#!/bin/bash
# Round 6: bf16 mode with the tile handoff (k_attn_bwd_kv -> k_attn_bwd_qg, plain stores) instead of the recomputing
# query kernel: bfho = handoff (timing + bf16 parity tests), hip = shipped (k_attn_bwd_qr)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6z; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
CSA_HIP_LIB=$L/libcsa_bfho.so timeout -k 10 600 python -u -m pytest tests/test_bf16_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for i in 1 2 3; do
  for lib in libcsa_bfho.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --precision bf16 --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
