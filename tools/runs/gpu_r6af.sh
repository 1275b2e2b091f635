#!/bin/bash
# Round 6: k_attn_bwd_qg walks its (b,h) blocks in the reverse of k_attn_bwd_kv's order inside each XCD (the tiles kv
# wrote last are still in that XCD's L2): qgrev vs hip (shipped), headline, 4 rounds
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6af; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
CSA_HIP_LIB=$L/libcsa_qgrev.so timeout -k 10 300 python -u -m pytest tests/test_sbm_gpu.py -q -k "oracle or golden" --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4; do
  for lib in libcsa_qgrev.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
