#!/bin/bash
# Round 6: the forward's live tiles sampled before the softmax again (whole-tile compares, pack_bits), as at the
# round start; d24 = the committed tree (sampling after the softmax in two groups), fwdv = no dead-tile loop
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6j; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_bf16_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for i in 1 2 3; do
  for lib in libcsa_fwdv.so libcsa_d24.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
for lib in libcsa_d24.so libcsa_hip.so libcsa_d24.so libcsa_hip.so; do
  out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --padded --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('padded', sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
done 2>&1 | tee $O/ab_padded.txt
