#!/bin/bash
# Round 6: store policies. hip = plain w-tile stores everywhere (one- and two-plane), CSE g tiles non-temporal;
# st4nt = two-plane tiles (dense / map gradients) non-temporal; gt0 = CSE g tiles plain. Dense leg and CSE layer A/B.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6s; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_model_gpu.py tests/test_cse_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for i in 1 2 3; do
  for lib in libcsa_st4nt.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --dense --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('dense', sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab_dense.txt
for i in 1 2 3 4; do
  for lib in libcsa_gt0.so libcsa_hip.so; do
    echo -n "$lib "; CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 40 2>/dev/null | tail -1 || exit 1
  done
done 2>&1 | tee $O/ab_cse.txt
