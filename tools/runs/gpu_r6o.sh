#!/bin/bash
# Round 6: the forward runs its dead tiles after the live loop, their T images in chunks (one wait per chunk), no
# dropout bits; parity tests, the equal-length padding diagnostic and the headline / padded legs against r6n
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6o; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py tests/test_model_gpu.py tests/test_bf16_gpu.py -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for lib in libcsa_r6n.so libcsa_hip.so; do
  echo "== $lib"
  DIAG_NS=150,96,64,32 CSA_HIP_LIB=$L/$lib timeout -k 10 300 python tools/runs/diag_dead.py 2>/dev/null || exit 1
done 2>&1 | tee $O/diag.txt
for i in 1 2 3; do
  for lib in libcsa_r6n.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], 'padded', d['padded_mask']['ms_per_step'] if 'ms_per_step' in d['padded_mask'] else d['padded_mask'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
