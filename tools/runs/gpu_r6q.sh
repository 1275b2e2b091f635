#!/bin/bash
# Round 6: per-wave sampled-edge counts (plain stores) summed by k_sparsity_finish instead of a 64-bit atomic per wave;
# parity tests, then headline + padded legs and the n = 32 diagnostic against a3f (the committed tree)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6q; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for lib in libcsa_a3f.so libcsa_hip.so; do
  echo "== $lib"
  DIAG_NS=150,32,150,32 CSA_HIP_LIB=$L/$lib timeout -k 10 300 python tools/runs/diag_dead.py 2>/dev/null || exit 1
done 2>&1 | tee $O/diag.txt
for i in 1 2 3; do
  for lib in libcsa_a3f.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], 'padded', d['padded_mask']['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
