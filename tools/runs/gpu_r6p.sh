#!/bin/bash
# Round 6: does the forward's per-wave sparsity atomic (10240 adds on 8 counters of one cache line) cost time?
# noatom = no atomic (timing only); equal-length padding n = 150 / 32 twice, then the headline A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6p; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
for lib in libcsa_noatom.so libcsa_hip.so; do
  echo "== $lib"
  DIAG_NS=150,32,150,32 CSA_HIP_LIB=$L/$lib timeout -k 10 300 python tools/runs/diag_dead.py 2>/dev/null || exit 1
done 2>&1 | tee $O/diag.txt
for i in 1 2 3; do
  for lib in libcsa_noatom.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
