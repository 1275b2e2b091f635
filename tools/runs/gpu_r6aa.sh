#!/bin/bash
# Round 6: forward online softmax in log2 units (bare exp2) and the accumulator rescale skipped when no running max
# moved (wave ballot); parity tests, then headline A/B against 4ec (the committed tree)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6aa; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for i in 1 2 3 4; do
  for lib in libcsa_4ec.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
