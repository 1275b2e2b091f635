#!/bin/bash
# Round 6: does the dead-tile bookkeeping cost the unpadded forward? nodead = this tree with the forward's dead-tile
# order forced off (timing only); then the CSE java layer's kernel split and counters
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6i; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
for i in 1 2 3; do
  for lib in libcsa_fwdv.so libcsa_nodead.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
bash tools/gpu_cse_prof.sh $O/cse > $O/cse.txt 2>&1; rc=$?; cat $O/cse.txt; exit $rc
