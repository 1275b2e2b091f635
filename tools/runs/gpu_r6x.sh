#!/bin/bash
# Round 6: k_attn_bwd_qg occupancy vs its dispatch rounds (10240 waves): hip = 4 waves per SIMD (2.5 rounds),
# qg3 = 3 per SIMD by LDS (3.3 rounds), qg2 = 2 per SIMD (5 rounds exactly); timing only
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6x; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
for i in 1 2 3; do
  for lib in libcsa_qg2.so libcsa_qg3.so libcsa_hip.so; do
    out=$(CSA_HIP_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-bf16-leg --no-side-legs --no-cpu-config1 --no-padded-leg 2>/dev/null) || exit 1
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(sys.argv[2], d['ms_per_step'], {k: round(v, 4) for k, v in d['stage_ms'].items()})" "$out" "$lib"
  done
done 2>&1 | tee $O/ab.txt
# the train legs with and without the side legs run before them (allocator state), one process each
timeout -k 10 600 python bench.py --no-cpu-baseline --no-cpu-config1 --no-bf16-leg --no-side-legs --no-padded-leg > $O/bench_noside.json 2>/dev/null || exit 1
timeout -k 10 900 python bench.py --no-cpu-baseline --no-cpu-config1 --no-bf16-leg --no-padded-leg > $O/bench_side.json 2>/dev/null || exit 1
for f in bench_noside bench_side; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['train']['ms_per_step'], d['train_ddp_world1']['ms_per_step'], d['train_torch_ddp_world1']['ms_per_step'])" $O/$f.json $f; done 2>&1 | tee $O/train_legs.txt
