#!/bin/bash
# Round 5: sparsity formed by k_attn_fwd's last wave (no k_sparsity_finish launch): full GPU tests, 3 bench runs
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-train --no-cpu-config1 --no-padded-leg --no-bf16-leg > $O/b$i.json 2>/dev/null || exit 1; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['stage_ms'])" $O/b$i.json; done
