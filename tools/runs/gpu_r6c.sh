#!/bin/bash
# Round 6: k_attn_bwd_kv forms the row constants itself (gamma from the dX image and the lane's X row; no
# k_attn_rowprep launch): GPU tests, then a same-box A/B against the round-start tree (base) and a no-SLP build,
# then bench.py with the side legs
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6c; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch|assert" $O/pytest.txt | head -30; exit $rc; }
bash tools/ab3.sh 3 $L/libcsa_base.so $L/libcsa_hip.so $L/libcsa_noslp.so 2>&1 | tee $O/ab.txt || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cpu-config1 --no-train > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["ms_per_step"], d["step_frac_of_f32_mfma_peak"], d.get("padded_mask", {}).get("ms_per_step"), d.get("bf16_mode", {}).get("ms_per_step"))
for k in ("cse", "dense"):
    print(k, json.dumps({a: d[k][a] for a in d[k] if a != "stage_ms"}))
for k, v in d["long_ast"].items():
    print(k, v if isinstance(v, str) else json.dumps({a: v[a] for a in v if a != "stage_ms"}))
PY
