#!/bin/bash
# Round 6: bench.py with the new side legs (CSE java layer, dense config 4, long-AST config 5) beside the headline
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6b; mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cpu-config1 --no-train > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["value"], d["ms_per_step"], d["step_frac_of_f32_mfma_peak"])
for k in ("cse", "dense"):
    print(k, json.dumps({a: d[k][a] for a in d[k] if a != "stage_ms"}))
for k, v in d["long_ast"].items():
    print(k, v if isinstance(v, str) else json.dumps({a: v[a] for a in v if a != "stage_ms"}))
PY
