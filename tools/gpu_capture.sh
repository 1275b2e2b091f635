#!/bin/bash
# Headline evidence capture (one box): rocprofv3 kernel stats of the layer bench, one FETCH_SIZE pass and one
# WRITE_SIZE pass (separate --pmc runs, MI355X_MICROARCH.md), then the PMC table bench.py ships with
# (csa_amd/pmc_gfx950.json). usage: bash tools/gpu_capture.sh <tag>   (outputs under gpurun_out/cap_<tag>)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
OUT=$R/gpurun_out/cap_$TAG
mkdir -p $OUT
CMD="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $CMD > $OUT/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.log 2>&1 || exit $?
cd $R
H=$(python3 -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash; print(source_hash())")
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv \
  $OUT/stats/run_kernel_stats.csv --source-hash "$H" --cmd "bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg" > $OUT/pmc_gfx950.json || exit $?
python3 - $OUT/pmc_gfx950.json <<'PY'
import json, sys
t = json.load(open(sys.argv[1]))
for n, v in sorted(t["kernels"].items(), key=lambda kv: -(kv[1]["rocprof_avg_ns"] or 0)):
    if v["rocprof_avg_ns"]:
        print(f"{n:22s} {v['rocprof_avg_ns']/1000:8.1f} us  {v['bytes']/1e6:8.1f} MB  {v['bytes']/v['rocprof_avg_ns']:7.1f} GB/s")
PY
