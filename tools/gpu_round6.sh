#!/bin/bash
# Round-6 capture on the final tree: GPU tests, smoke(), the headline evidence (kernel stats + FETCH / WRITE passes ->
# the shipped PMC table csa_amd/pmc_gfx950.json, now with the side legs' rocprof kernel stats: CSE java layer, dense
# config 4, long-AST config 5 k = 16..128), the SQ counter passes, the default bench line, CSE kernel stats.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${CAP_TAG:-r6final}
OUT=$R/gpurun_out/${OUT_TAG:-r6}
CAP=$R/gpurun_out/cap_$TAG
mkdir -p $OUT $CAP
cd $R
python -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash, built_hash; assert source_hash() == built_hash(), 'stale libcsa_hip.so'" || exit 1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
HEAD="--no-cpu-baseline --no-cpu-config1 --no-train --no-bf16-leg --no-side-legs"
CMD="python3 $R/bench.py --steps 10 --warmup 2 $HEAD"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $CAP/stats -o run -- $CMD > $CAP/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $CAP/fetch -o run -- $CMD > $CAP/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $CAP/write -o run -- $CMD > $CAP/write.log 2>&1 || exit $?
LEGS=""
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $CAP/leg_cse -o run -- python3 $R/tools/cse_bench.py 64 20 > $CAP/leg_cse.log 2>&1 || exit $?
LEGS="$LEGS --leg cse=$CAP/leg_cse/run_kernel_stats.csv"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $CAP/leg_dense -o run -- python3 $R/bench.py --dense --steps 10 --warmup 2 $HEAD --no-padded-leg > $CAP/leg_dense.log 2>&1 || exit $?
LEGS="$LEGS --leg dense=$CAP/leg_dense/run_kernel_stats.csv"
for K in 16 32 64 128; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $CAP/leg_long_k$K -o run -- python3 $R/bench.py --seq-len 1024 --clusters $K --batch 16 --steps 5 --warmup 2 $HEAD > $CAP/leg_long_k$K.log 2>&1 || exit $?
  LEGS="$LEGS --leg long_k$K=$CAP/leg_long_k$K/run_kernel_stats.csv"
done
rm -f $CAP/*/run_kernel_trace.csv
cd $R
H=$(python3 -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash; print(source_hash())")
python3 tools/pmc_traffic.py $CAP/fetch/run_counter_collection.csv $CAP/write/run_counter_collection.csv \
  $CAP/stats/run_kernel_stats.csv --source-hash "$H" --cmd "bench.py --steps 10 --warmup 2 $HEAD" $LEGS > $CAP/pmc_gfx950.json || exit $?
cp $CAP/pmc_gfx950.json $R/code-structure-aware-transformer_amd/csa_amd/pmc_gfx950.json || exit 1
PMC_CMD="python bench.py --steps 2 --warmup 1 $HEAD --no-padded-leg" bash tools/gpu_pmc.sh $OUT/pmc > /dev/null || exit $?
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
tail -c 600 $OUT/bench_default.json; echo
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cse -o run -- python3 $R/tools/cse_bench.py 64 20 > $OUT/cse.log 2>&1 || exit $?
rm -f $OUT/*/run_kernel_trace.csv
grep "CSE rel_attn" $OUT/cse.log
echo done
