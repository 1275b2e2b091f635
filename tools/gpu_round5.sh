#!/bin/bash
# Round-5 capture on the final tree: GPU tests, smoke(), the headline evidence (kernel stats + FETCH / WRITE passes
# -> the shipped PMC table csa_amd/pmc_gfx950.json), the SQ counter passes, the default bench line (CPU baselines,
# config 1, padded-mask leg, bf16 leg, train legs with the bucketed reducer and torch DDP beside it), the CSE layer.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${OUT_TAG:-r5}
mkdir -p $OUT
cd $R
python -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash, built_hash; assert source_hash() == built_hash(), 'stale libcsa_hip.so'" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_capture.sh ${CAP_TAG:-r5final} || exit $?
# the box's copy of the tree ships the table just measured for this source hash, so the bench line below reads it
cp $R/gpurun_out/cap_${CAP_TAG:-r5final}/pmc_gfx950.json $R/code-structure-aware-transformer_amd/csa_amd/pmc_gfx950.json || exit 1
PMC_CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-bf16-leg --no-padded-leg --no-cpu-config1" bash tools/gpu_pmc.sh $OUT/pmc > /dev/null || exit $?
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
tail -c 400 $OUT/bench_default.json; echo
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cse -o run -- python3 $R/tools/cse_bench.py 64 20 > $OUT/cse.log 2>&1 || exit $?
rm -f $OUT/*/run_kernel_trace.csv
grep "CSE rel_attn" $OUT/cse.log
echo done
