#!/bin/bash
# GEMM table on the box: with "retune", rebuild csa_amd/gemm_tuned_gfx950.csv first (copied back under
# gpurun_out/tune/); then the model GPU tests (incl. the tuned-table test), the train legs of bench.py and
# the CSE layer bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/tune
mkdir -p $OUT
T=code-structure-aware-transformer_amd/csa_amd/gemm_tuned_gfx950.csv
if [ "$1" = retune ]; then
  timeout -k 10 400 python -u tools/tune_gemms.py $T > $OUT/tune.log 2>&1 || exit $?
  tail -1 $OUT/tune.log; cp $T $OUT/
fi
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -m gpu -x -v -s --timeout 200 --timeout-method thread \
  > $OUT/pytest_model.log 2>&1; rc=$?; grep -E "worst|passed|failed|Error" $OUT/pytest_model.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bf16-leg > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('train','train_ddp_world1','train_default_gemms','config1_gpu')})"
timeout -k 10 120 python -u tools/cse_bench.py 64 50 > $OUT/cse.log 2>&1 || exit $?
tail -1 $OUT/cse.log
