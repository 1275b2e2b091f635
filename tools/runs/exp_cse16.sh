#!/bin/bash
# CSE 16-row backward: parity tests on the shipped build, then alternating CSE layer timings of
#   new = k_rel_bwd_qh / kh (16-row waves)   old = k_rel_bwd_qf / kf (CSA_EXP_REL32 build)
# and a rocprofv3 kernel-stats pass of the new build. usage: bash tools/exp_cse16.sh [rounds]
set -o pipefail
export TMPDIR=/tmp
R=${1:-3}
OUT=gpurun_out/cse16
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_cse_gpu.py tests/test_property_gpu.py tests/test_model_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 "$R"); do
  echo "new $(timeout -k 10 120 python tools/cse_bench.py 64 50 | tail -1)" || exit 1
  echo "old $(CSA_HIP_LIB=$LIB/libcsa_exp_REL32.so timeout -k 10 120 python tools/cse_bench.py 64 50 | tail -1)" || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python tools/cse_bench.py 64 20 > $OUT/trace.log 2>&1 || exit $?
python3 - $OUT/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
