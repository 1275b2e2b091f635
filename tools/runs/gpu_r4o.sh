#!/bin/bash
# Round 4: GPU tests (CSE logits: two row blocks per wave, buffer stores) and a same-box CSE layer A/B against
# the last commit (CSA_HIP_LIB=libcsa_CSE0.so), three alternating rounds of tools/cse_bench.py 64 20.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
mkdir -p $R/gpurun_out
python -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash, built_hash; assert source_hash() == built_hash(), 'stale libcsa_hip.so'" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_o.log 2>&1; rc=$?; tail -2 gpurun_out/pt_o.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in hip CSE0; do
    echo -n "cse $v: "; CSA_HIP_LIB=$LIB/libcsa_$v.so timeout -k 10 120 python tools/cse_bench.py 64 20 2>&1 | tail -1 || exit 1
  done
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cse_prof5 -o run -- python3 $R/tools/cse_bench.py 64 20 > $R/gpurun_out/cse_prof5.log 2>&1 || exit $?
python3 - $R/gpurun_out/cse_prof5/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
