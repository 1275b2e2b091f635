#!/bin/bash
# Round 5: k_rel_prep one 32-row block per workgroup (LDS-staged rows): CSE parity, then cse_bench A/B vs the
# previous tree's library (libcsa_STPH: same CSE code as before the change)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cse_gpu.py > $O/pytest_cse.txt 2>&1; rc=$?; tail -3 $O/pytest_cse.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for lib in libcsa_STPH.so libcsa_hip.so; do echo -n "$lib "; CSA_HIP_LIB=$L/$lib timeout -k 10 120 python tools/cse_bench.py 64 50 in_order || exit 1; done; done 2>&1 | grep CSE | tee $O/ab.txt
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/cse_bench.py 64 20 in_order > $O/trace.log 2>&1 || exit 1
python3 - $O/trace/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us")
PY
rm -f $O/trace/run_kernel_trace.csv
