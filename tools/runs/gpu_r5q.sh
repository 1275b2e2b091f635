#!/bin/bash
# Round 5: CSE backward over two (b,h) halves on two streams (auto/concurrent) vs in order: parity, then cse_bench A/B
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5q; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cse_gpu.py > $O/pytest_cse.txt 2>&1; rc=$?; tail -3 $O/pytest_cse.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for s in in_order auto; do timeout -k 10 120 python tools/cse_bench.py 64 50 $s || exit 1; done; done 2>&1 | grep CSE | tee $O/ab.txt
