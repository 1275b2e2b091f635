#!/bin/bash
# Round 5: LDS fragment lookahead pinned in the projection forward (parity + same-box A/B against the sunk schedule),
# then the bucket-ready timeline and one default bench.py run.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5l; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sbm_gpu.py > $O/pytest_sbm.txt 2>&1; rc=$?; tail -3 $O/pytest_sbm.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh $L/libcsa_SINK.so $L/libcsa_hip.so 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ddp_timeline.py 16 32 64 128 > $O/timeline.txt 2>&1; rc=$?; tail -c 2500 $O/timeline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 1500 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
