#!/bin/bash
# Round 5: bucket-ready timeline of the java train step (tools/ddp_timeline.py, caps 16/32/64/128 MB) and one default
# bench.py run (bucketed world-1 leg, padded-mask leg).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5k; mkdir -p $O
timeout -k 10 400 python -u tools/ddp_timeline.py 16 32 64 128 > $O/timeline.txt 2>&1; rc=$?; tail -c 3000 $O/timeline.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 1500 $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
