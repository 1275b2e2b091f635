#!/bin/bash
# Round 5: DDP wrapper cost at world size 1: same-box ms/step of the java train step under the
# wrap_ddp switches, then rocprofv3 kernel stats of the plain and the DDP-wrapped step (10 warm-up + 30 steps each).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5i; mkdir -p $O
timeout -k 10 600 python -u tools/ddp_variants.py 2 plain ddp "ddp:broadcast_buffers=0" "ddp:static_graph=1" "ddp:comm_hook=world1_none" "ddp:broadcast_buffers=0,static_graph=1" > $O/variants.txt 2>&1; rc=$?; grep variant $O/variants.txt; [ $rc -eq 0 ] || { tail -20 $O/variants.txt; exit $rc; }
cd /tmp
for v in plain ddp; do
  CSA_DDP_PROF=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 $R/tools/ddp_variants.py > $O/prof_$v.log 2>&1 || exit 1
done
ls -R $O | head -30
