#!/bin/bash
# Round 5: the bucketed data-parallel reducer against torch DDP and the unwrapped step (world size 1, same box),
# its GPU parity test, the 2-rank gloo-on-one-GPU gradient check for both reducers, kernel stats of the wrapped step.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5j; mkdir -p $O
timeout -k 10 600 python -u tools/ddp_variants.py 2 plain ddp "ddp:impl=torch" > $O/variants.txt 2>&1; rc=$?; grep variant $O/variants.txt; [ $rc -eq 0 ] || { tail -20 $O/variants.txt; exit $rc; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_gpu.py -k ddp > $O/pytest.txt 2>&1; rc=$?; tail -4 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for impl in bucketed torch; do
  CSA_DDP_IMPL=$impl timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/ddp_one_gpu.py > $O/one_gpu_$impl.txt 2>&1; rc=$?; grep test $O/one_gpu_$impl.txt; [ $rc -eq 0 ] || { tail -20 $O/one_gpu_$impl.txt; exit $rc; }
done
cd /tmp
CSA_DDP_PROF=ddp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ddp -o run -- python3 $R/tools/ddp_variants.py > $O/prof_ddp.log 2>&1 || exit 1
find $O -name "*stats*"
