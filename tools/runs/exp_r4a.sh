#!/bin/bash
# Round 4 first probe: multi-block MFMA layout/rate, SBM GPU tests on the mfma4b dQh/dT build, and a
# removal decomposition of the two attention backward kernels (same box, alternating builds).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib
timeout -k 10 60 ./tools/mfma_probe > gpurun_out/mfma_probe.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_sbm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_sbm.log 2>&1; rc=$?; tail -3 gpurun_out/pt_sbm.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_multi.sh 2 $LIB/libcsa_hip.so $LIB/libcsa_NO_MB4.so $LIB/libcsa_NO_LDMA.so $LIB/libcsa_NO_ELEM.so $LIB/libcsa_NO_LDMA_ELEM.so
