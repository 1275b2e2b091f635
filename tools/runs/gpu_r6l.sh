#!/bin/bash
# Round 6: k_attn_bwd_kv's dead key blocks fetch their query blocks' Qh images and bit words in one chunk (no round
# trip per query block); parity tests, then the equal-length padding diagnostic for 8b5 (previous) and hip
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6l; mkdir -p $O
L=$R/code-structure-aware-transformer_amd/csa_amd/lib
cd $R
timeout -k 10 600 python -u -m pytest tests/test_sbm_gpu.py -q -k "dead or padded or mask or shapes" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "^E  +|FAILED" $O/pytest.txt | head -40; exit $rc; }
for lib in libcsa_8b5.so libcsa_hip.so; do
  echo "== $lib"
  CSA_HIP_LIB=$L/$lib timeout -k 10 300 python tools/runs/diag_dead.py 2>/dev/null || exit 1
done 2>&1 | tee $O/diag.txt
