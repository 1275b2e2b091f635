#!/bin/bash
# Round 5, final tree (source hash = the shipped PMC table's): GPU tests, smoke(), then the default bench line, whose
# roofline now reads the matching PMC table (pmc_table_matches_library true)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5af; mkdir -p $O
cd $R
python -c "import sys; sys.path.insert(0,'code-structure-aware-transformer_amd'); from csa_amd.build import source_hash, built_hash; assert source_hash() == built_hash(), 'stale libcsa_hip.so'" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['ms_per_step'], d['step_frac_of_f32_mfma_peak'], d['roofline'].get('pmc_table_matches_library'), d['roofline'].get('traffic'))"
