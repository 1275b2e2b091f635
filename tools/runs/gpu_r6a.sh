#!/bin/bash
# Round 6 baseline on the hygiene tree (experiment variants and dead kernels removed): GPU tests, smoke, headline
# bench (no CPU legs) and kernel stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6a; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED|Mismatch" $O/pytest.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cpu-config1 --no-train > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d.get('stage_ms'), d.get('padded_mask',{}).get('ms_per_step'), d.get('bf16_mode',{}).get('ms_per_step'))"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-cpu-config1 --no-train --no-bf16-leg --no-padded-leg > $O/stats.log 2>&1 || exit $?
rm -f $O/stats/run_kernel_trace.csv
head -12 $O/stats/run_kernel_stats.csv | cut -d, -f1-8
