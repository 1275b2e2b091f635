#!/bin/bash
# GPU session: every -m gpu test (one process), smoke, and one short bench line. Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/t}
TESTS=${2:-tests}
BENCH_ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3 --no-cpu-baseline"}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR" "$OUT/pytest.log" | tail -5; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
