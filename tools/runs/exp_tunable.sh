#!/bin/bash
# A/B: the java train step's hipBLASLt/rocBLAS GEMMs with PyTorch TunableOp (per-shape solution search)
#   base  = default heuristics     tune = TunableOp search (results file written)     use = tuned file, no search
# usage: bash tools/exp_tunable.sh [steps]
set -o pipefail
export TMPDIR=/tmp
S=${1:-30}
OUT=gpurun_out/tunable
mkdir -p $OUT
timeout -k 10 200 python -u tools/prof_train.py $S > $OUT/base.log 2>&1 || exit $?
echo "base: $(tail -1 $OUT/base.log)"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=15 PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results.csv \
  timeout -k 10 700 python -u tools/prof_train.py $S > $OUT/tune.log 2>&1 || exit $?
echo "tune: $(tail -1 $OUT/tune.log)"
ls $OUT
F=$(ls $OUT/tunableop_results*.csv | head -1)
for i in 1 2; do
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$F \
  timeout -k 10 200 python -u tools/prof_train.py $S > $OUT/use$i.log 2>&1 || exit $?
echo "use: $(tail -1 $OUT/use$i.log)"
timeout -k 10 200 python -u tools/prof_train.py $S > $OUT/base$i.log 2>&1 || exit $?
echo "base: $(tail -1 $OUT/base$i.log)"
done
