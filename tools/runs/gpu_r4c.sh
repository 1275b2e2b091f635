#!/bin/bash
# Round 4: kernel trace of the layer bench (+ a no-ds/G-store variant) and PMC passes on the new backward.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
LIB=$R/code-structure-aware-transformer_amd/csa_amd/lib
B="--steps 10 --warmup 2 --no-cpu-baseline --no-train --no-bf16-leg"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c -o run -- python3 $R/bench.py $B > $R/gpurun_out/prof_c.log 2>&1 || exit $?
CSA_HIP_LIB=$LIB/libcsa_NO_DSG.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c_nodsg -o run -- python3 $R/bench.py $B > $R/gpurun_out/prof_c2.log 2>&1 || exit $?
cd $R
PMC_CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-train --no-bf16-leg" bash tools/gpu_pmc.sh gpurun_out/pmc_c > /dev/null 2>&1 || exit $?
for f in gpurun_out/prof_c/run_kernel_stats.csv gpurun_out/prof_c_nodsg/run_kernel_stats.csv; do echo $f; head -14 $f | cut -d, -f1-4 | sed 's/(anonymous namespace):://g' | cut -c1-140; done
grep "k_attn\|k_proj" gpurun_out/pmc_c/summary.txt | cut -c1-400
