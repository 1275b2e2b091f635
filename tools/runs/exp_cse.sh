export TMPDIR=/tmp
mkdir -p gpurun_out/t6
for v in csa_hip csa_exp_NOSCATTER csa_exp_NOBT; do
  CSA_HIP_LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t6/$v -o run -- python tools/cse_bench.py 64 10 > gpurun_out/t6/$v.log 2>&1 || exit $?
  python3 - gpurun_out/t6/$v/run_kernel_stats.csv $v <<'PY'
import csv, sys
print(sys.argv[2], {r['Name'][30:50]: round(float(r['AverageNs'])/1e3,1) for r in csv.DictReader(open(sys.argv[1])) if 'rel' in r['Name'] or 'bgemm' in r['Name']})
PY
done
