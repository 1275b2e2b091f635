export TMPDIR=/tmp
O=gpurun_out/lg
mkdir -p $O
for i in 1 2 3; do
for v in ${VARIANTS:-csa_lgsh csa_hip}; do
  CSA_HIP_LIB=$PWD/code-structure-aware-transformer_amd/csa_amd/lib/lib$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v$i -o run -- python tools/cse_bench.py 64 20 > $O/$v$i.log 2>&1 || exit $?
  python3 - $O/$v$i/run_kernel_stats.csv $v $O/$v$i.log <<'PY'
import csv, sys
st={r['Name'][22:40]: round(float(r['AverageNs'])/1e3,1) for r in csv.DictReader(open(sys.argv[1])) if 'rel' in r['Name'] or 'split' in r['Name']}
print(sys.argv[2], [l.strip() for l in open(sys.argv[3]) if 'CSE' in l][-1:], st)
PY
done
done
