set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_check.sh || exit 1
for n in 95000 6900000; do
  for nt in 1 2; do
    rm -rf gpurun_out/mp
    BGX_MLP_NT=$nt timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mp -o run --output-format csv -- python tools/mlp_micro.py $n > /dev/null 2>&1 || exit 1
    f=$(find gpurun_out/mp -name "*kernel_stats.csv" | head -1)
    python -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'mlp_kernel' in r['Name']: print('rows=$n nt=$nt', r['Name'][:40], 'avg_us', round(float(r['AverageNs'])/1e3,2), 'calls', r['Calls'])"
  done
done
