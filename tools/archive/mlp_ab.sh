# MLP A/B (development): kernel averages at 2-ply size for BGX_MLP_IL x BGX_MLP_NT
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q -k "value or two_ply or engine" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for il in 0 1; do for nt in 1 2; do
  rm -rf gpurun_out/mp
  BGX_MLP_NT=$nt BGX_MLP_IL=$il timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mp -o run --output-format csv -- python tools/mlp_micro.py ${ROWS:-6900000} > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/mp -name "*kernel_stats.csv" | head -1)
  python tools/kstat.py "$f" mlp_kernel "IL=$il NT=$nt"
done; done
