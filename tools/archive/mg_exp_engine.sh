# movegen subtraction experiments inside the 2-ply engine (development; results invalid)
set -o pipefail
export TMPDIR=/tmp
for e in 0 1 2 3; do
  rm -rf gpurun_out/mge
  BGX_MG_EXP=$e timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mge -o run --output-format csv -- python bench.py --ply 2 --steps 30 --warmup 10 --two-ply-steps 0 --kall-steps 0 --timing-steps 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/mge -name "*kernel_stats.csv" | head -1)
  python tools/kstat.py "$f" "movegen_lds_kernel" "exp=$e"
done
