# one-register job prefetch A/B + instruction counts per job kind
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2j; mkdir -p $OUT
bash tools/mg_pmc_kind.sh r2j/mgk || exit 1
bash tools/ab_multi.sh r2j/ab tools/diag/libbgx_prev.so
