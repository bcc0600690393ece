# SQ / GRBM counter passes (rocprofv3 --pmc, one pass per group, never with
# tracing) for the kernels of one bench leg; output gpurun_out/$OUT/sq_<leg>_<i>/.
#   $1 = output dir under gpurun_out, $2 = leg (2ply_k4 | 2ply_kall | 1ply), $3 = kernel regex,
#   $4 = lanes (default 8192; another count names the leg l<lanes>_<leg>)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sq}; LEG=${2:-2ply_k4}; RX=${3:-"movegen_pool|mlp_kernel_il"}; LANES=${4:-8192}
mkdir -p $OUT
if [ $LEG = 2ply_k4 ]; then
  ARGS="--ply 2 --k-top 4 --steps 30 --warmup 10 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"
elif [ $LEG = 2ply_kall ]; then
  ARGS="--ply 2 --k-top 0 --steps 6 --warmup 2 --desync-steps 30 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"
else
  ARGS="--steps 300 --warmup 100 --timing-steps 1 --two-ply-steps 0 --kall-steps 0 --config1-steps 0 --config2-steps 0 --no-cpu-baseline"
fi
if [ $LANES != 8192 ]; then ARGS="$ARGS --lanes $LANES"; N=l${LANES}_$LEG; else N=$LEG; fi
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i+1)); rm -rf $OUT/sq_${N}_$i
  echo "[sq] $N pass $i: $grp"
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "$RX" -d $OUT/sq_${N}_$i -o run --output-format csv -- python bench.py $ARGS > $OUT/sq_${N}_$i.log 2>&1 || { tail -5 $OUT/sq_${N}_$i.log; exit 1; }
done
python tools/sq_summary.py $OUT $N > $OUT/sq_${N}.json && cat $OUT/sq_${N}.json
