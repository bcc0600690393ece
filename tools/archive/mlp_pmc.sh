# MLP PMC (development): counters for the NT=2 kernel at 2-ply size, one pass per group
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU"; do
  i=$((i+1)); rm -rf gpurun_out/mpmc$i
  BGX_MLP_NT=2 timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "mlp_kernel" -d gpurun_out/mpmc$i -o run --output-format csv -- python tools/mlp_micro.py 6900000 > /dev/null 2>&1 || exit 1
done
python - <<'PY'
import csv,glob,collections
tot=collections.defaultdict(float); n=collections.defaultdict(set)
for i in (1,2,3):
    f=glob.glob(f'gpurun_out/mpmc{i}/**/*counter_collection.csv',recursive=True)[0]
    for r in csv.DictReader(open(f)):
        tot[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']].add(r['Dispatch_Id'])
for k in sorted(tot): print(k, '%.4g'%(tot[k]/len(n[k])), 'per dispatch')
PY
