# movegen PMC (development): the 2-ply reply launch (movegen_lds_kernel<512>) in the engine
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH" "SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU"; do
  i=$((i+1)); rm -rf gpurun_out/gpmc$i
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex "movegen_lds_kernel" -d gpurun_out/gpmc$i -o run --output-format csv -- python bench.py --ply 2 --steps 20 --warmup 10 --two-ply-steps 0 --timing-steps 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
done
python - <<'PY'
import csv,glob,collections
tot=collections.defaultdict(float); n=collections.defaultdict(set)
for i in (1,2,3,4):
    f=glob.glob(f'gpurun_out/gpmc{i}/**/*counter_collection.csv',recursive=True)[0]
    for r in csv.DictReader(open(f)):
        tot[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']].add(r['Dispatch_Id'])
jobs=4096*84
for k in sorted(tot):
    v=tot[k]/len(n[k]); print(k, '%.4g'%v, 'per dispatch', '%.1f'%(v/jobs), 'per job')
PY
