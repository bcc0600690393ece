# movegen subtraction experiments (development): mg_micro with parts skipped (results invalid)
set -o pipefail
export TMPDIR=/tmp
for e in 0 1 2 3; do   # never skip the table clear: probing a full table does not end
  echo -n "exp=$e "; BGX_MG_FEW=0 BGX_MG_EXP=$e timeout -k 10 120 python tools/mg_micro.py 200000 2>&1 | grep -v amdgpu | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v['ms']*1000,1) for k,v in d.items()}, 'us per 200k jobs')"
done
