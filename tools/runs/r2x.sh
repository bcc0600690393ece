# trainer kernel section clocks (stamp build) + timing of the 512-thread build
set -o pipefail
export TMPDIR=/tmp; OUT=gpurun_out/r2x; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/train_micro.py 10 > $OUT/micro.json 2> $OUT/micro.err || { tail $OUT/micro.err; exit 1; }
cat $OUT/micro.json
BGX_LIB=tools/diag/libbgx_tstamp.so timeout -k 10 300 python - > $OUT/stamps.txt 2> $OUT/stamps.err <<'PY' || { tail $OUT/stamps.err; exit 1; }
import ctypes, sys, os
sys.argv = ["x", "3"]
sys.path[:0] = ["tools", "mlp-ppo-2ply-multi_amd"]
import train_micro
from bgx import _lib
train_micro.main()
L = _lib.lib(); f = L.bgx_diag_train_stamps; f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
o = (ctypes.c_ulonglong * 6)(); f(o)
names = ["setup", "load_chunk", "forward", "backward", "clip+adam", "metrics"]
tot = sum(o)
print({n: round(v / tot, 3) for n, v in zip(names, o)}, "total cycles", tot)
PY
cat $OUT/stamps.txt
