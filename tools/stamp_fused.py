#!/usr/bin/env python3
"""Tier-1 job section clocks of the fused 1-ply kernel (tools only; needs the
diagnostic build: make EXTRA=-DBGX_STAMP OUT=tools/diag/libbgx_stamp.so, run
with BGX_LIB pointing at it). Shader-clock cycles per job and section."""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd")]
from bgx import Engine  # noqa: E402
from bgx import _lib  # noqa: E402

lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
L = _lib.lib()
fn = L.bgx_diag_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
out = (ctypes.c_ulonglong * 32)()
e = Engine(lanes=lanes, seed=3, ply=1)
e.set_weights(w, temperature=1.5)
e.step(200)
e.sync()
e.harvest()
fn(out)   # zero
e.step(200)
e.sync()
assert fn(out) == 0
s = list(out)
nd, dd = max(1, s[4]), max(1, s[11])
nnd = s[0] / max(1, s[13]) if s[13] else 0
names = {0: "nd make_job", 1: "nd level-1 (root moves, child moves)", 2: "nd expand_keep", 13: "nd job_records total",
         3: "nd emit", 5: "d make_job", 6: "d levels 0-1", 7: "d level 2", 8: "d level 3", 9: "d records compaction",
         12: "d job_records total", 10: "d emit"}
res = {"rule nd jobs": s[4], "path d jobs": s[11], "nd results": s[14], "d results": s[15],
       "overflow: table full": s[20], "overflow: table-mode frontier": s[21], "overflow: nd rule list": s[22],
       "overflow: doubles path list": s[23], "overflow: nd table job": s[24], "overflow: doubles table job": s[25]}
for k, n in names.items():
    den = s[11] if n.startswith("d ") else s[4]
    res[n] = round(s[k] / max(1, den), 1)
print(json.dumps(res, indent=1))
