"""VERDICT r5 item 5 probe (tools only): a hi-only first pass of the reply MLP
(split-fp16 W1 without its lo terms) and an exact pass for the rows that can
enter a (candidate, roll)'s top 5. Reports, over 2-ply reply lists of
trajectory positions (tests/golden/env_traj.npz), the share of rows in a top 5,
the observed max |V_hi - V| and the share of rows that a margin of 2 x err
around the 5th-best hi value adds, for err = the observed max and for the
rigorous per-row bound that avoids a second GEMM:
|dV| <= 1/4 sum_j |w2_j| max_k |lo_jk| * sum_k x_k (lo = W1 - hi, fp16 split of
bgx_frag.h at the global 2^e scale)."""
import sys
import numpy as np
sys.path[:0] = ['/root/repo/oracle', '/root/repo/tests']
import oracle as orc

d = np.load('/root/repo/tests/golden/env_traj.npz')
rng = np.random.default_rng(1)
idx = rng.choice(d['after'].shape[0], 150, replace=False)
rolls = [(a, b) for a in range(1, 7) for b in range(a, 7)]
for wf in ("weights_seed0.npz", "weights_ckpt2100000.npz"):
    w = dict(np.load('/root/repo/tests/golden/' + wf))
    W1 = w["W1"].astype(np.float64)
    e = 14 - int(np.floor(np.log2(np.abs(W1 * 1.4426950408889634).max())))
    sc = 2.0 ** e
    Wh = (W1 * sc).astype(np.float32).astype(np.float16).astype(np.float64) / sc
    lo = np.abs(W1 - Wh)
    C = 0.25 * np.sum(np.abs(w["w2"]) * lo.max(axis=1))
    groups = []
    for i in idx:
        root = d['after'][i]; opp = 1 - int(d['player'][i])
        for a, b in rolls:
            n, res, _ = orc.movegen(root, opp, a, b)
            if n == 0:
                continue
            x = orc.encode_many(res[:n], [opp] * n).astype(np.float64)
            v = orc.value(w, x.astype(np.float32))
            h = 1 / (1 + np.exp(-(x @ Wh.T + w["b1"])))
            vh = h @ w["w2"].astype(np.float64) + float(w["b2"][0])
            groups.append((v, vh, C * x.sum(axis=1)))
    tot = sum(len(g[0]) for g in groups)
    top = sum(min(5, len(g[0])) for g in groups)
    err = max(np.abs(g[1] - g[0]).max() for g in groups)
    rig = max(g[2].max() for g in groups)
    print(f"{wf}: {tot} reply rows, top-5 share {top / tot:.3f}, observed max |V_hi - V| {err:.2e}, "
          f"rigorous per-row bound up to {rig:.2e}")
    for name, margin in (("observed", lambda g: 2 * err), ("rigorous", lambda g: g[2] + g[2].max())):
        extra = 0
        for g in groups:
            k = min(5, len(g[1])); t5 = np.sort(g[1])[::-1][k - 1]
            extra += int(np.sum(g[1] >= t5 - margin(g))) - k
        print(f"   margin {name}: rows refined {(top + extra) / tot:.3f}")
