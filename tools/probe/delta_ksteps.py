import sys, numpy as np
sys.path[:0] = ['/root/repo/oracle', '/root/repo/tests']
import oracle as orc
d = np.load('/root/repo/tests/golden/env_traj.npz')
rng = np.random.default_rng(1)
idx = rng.choice(d['after'].shape[0], 120, replace=False)
rolls = [(a, b) for a in range(1, 7) for b in range(a, 7)]
def groups(b):  # 24 byte groups (pairs of points per player) + group 24 (bar/off)
    p = np.concatenate([b[0:24], b[24:48]]).reshape(24, 2)
    return p, b[48:52]
tot_steps = 0; tiles = 0; hist = []; fixed = []
for i in idx:
    root = d['after'][i]; opp = 1 - int(d['player'][i])
    rp, rx = groups(root)
    rows = []
    for a, b in rolls:
        n, res, _ = orc.movegen(root, opp, a, b)
        rows += list(res[:n])
    for t in range(0, len(rows), 32):
        m = np.zeros(25, bool)
        for bd in rows[t:t+32]:
            p, x = groups(bd)
            m[:24] |= (p != rp).any(axis=1); m[24] |= (x != rx).any()
        g = int(m.sum()); hist.append(g); tot_steps += (g + 1) // 2; tiles += 1; ks = m[:24].reshape(12, 2).any(axis=1).sum() + 1; fixed.append(ks)
h = np.array(hist)
print('fixed-pair ksteps', np.mean(fixed)); print('tiles', tiles, 'mean groups', h.mean(), 'p50', np.median(h), 'p90', np.percentile(h, 90), 'mean ksteps', tot_steps / tiles, 'vs 13')
