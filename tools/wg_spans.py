"""Per-workgroup spans of a fused launch (BGX_FUSED_PROF_DUMP csv): end time
vs the launch's first begin, by lane-steps taken and tier-2 jobs; the late
workgroups listed. Development tool."""
import csv
import sys

import numpy as np

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    b = np.array([int(r["begin"]) for r in rows], np.float64)
    e = np.array([int(r["end"]) for r in rows], np.float64)
    l0 = np.array([int(r["loop0"]) for r in rows], np.float64)
    l1 = np.array([int(r["loop1"]) for r in rows], np.float64)
    st = np.array([int(r["lane_steps"]) for r in rows]) // 32
    t2 = np.array([int(r["tier2"]) for r in rows])
    t0 = b.min()
    end = (e - t0) / 100.0
    per_step = (l1 - l0) / 100.0 / np.maximum(st, 1)
    print(f"{path}: {len(rows)} workgroups, end us mean {end.mean():.1f} max {end.max():.1f}")
    for s in sorted(set(st.tolist())):
        m = st == s
        print(f"  {s} steps: {m.sum():3d} wgs, end mean {end[m].mean():.1f} max {end[m].max():.1f}, "
              f"us/step {per_step[m].mean():.2f}, tier-2 jobs {t2[m].mean():.2f}")
    late = np.argsort(-end)[:6]
    print("  latest:", [(int(rows[i]["wg"]), round(end[i], 1), int(st[i]), int(t2[i]), round(per_step[i], 2)) for i in late])
