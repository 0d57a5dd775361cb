"""Per-kernel duration summary of a rocprofv3 kernel-trace database (rocpd sqlite output; the first dispatch
of each kernel -- code-object load, cold caches -- reported apart).
    python tools/kt_db.py <results.db> [name-substring ...]"""
import sqlite3
import sys

import numpy as np

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, duration, scratch_size, vgpr_count, lds_size from kernels order by start").fetchall()
keep = sys.argv[2:]
agg, res = {}, {}
for nm, d, scr, vg, lds in rows:
    short = nm.split("(dat::")[0].replace("(anonymous namespace)::", "")
    if keep and not any(k in short for k in keep):
        continue
    agg.setdefault(short, []).append(d / 1e3)
    res[short] = (scr, vg, lds)
print(f"{'kernel':34s} {'calls':>5s} {'first us':>9s} {'avg us':>9s} {'p50 us':>9s} {'max us':>9s} {'scratch':>7s} "
      f"{'vgpr':>4s} {'lds':>6s}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    r = np.array(v[1:] if len(v) > 1 else v)
    print(f"{k[:34]:34s} {len(v):5d} {v[0]:9.1f} {r.mean():9.1f} {np.median(r):9.1f} {r.max():9.1f} {res[k][0]:7d} "
          f"{res[k][1]:4d} {res[k][2]:6d}")
