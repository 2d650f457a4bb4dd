"""Per-kernel summary of a rocprofv3 results database (kernel-trace run):
python tools/prof_kernels.py <run_results.db> [name-substring ...] [--by-grid]"""
import collections
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
by_grid = "--by-grid" in sys.argv
db, pats = args[0], args[1:]
c = sqlite3.connect(db)
rows = c.execute("select name, grid_x, grid_y, grid_z, end-start from kernels").fetchall()
agg = collections.defaultdict(list)
for n, gx, gy, gz, d in rows:
    if pats and not any(p in n for p in pats):
        continue
    key = (n[:90], (gx, gy, gz)) if by_grid else (n[:90], None)
    agg[key].append(d)
for (n, g), ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(ds) / 1e6:9.3f} ms  calls {len(ds):6d}  avg {sum(ds) / len(ds) / 1e3:9.2f} us  {n} {g or ''}")
