"""Per-(kernel, grid) breakdown of the last step of a rocprofv3 --kernel-trace run of bench.py: which layer is
which launch. usage: python tools/prof_grid.py <run_results.db> [--anchor corr_pyramid]"""
import argparse
import collections
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--anchor", default="corr_pyramid")
args = ap.parse_args()
c = sqlite3.connect(args.db)
rows = list(c.execute("select name, start, end, grid_x, grid_y, workgroup_x, vgpr_count, accum_vgpr_count, lds_size "
                      "from kernels order by start"))
anchors = [i for i, r in enumerate(rows) if args.anchor in r[0]]
lo, hi = anchors[-2], anchors[-1]
agg = collections.OrderedDict()
for name, s, e, gx, gy, wx, vg, ag, lds in rows[lo:hi]:
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    short = (m.group(1) + (m.group(2) or "")) if m else name[:60]
    key = (short[:70], gx // max(wx, 1), gy)
    a = agg.setdefault(key, [0, 0.0, vg, ag, lds])
    a[0] += 1
    a[1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"# step span {(rows[hi][1] - rows[lo][1]) / 1e6:.3f} ms, busy {tot / 1e3:.3f} ms")
for (k, gx, gy), (n, us, vg, ag, lds) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{us / 1e3:7.3f} ms {n:3d}x {us / n:8.1f} us  grid {gx:6d}x{gy:<3d} vgpr {vg}/{ag} lds {lds:6d}  {k}")
