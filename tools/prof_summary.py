"""Per-step kernel breakdown of a `rocprofv3 --kernel-trace` run of bench.py (rocpd SQLite database or the
kernel_trace.csv of `--output-format csv`).

A step is anchored on the corr-pyramid launch (one per RAFT forward): the span from the k-th to the (k+1)-th
anchor holds exactly one step's kernels. The last `--steps` anchors are used (the timed region), giving
steps - 1 full spans. Prints ms/step, share, launches/step and mean duration per kernel, plus span / busy / idle.

usage: python tools/prof_summary.py <run_results.db | kernel_trace.csv> [--steps 5] [--anchor corr_pyramid] [--skip-last 2]
"""
import argparse
import collections
import csv
import sqlite3


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, start, end in c.execute("select name, start, end from kernels order by start"):
            rows.append((name, int(start), int(end)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        rows.sort(key=lambda r: r[1])
    return rows


def short(name, width=110):
    n = name.replace("void ", "")
    return n if len(n) <= width else n[: width - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--skip-last", type=int, default=0,
                    help="anchors after the timed region to ignore (bench.py's API lookup leg builds 2 pyramids)")
    ap.add_argument("--anchor", default="corr_pyramid")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = load(a.path)
    anchors = [i for i, r in enumerate(rows) if a.anchor in r[0]]
    if len(anchors) < 2:
        raise SystemExit(f"need >= 2 '{a.anchor}' launches, found {len(anchors)}")
    sel = anchors[: len(anchors) - a.skip_last][-a.steps:]
    lo, hi = sel[0], sel[-1]
    spans = len(sel) - 1
    part = rows[lo:hi]
    t0, t1 = part[0][1], rows[hi][1]
    busy = 0
    last_end = t0
    for _, s, e in part:  # union of kernel intervals (single stream: effectively sequential)
        if e > last_end:
            busy += e - max(s, last_end)
            last_end = e
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e in part:
        agg[n][0] += 1
        agg[n][1] += e - s
    span_ms = (t1 - t0) / 1e6 / spans
    busy_ms = busy / 1e6 / spans
    print(f"# {a.path}: {spans} step spans anchored on '{a.anchor}'")
    print(f"# span {span_ms:.3f} ms/step, kernel busy {busy_ms:.3f} ms/step, idle gaps {span_ms - busy_ms:.3f} ms/step")
    print("# ms/step  share  launches/step  mean_us  kernel")
    tot = sum(v[1] for v in agg.values())
    for n, (cnt, dur) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{dur / 1e6 / spans:9.3f} {100 * dur / tot:5.1f}% {cnt / spans:8.1f} {dur / cnt / 1e3:9.1f}  {short(n)}")


if __name__ == "__main__":
    main()
