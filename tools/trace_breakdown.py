"""Per-step breakdown of a rocprofv3 kernel trace (CSV, optionally .gz) of bench.py: steps are delimited by the corr
pyramid launches; prints the busy (union) time per step and per-kernel summed durations over the last N steps.
    python tools/trace_breakdown.py gpurun_out/prof/run_kernel_trace.csv.gz [--steps 4]"""
import argparse
import collections
import csv
import gzip
import re


def short(name: str) -> str:
    n = name.replace("void ", "")
    n = n.replace("oflow::(anonymous namespace)::", "")
    n = re.sub(r"\(oflow::.*|\(float const\*.*|\(at::.*|\(unsigned.*|\(int,.*", "", n)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--marker", default="corr_pyramid_kernel")
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    rows = list(csv.DictReader(op(a.trace, "rt")))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    marks = [s for s, e, n in ev if a.marker in n]
    bounds = list(zip(marks[-a.steps - 1 : -1], marks[-a.steps:]))
    per = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    busy = 0.0
    for lo, hi in bounds:
        iv = sorted((s, e) for s, e, n in ev if lo <= s < hi)
        cur_s, cur_e = None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        for s, e, n in ev:
            if lo <= s < hi:
                per[short(n)] += (e - s)
                cnt[short(n)] += 1
    k = len(bounds)
    wall = sum(hi - lo for lo, hi in bounds) / k / 1e3
    print(f"steps {k}: wall {wall:.1f} us/step, GPU busy (union) {busy / k / 1e3:.1f} us/step "
          f"({busy / (wall * 1e3 * k):.1%}), summed kernel time {sum(per.values()) / k / 1e3:.1f} us/step")
    for n, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{v / k / 1e3:10.1f} us/step  {cnt[n] / k:6.1f} launches  {v / cnt[n] / 1e3:8.1f} us/launch  {n}")


if __name__ == "__main__":
    main()
