"""From a rocprofv3 kernel-trace CSV: for the fused lookup + convc1 kernel, the mean duration and how much of its
time another corr_convc1 launch (the other pair lane) runs at the same time -- do the two lanes' launches overlap?
    python tools/exp/lane_overlap.py <kernel_trace.csv>"""
import csv
import statistics
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if "corr_convc1" in r["Kernel_Name"]]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    durs = [(e - s) / 1e3 for s, e in iv]
    ov = []
    for i, (s, e) in enumerate(iv):
        o = 0
        for j, (s2, e2) in enumerate(iv):
            if j != i and s2 < e and e2 > s:
                o += min(e, e2) - max(s, s2)
        ov.append(o / max(1, e - s))
    print(f"launches {len(iv)}  mean {statistics.mean(durs):.1f} us  median {statistics.median(durs):.1f} us  "
          f"overlapped fraction mean {statistics.mean(ov):.2f}")


if __name__ == "__main__":
    main()
