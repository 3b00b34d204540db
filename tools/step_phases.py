"""Phases of one RAFT step from a rocprofv3 kernel trace of bench.py (CSV): the encoder phase (first kernel of the step
-> the corr pyramid's start), the pyramid, the update loop (pyramid end -> the step's last kernel), and per stream the
busy time of the encoder phase, so the critical path of the encoders can be read off.
    python tools/step_phases.py gpurun_out/prof/run_kernel_trace.csv [--steps 3]"""
import argparse
import collections
import csv
import re


def short(n):
    n = n.replace("void ", "").replace("oflow::(anonymous namespace)::", "")
    return re.sub(r"\(oflow::.*|\(float const\*.*|\(at::.*|\(unsigned.*|\(int,.*", "", n)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
    pyr = [i for i, e in enumerate(ev) if "corr_pyramid" in e[2]]
    # step k: from the first kernel after pyramid k-1's step end ... use the pyramids as anchors: the encoder phase of
    # step k is the run of kernels between the last convex_upsample before pyramid k and pyramid k
    ups = [i for i, e in enumerate(ev) if "convex_upsample" in e[2]]
    out = []
    for pk in pyr[-a.steps - 1 : -1]:
        prev_up = max([u for u in ups if u < pk], default=None)
        if prev_up is None:
            continue
        nxt_up = min([u for u in ups if u > pk], default=None)
        if nxt_up is None:
            continue
        enc = ev[prev_up + 1 : pk]
        t0 = min(e[0] for e in enc)
        p0, p1 = ev[pk][0], ev[pk][1]
        t_end = ev[nxt_up][1]
        per_stream = collections.defaultdict(float)
        per_kernel = collections.defaultdict(float)
        for s, e, n, st in enc:
            per_stream[st] += (e - s) / 1e3
            per_kernel[short(n)] += (e - s) / 1e3
        out.append((p0 - t0, p1 - p0, t_end - p1, dict(per_stream), per_kernel))
    for enc_ns, pyr_ns, upd_ns, ps, pk in out:
        print(f"encoders {enc_ns / 1e3:8.1f} us | pyramid {pyr_ns / 1e3:7.1f} us | update loop {upd_ns / 1e3:8.1f} us | "
              f"encoder busy per stream (us): " + ", ".join(f"{k}: {v:.0f}" for k, v in sorted(ps.items())))
    if out:
        print("encoder-phase kernel time (us, summed over streams, last step):")
        for n, v in sorted(out[-1][4].items(), key=lambda x: -x[1])[:25]:
            print(f"  {v:8.1f}  {n}")


if __name__ == "__main__":
    main()
