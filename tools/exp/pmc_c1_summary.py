"""Summarise tools/exp/pmc_c1_job.sh: per fused-kernel variant (kernel name + grid), the median per dispatch of every
counter of the passes, and derived memory-pipe figures:
  ta_busy        = TA_TA_BUSY_sum / (SQ_BUSY_CYCLES / 32 * 256 / 8 ...)  -> reported raw and per CU-cycle
  l2_lat_cycles  = TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum (mean TCP->TCC read latency)
  rdreq_mix      = TCC_EA0_RDREQ_{32B,64B,128B} shares of TCC_EA0_RDREQ
    python tools/exp/pmc_c1_summary.py gpurun_out/pmcc1 [--json out.json]"""
import argparse
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pmc_mfma import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    a = ap.parse_args()
    per = {}
    for path in sorted(glob.glob(os.path.join(a.root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for (k, grid, _), d in load(path).items():
            e = per.setdefault((k, grid), {})
            for c, v in d.items():
                e.setdefault(c, []).append(v)
    out = []
    for (k, grid), e in sorted(per.items()):
        m = {c: statistics.median(v) for c, v in e.items()}
        dur_cyc = m.get("SQ_BUSY_CYCLES", 0) / 32.0  # per-SE busy cycles summed over 32 SEs -> chip cycles
        r = {"kernel": k, "grid": grid, "us": round(m["_dur_ns"] / 1e3, 2), "dispatches": len(e["_dur_ns"])}
        for c in sorted(m):
            if c != "_dur_ns":
                r[c] = m[c]
        if dur_cyc > 0:
            for c in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum",
                      "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum",
                      "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum", "TCP_TD_TCP_STALL_CYCLES_sum", "TD_TC_STALL_sum"):
                if c in m:
                    r[c.replace("_sum", "") + "_per_cu"] = round(m[c] / 256.0 / dur_cyc, 3)
        if m.get("TCP_TCC_READ_REQ_sum"):
            r["l2_lat_cycles"] = round(m.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / m["TCP_TCC_READ_REQ_sum"], 1)
        if m.get("TCC_EA0_RDREQ_sum"):
            t = m["TCC_EA0_RDREQ_sum"]
            r["rdreq_mix_32_64_128"] = [round(m.get(f"TCC_EA0_RDREQ_{b}B_sum", 0) / t, 3) for b in (32, 64, 128)]
        if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
            r["tcc_hit_rate"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3)
        out.append(r)
        print(json.dumps(r))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
