"""Summarise tools/pmc_mfma_job.sh: per MFMA kernel of the step (name with template arguments + grid size), the median per
dispatch of its counters and the derived matrix-core figures.

    python tools/pmc_mfma.py <pass1 counter_collection.csv> <pass2 counter_collection.csv> [--json out.json]

Derived (MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles, 32 per 32x32x16 f16 MFMA; SQ_WAVE_CYCLES /
SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs, SQ_BUSY_CYCLES over the 32
shader engines):
  clock_ghz_grbm = GRBM_GUI_ACTIVE / 8 / duration: reads high on dispatches shorter than ~0.3 ms (the guide's DVFS
                   note; r04 saw 2.9-3.6 GHz for short kernels, above the chip's 2.4 GHz)
  clock_ghz      = the dispatch's own clock: SQ_BUSY_CYCLES / 32 / duration when that lies in [1.0, 2.4] GHz, else
                   min(clock_ghz_grbm, 2.4); `clock_source` says which
  mfma_util      = SQ_VALU_MFMA_BUSY_CYCLES / (duration * clock_ghz * 1024 SIMDs)   (fraction of SIMD-cycles busy on MFMA)
  mfma_util_2p4  = the same at the nominal 2.4 GHz (a lower bound on the fraction)
  busy_per_mfma = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA   (32 expected for 32x32x16 f16)
  wait_any / wait_inst / active = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  lds_conflict  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
Durations come from the PMC run's dispatch timestamps (dispatches serialised: each kernel alone).
"""
import argparse
import csv
import json
import re
import statistics
from collections import defaultdict


def short_name(k: str) -> str:
    m = re.search(r"(\w+_kernel(?:<[^()]*>)?)", k)
    return m.group(1).replace(" ", "") if m else k[:80]


def load(path):
    per = defaultdict(dict)  # (kernel, grid, dispatch) -> counter -> value ; "_dur_ns"
    for r in csv.DictReader(open(path)):
        key = (short_name(r["Kernel_Name"]), int(r["Grid_Size"]), r["Dispatch_Id"])
        d = per[key]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["_dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    groups = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [per-dispatch values]
    for p in a.paths:
        for (k, g, _), d in load(p).items():
            for c, v in d.items():
                groups[(k, g)][c].append(v)
    out = []
    for (k, g), cs in sorted(groups.items(), key=lambda kv: -statistics.median(kv[1]["_dur_ns"]) * len(kv[1]["_dur_ns"])):
        med = {c: statistics.median(v) for c, v in cs.items()}
        row = {"kernel": k, "grid": g, "dispatches": len(cs["_dur_ns"]), "us": round(med["_dur_ns"] / 1e3, 2)}
        gui = med.get("GRBM_GUI_ACTIVE")
        dur = med["_dur_ns"]
        clk, src = None, None
        if med.get("SQ_BUSY_CYCLES"):
            c = med["SQ_BUSY_CYCLES"] / 32 / dur
            row["clock_ghz_sq_busy"] = round(c, 3)
            if 1.0 <= c <= 2.4:
                clk, src = c, "SQ_BUSY_CYCLES"
        if gui:
            row["clock_ghz_grbm"] = round(gui / 8 / dur, 3)
            if clk is None:
                clk, src = min(gui / 8 / dur, 2.4), "GRBM_GUI_ACTIVE (capped at 2.4 GHz)"
        if clk is not None:
            row["clock_ghz"], row["clock_source"] = round(clk, 3), src
            if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
                row["mfma_util"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (dur * clk * 1024), 4)
                row["mfma_util_2p4"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / (dur * 2.4 * 1024), 4)
        if med.get("SQ_INSTS_MFMA"):
            row["mfma_insts"] = med["SQ_INSTS_MFMA"]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
                row["busy_per_mfma"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / med["SQ_INSTS_MFMA"], 2)
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c, nm in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"), ("SQ_ACTIVE_INST_ANY", "active"),
                          ("SQ_WAIT_INST_LDS", "wait_inst_lds")):
                if c in med:
                    row[nm] = round(med[c] / wc, 4)
        if med.get("SQ_LDS_IDX_ACTIVE"):
            row["lds_conflict"] = round(med.get("SQ_LDS_BANK_CONFLICT", 0.0) / med["SQ_LDS_IDX_ACTIVE"], 4)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SALU", "SQ_WAVES"):
            if c in med:
                row[c] = med[c]
        out.append(row)
    for r in out:
        print(json.dumps(r))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
