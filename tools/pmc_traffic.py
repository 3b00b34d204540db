"""Per-launch HBM traffic of the corr_lookup kernel from rocprofv3 PMC passes -> profiles/lookup_traffic.json.

Counters are collected in separate passes of the same bench command (MI355X_MICROARCH.md §HBM / rocprofv3 PMC):
    rocprofv3 --pmc TCC_EA0_RDREQ_sum --kernel-include-regex corr_lookup ... -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE        --kernel-include-regex corr_lookup ... -- python bench.py ...
Corrections (gfx950):
  * reads: FETCH_SIZE = TCC_EA0_RDREQ x 64 B, but the guide notes that wide reads issue 128-B requests tallied at
    64 B. Calibrated on this kernel's own pattern: the canonical-layout lookup issues 1.81 M requests per Sintel x8
    launch against ~2.17 M predicted 128-B line touches of its 10 x 10 windows (~2.97 M if the requests were
    64-B sectors), so each request is one 128-B line: read bytes = TCC_EA0_RDREQ_sum x 128.
  * writes: WRITE_SIZE (KiB) is exact for this kernel: 71,280 KiB = the 72.99 MB fp32 output, per launch.

usage: python tools/pmc_traffic.py <rdreq_counter_collection.csv> <write_size_counter_collection.csv> <key> [kernel regex]
(key = "<workload>:<pairs per GPU>:<kernel tag>", the name bench.py looks up; the regex selects the kernel's rows)
"""
import csv
import json
import os
import re
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "lookup_traffic.json")


def per_launch(path, counter, regex=None):
    pat = re.compile(regex) if regex else None
    rows = [r for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and (pat is None or pat.search(r.get("Kernel_Name", "")))]
    # the bench's own launches are the largest grid (the golden-EPE check before the timed region runs 1 pair)
    big = max((int(r["Grid_Size"]) for r in rows), default=0)
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == big]
    if not vals:
        raise SystemExit(f"{path}: no {counter} rows")
    return statistics.median(vals), len(vals)


def main():
    rd_csv, wr_csv, key = sys.argv[1:4]
    regex = sys.argv[4] if len(sys.argv) > 4 else None
    req, n1 = per_launch(rd_csv, "TCC_EA0_RDREQ_sum", regex)
    wr_kib, n2 = per_launch(wr_csv, "WRITE_SIZE", regex)
    rd, wr = int(req * 128), int(wr_kib * 1024)
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    data[key] = {
        "hbm_bytes_per_launch": rd + wr,
        "read_bytes_per_launch": rd,
        "write_bytes_per_launch": wr,
        "tcc_ea0_rdreq_per_launch": req,
        "write_size_kib_per_launch": wr_kib,
        "launches_sampled": [n1, n2],
        "sources": [os.path.relpath(rd_csv, REPO), os.path.relpath(wr_csv, REPO)],
        "correction": "reads = TCC_EA0_RDREQ_sum x 128 B (128-B requests tallied at 64 B by FETCH_SIZE); writes = WRITE_SIZE KiB x 1024",
    }
    json.dump(data, open(OUT, "w"), indent=1)
    print(json.dumps(data[key]))


if __name__ == "__main__":
    main()
