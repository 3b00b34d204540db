"""Summarise rocprofv3 PMC results (rocpd sqlite run_results.db or counter_collection.csv): per kernel (name match),
the median per dispatch of every counter.   python tools/pmc_db.py <db-or-csv>... [--kernel REGEX]"""
import argparse
import csv
import glob
import re
import sqlite3
import statistics
from collections import defaultdict


def rows_db(path):
    con = sqlite3.connect(path)
    q = """select s.string as kname, p.name as cname, e.value as val, e.event_id as eid
           from rocpd_pmc_event e
           join rocpd_info_pmc p on p.id = e.pmc_id
           join rocpd_event ev on ev.id = e.event_id
           join rocpd_kernel_dispatch d on d.event_id = ev.id
           join rocpd_info_kernel_symbol k on k.id = d.kernel_id
           join rocpd_string s on s.id = k.kernel_name_id"""
    try:
        for r in con.execute(q):
            yield r
    except sqlite3.Error:
        # schema variant: kernel name stored directly
        for r in con.execute("""select k.kernel_name, p.name, e.value, e.event_id from rocpd_pmc_event e
                                join rocpd_info_pmc p on p.id = e.pmc_id join rocpd_kernel_dispatch d on d.event_id = e.event_id
                                join rocpd_info_kernel_symbol k on k.id = d.kernel_id"""):
            yield r


def rows_csv(path):
    for r in csv.DictReader(open(path)):
        yield r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r["Dispatch_Id"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--kernel", default=".")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> sum
    for pat in a.paths:
        for path in glob.glob(pat):
            it = rows_db(path) if path.endswith(".db") else rows_csv(path)
            for kname, cname, val, eid in it:
                if re.search(a.kernel, kname):
                    short = re.sub(r"\(.*", "", kname.split("::")[-1]) if "(" in kname else kname
                    acc[short][cname][(path, eid)] += float(val)
    for k, cs in acc.items():
        print(k)
        for c in sorted(cs):
            vals = list(cs[c].values())
            print(f"   {c:32s} median {statistics.median(vals):16.1f}   n={len(vals)}")


if __name__ == "__main__":
    main()
