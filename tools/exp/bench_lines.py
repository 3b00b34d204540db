"""Print value / ms_per_step / in-flight / roofline of the bench lines in gpurun_out/<prefix>*.log (A/B summaries):
python tools/exp/bench_lines.py r5s36_"""
import glob
import json
import os
import sys

for path in sorted(glob.glob(os.path.join("gpurun_out", sys.argv[1] + "*.log")), key=os.path.getmtime):
    name = os.path.basename(path)[:-4]
    text = open(path).read()
    try:
        d = json.loads(text[text.index('{"metric'):].split("\n")[0])
    except ValueError:
        print(name, "NO LINE:", text[-400:].replace("\n", " | "))
        continue
    print(name, d["value"], d["ms_per_step"], "inflight", d["config"].get("steps_in_flight"),
          "lookup_us", round(d.get("roofline", {}).get("launch_us", 0) or 0, 1), "frac", d.get("roofline", {}).get("frac"))
