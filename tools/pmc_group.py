"""Summarise rocprofv3 --pmc counter CSVs under a directory per kernel name (tooling): mean
counter value per dispatch, plus the mean kernel duration from the kernel trace.
  python tools/pmc_group.py gpurun_out/pmcany_x [name-substring ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2:]
vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)


def short(name):
    name = re.sub(r"\(.*$", "", name)
    return name.replace("void ", "").replace("maxk::", "")[:70]


for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = short(r.get("Kernel_Name", ""))
        if filt and not any(s in n for s in filt):
            continue
        vals[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(root, "pass*", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = short(r.get("Kernel_Name", ""))
        if n in vals:
            durs[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for kern, cs in vals.items():
    d = durs.get(kern, [])
    print(f"{kern}  (mean {sum(d) / max(1, len(d)):.4f} ms over {len(d)} dispatches)")
    for c, v in sorted(cs.items()):
        print(f"  {c:40s} {sum(v) / len(v):.6g}")
