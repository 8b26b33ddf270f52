"""Summarise gpurun_out/pmc*/pass*/ counter CSVs per kernel (tooling)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        short = ("spgemm_fwd" if "spgemm_fwd_kernel" in name else
                 "sspmm_bwd" if "sspmm_bwd" in name else
                 "pack_cbsr" if "pack_cbsr" in name else None)
        if short is None:
            continue
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kern, cs in vals.items():
    print(kern)
    for c, v in sorted(cs.items()):
        print(f"  {c:40s} mean {sum(v) / len(v):.6g}  (n={len(v)})")
