"""Summarise tools/pmc_bimodal.sh (tooling): per pass, the sspmm_bwd4 dispatches split at the
midpoint of their duration range into fast and slow, and each counter's mean per group."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_bimodal"
for pdir in sorted(glob.glob(os.path.join(root, "pass*"))):
    if not os.path.isdir(pdir):
        continue
    dur = {}
    for f in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "sspmm_bwd4" in r["Kernel_Name"]:
                dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt = defaultdict(dict)
    for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "sspmm_bwd4" in r["Kernel_Name"]:
                cnt[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    if not dur:
        continue
    lo, hi = min(dur.values()), max(dur.values())
    mid = (lo + hi) / 2
    groups = {"fast": [d for d in dur if dur[d] < mid], "slow": [d for d in dur if dur[d] >= mid]}
    print(f"{os.path.basename(pdir)}: {len(dur)} dispatches, {lo / 1e3:.1f}-{hi / 1e3:.1f} us")
    names = sorted({c for d in cnt.values() for c in d})
    for g, ids in groups.items():
        if not ids:
            continue
        mean_t = sum(dur[d] for d in ids) / len(ids) / 1e3
        vals = {c: sum(cnt[d].get(c, 0.0) for d in ids) / len(ids) for c in names}
        print(f"  {g}: n={len(ids)} mean {mean_t:.1f} us  " +
              "  ".join(f"{c}={v:.4g}" for c, v in vals.items()))
