"""Summary of tools/pmc_alloc.sh (tooling, round 6): per pass, the sspmm_bwd4 dispatches of
tools/shard_alloc.py --plans-only in launch order are grouped per (round, plan) (one untimed
launch first, then 1 + 3 x reps per timing), each group's mean duration and counters computed,
and the plans split at the median duration into a fast and a slow half; printed per counter:
the two halves' means (per dispatch) and their ratio.

  python tools/pmc_alloc_summary.py gpurun_out/pmc_alloc [--reps 10] [--plans 9]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(pdir):
    trace = {}
    for f in glob.glob(os.path.join(pdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "sspmm_bwd4" in r["Kernel_Name"]:
                trace[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ctr = defaultdict(dict)
    for f in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "sspmm_bwd4" in r["Kernel_Name"]:
                ctr[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return trace, ctr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--plans", type=int, default=9)
    a = ap.parse_args()
    per = 1 + 3 * a.reps
    out = {}
    for pdir in sorted(glob.glob(os.path.join(a.root, "pass*/"))):
        trace, ctr = load(pdir)
        ids = sorted(trace)[1:]                               # the untimed reference launch
        groups = []
        for gi in range(len(ids) // per):
            g = ids[gi * per:(gi + 1) * per][1:]               # drop each timing's warm-up
            us = sum(trace[i] for i in g) / len(g)
            cs = defaultdict(float)
            for i in g:
                for c, v in ctr.get(i, {}).items():
                    cs[c] += v / len(g)
            groups.append({"plan": gi % a.plans, "round": gi // a.plans, "us": us, "ctr": dict(cs)})
        if not groups:
            continue
        med = sorted(x["us"] for x in groups)[len(groups) // 2]
        fast = [x for x in groups if x["us"] < med]
        slow = [x for x in groups if x["us"] >= med]
        names = sorted({c for x in groups for c in x["ctr"]})
        res = {"plans_us": [[round(x["us"], 1) for x in groups if x["round"] == r]
                            for r in range(2)],
               "fast_us": sum(x["us"] for x in fast) / max(1, len(fast)),
               "slow_us": sum(x["us"] for x in slow) / max(1, len(slow))}
        for c in names:
            f = sum(x["ctr"].get(c, 0) for x in fast) / max(1, len(fast))
            s = sum(x["ctr"].get(c, 0) for x in slow) / max(1, len(slow))
            res[c] = {"fast": f, "slow": s, "slow_over_fast": s / f if f else None}
        out[os.path.basename(pdir.rstrip("/"))] = res
        print(os.path.basename(pdir.rstrip("/")), json.dumps(res["plans_us"]))
        print(f"  fast {res['fast_us']:.1f} us  slow {res['slow_us']:.1f} us")
        for c in names:
            r = res[c]
            print(f"  {c:48s} fast {r['fast']:.4g}  slow {r['slow']:.4g}  "
                  f"x{(r['slow_over_fast'] or 0):.3f}")
    with open(os.path.join(a.root, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
