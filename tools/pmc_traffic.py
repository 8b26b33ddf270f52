"""Per-launch HBM-side traffic from rocprofv3 PMC passes (tooling) -> profiles/pmc_traffic.json.

  python tools/pmc_traffic.py gpurun_out/pmc [--key reddit:k16:d256:n1] [--out profiles/pmc_traffic.json]

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch. MI355X_MICROARCH.md (HBM section):
FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read on gfx950, so it is doubled;
WRITE_SIZE is exact for streaming stores and float atomics. Both count L2 memory-side requests,
so Infinity-Cache hits are included: the figure is L2-miss traffic (upper bound on HBM bytes).
bench.py reads the file to fill roofline.traffic for the dominant kernel.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SHORT = (("spgemm_fwd_kernel", "spgemm_fwd"), ("sspmm_bwd", "sspmm_bwd"),
         ("pack_cbsr", "pack_cbsr"), ("topk_exact", "topk"))


def collect(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            for pat, short in SHORT:
                if pat in name:
                    vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--key", default="reddit:k16:d256:n1")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
    args = ap.parse_args()
    vals = collect(args.root)
    entry = {}
    for kern, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        entry[kern] = fetch + write
        entry[kern + "_detail"] = {"fetch_bytes_x2": fetch, "write_bytes": write,
                                   "dispatches": len(cs["FETCH_SIZE"])}
        if "TCP_TCC_READ_REQ_sum" in cs:  # L1-miss line requests (128 B) per launch
            r = cs["TCP_TCC_READ_REQ_sum"]
            entry[kern + "_detail"]["l1_miss_requests"] = sum(r) / len(r)
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h, m = sum(cs["TCC_HIT_sum"]), sum(cs["TCC_MISS_sum"])
            entry[kern + "_detail"]["l2_hit_rate"] = h / max(h + m, 1.0)
    doc = json.load(open(args.out)) if os.path.exists(args.out) else {}
    doc[args.key] = entry
    json.dump(doc, open(args.out, "w"), indent=1, sort_keys=True)
    print(json.dumps({args.key: entry}, indent=1))


if __name__ == "__main__":
    main()
