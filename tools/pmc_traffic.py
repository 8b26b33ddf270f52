"""Per-call HBM-side traffic from rocprofv3 PMC passes (tooling) -> profiles/pmc_traffic.json.

  python tools/pmc_traffic.py gpurun_out/pmc [--key reddit:k16:d256:n1]
  python tools/pmc_traffic.py --all gpurun_out      (every gpurun_out/pmc_<ds>_<kind>_k<k>)
  python tools/pmc_traffic.py --locality gpurun_out (gpurun_out/pmc_loc_* -> profiles/r03/pmc_locality.json)

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch. MI355X_MICROARCH.md (HBM section):
FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read on gfx950, so it is doubled;
WRITE_SIZE is exact for streaming stores and float atomics. Both count L2 memory-side requests,
so Infinity-Cache hits are included: the figure is L2-miss traffic (upper bound on HBM bytes).

Per kernel family (cbsr_stats4 = the fused pack + statistics, spgemm_fwd, pack_sel, sspmm_bwd4,
sspmm_bwd_rows, ...): bytes
per dispatch, dispatches per call (tools/pmc_driver.py makes 4 calls per direction), the
average kernel duration of the same passes (kernel trace) and the resulting GB/s. Direction
totals: "spgemm_fwd" = the forward kernel, "sspmm_bwd" = all SSpMM kernels of one backward
call (two-pass: rows + columns), "fwd_total" / "bwd_total" also count the per-call packs.
bench.py reads "spgemm_fwd" / "sspmm_bwd" for roofline.traffic and the k sweep.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

CALLS = 4  # tools/pmc_driver.py: 1 + 3 calls per direction
FWD = ("cbsr_stats4_kernel", "cbsr_stats_kernel", "pack_cbsr3_kernel", "zero_rows_kernel",
       "spgemm_fwd_kernel")
BWD_PACK = ("pack_sel_kernel", "pack_sel2_kernel", "bwd_combine_kernel")  # per-call, beside the SSpMM


def family(name):
    m = re.search(r"maxk::(\w+?)(<|\(|$)", name)
    return m.group(1) if m else None


def collect(root):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r.get("Kernel_Name", ""))
            if fam:
                vals[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(root, "pass1", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            fam = family(r.get("Kernel_Name", ""))
            if fam:
                durs[fam].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return vals, durs


def entry_for(root):
    vals, durs = collect(root)
    entry = {}
    sha = os.path.join(root, "lib_sha256.txt")
    # the libmaxk_hip.so the counters were collected on (tools/pmc_driver.py)
    entry["lib_sha256"] = open(sha).read().strip() if os.path.exists(sha) else None
    fam_bytes = {}
    fam_secs = {}
    for fam, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        per_call = len(cs["FETCH_SIZE"]) / CALLS
        d = {"bytes_per_dispatch": fetch + write, "fetch_bytes_x2": fetch, "write_bytes": write,
             "dispatches_per_call": per_call}
        if "TCP_TCC_READ_REQ_sum" in cs:  # L1-miss line requests (128 B) per dispatch
            r = cs["TCP_TCC_READ_REQ_sum"]
            d["l1_miss_requests"] = sum(r) / len(r)
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h, m = sum(cs["TCC_HIT_sum"]), sum(cs["TCC_MISS_sum"])
            d["l2_hit_rate"] = h / max(h + m, 1.0)
        if durs.get(fam):
            d["avg_ms"] = sum(durs[fam]) / len(durs[fam]) * 1e3
            d["GBps"] = (fetch + write) / (d["avg_ms"] * 1e-3) / 1e9
        entry[fam + "_detail"] = d
        fam_bytes[fam] = (fetch + write) * per_call
        fam_secs[fam] = d.get("avg_ms", 0.0) * 1e-3 * per_call
    fwd = [f for f in fam_bytes if f == "spgemm_fwd_kernel"]
    bwd = [f for f in fam_bytes if f.startswith("sspmm_bwd")]
    if fwd:
        entry["spgemm_fwd"] = sum(fam_bytes[f] for f in fwd)
        entry["fwd_total"] = sum(v for f, v in fam_bytes.items() if f in FWD)
        entry["spgemm_fwd_detail"] = dict(entry["spgemm_fwd_kernel_detail"])
    if bwd:
        entry["sspmm_bwd"] = sum(fam_bytes[f] for f in bwd)
        entry["bwd_total"] = entry["sspmm_bwd"] + sum(fam_bytes.get(f, 0.0) for f in BWD_PACK)
        secs = sum(fam_secs[f] for f in bwd)
        det = {"kernels": bwd, "GBps": entry["sspmm_bwd"] / secs / 1e9 if secs else None,
               "ms_per_call": secs * 1e3}
        if len(bwd) == 1:
            det.update(entry[bwd[0] + "_detail"])
        entry["sspmm_bwd_detail"] = det
    return entry


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--key", default="reddit:k16:d256:n1")
    ap.add_argument("--all", action="store_true",
                    help="root holds pmc_<dataset>_<kind>_k<k> directories")
    ap.add_argument("--locality", action="store_true",
                    help="root holds pmc_loc_<graph>_<order>_k<k> directories (round 3; pmc_loc_* passes over tools/pmc_driver.py)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
    args = ap.parse_args()
    if args.locality:
        out = os.path.join(os.path.dirname(args.out), "r03", "pmc_locality.json")
        doc = {}
        for d in sorted(glob.glob(os.path.join(args.root, "pmc_loc_*_k*"))):
            ent = entry_for(d)
            keep = {"lib_sha256": ent.get("lib_sha256")}
            for fam in ("spgemm_fwd", "sspmm_bwd"):
                det = ent.get(fam + "_detail", {})
                keep[fam] = {x: det.get(x) for x in ("avg_ms", "ms_per_call", "bytes_per_dispatch",
                                                      "l1_miss_requests", "l2_hit_rate", "GBps")
                             if x in det}
            doc[os.path.basename(d)[len("pmc_loc_"):]] = keep
            print(os.path.basename(d), json.dumps(keep))
        json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
        return
    doc = json.load(open(args.out)) if os.path.exists(args.out) else {}
    if args.all:
        for d in sorted(glob.glob(os.path.join(args.root, "pmc_*_k*"))):
            m = re.match(r"pmc_(.+)_(sage|gcn)_k(\d+)$", os.path.basename(d))
            if not m:
                continue
            ds, kind, k = m.group(1), m.group(2), int(m.group(3))
            ent = entry_for(d)
            ent["values"] = kind
            doc[f"{ds}:k{k}:d256:n1"] = ent
            print(f"{ds}:k{k} ({kind}): fwd {ent.get('spgemm_fwd', 0) / 1e9:.2f} GB "
                  f"bwd {ent.get('sspmm_bwd', 0) / 1e9:.2f} GB")
    else:
        doc[args.key] = entry_for(args.root)
        print(json.dumps({args.key: doc[args.key]}, indent=1))
    json.dump(doc, open(args.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
