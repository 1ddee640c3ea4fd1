#!/usr/bin/env python3
"""HBM traffic per kernel from a tools/gpu_pmc.sh run (FETCH_SIZE / WRITE_SIZE passes).

FETCH_SIZE and WRITE_SIZE are reported in KiB per dispatch.  On gfx950 FETCH_SIZE counts half
the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so reads are doubled;
WRITE_SIZE is taken as is.  Per decode call over the whole batch (a k_destuff dispatch with the
largest grid and the dispatches up to the next k_destuff; DecodeSplit's part calls are left out) the
dispatches of each kernel are summed: k_entropy = the chunk/exact pass (k_entropy<false, *>), k_rows = both
K2 variants.  Writes profiles/pmc_traffic.json for bench.py's roofline.traffic.

    python3 tools/pmc_traffic.py gpurun_out/pmc_<tag> <batch> [out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys
import time

root, batch = sys.argv[1], int(sys.argv[2])
out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"


def group(name):
    n = name.split("(")[0].replace("void ", "").replace("rj::", "").strip()
    if n.startswith("k_entropy<false"):
        return "k_entropy"
    if n.startswith("k_rows_fix"):
        return "k_rows_fix"
    if n.startswith("k_rows<"):
        return "k_rows"
    return re.sub(r"<.*", "", n)


tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
calls = {}
for f in sorted(glob.glob(f"{root}/pass*/*counter_collection.csv")):
    p = f.split("/")[-2]
    rows = list(csv.DictReader(open(f)))
    # a call = a k_destuff dispatch and the dispatches after it up to the next one; only the calls
    # over the whole batch count (the largest K0 grid): DecodeSplit's part calls (the host-input
    # measurement) and smaller calls are other workloads
    first = {}
    for r in rows:
        first.setdefault(int(r["Dispatch_Id"]), r)
    k0_grid = max((int(r["Grid_Size"]) for r in first.values() if group(r["Kernel_Name"]) == "k_destuff"), default=0)
    keep, call_of, cur = set(), {}, None
    for d in sorted(first):
        r = first[d]
        if group(r["Kernel_Name"]) == "k_destuff":
            cur = d if int(r["Grid_Size"]) == k0_grid else None
            if cur is not None:
                keep.add(cur)
        call_of[d] = cur
    for r in rows:
        k = group(r["Kernel_Name"])
        c = r["Counter_Name"]
        d = int(r["Dispatch_Id"])
        if c in ("FETCH_SIZE", "WRITE_SIZE") and call_of.get(d) is not None:
            tot[k][(p, c)] += float(r["Counter_Value"]) * 1024.0
            disp[k][(p, c)].add(d)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        if any(r["Counter_Name"] == c for r in rows):
            calls[(p, c)] = len(keep)
res = {"source": root, "commit": os.environ.get("RJ_COMMIT", "?"), "date": time.strftime("%Y-%m-%d"),
       "batch": batch,
       "method": "per decode call: sum over the call's dispatches of 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes)",
       "kernels": {}}
for k in sorted(tot):
    if k.startswith("__amd"):
        continue
    fetch = [v / calls[pc] for pc, v in tot[k].items() if pc[1] == "FETCH_SIZE" and calls.get(pc)]
    write = [v / calls[pc] for pc, v in tot[k].items() if pc[1] == "WRITE_SIZE" and calls.get(pc)]
    if not fetch or not write:
        continue
    fb, wb = 2.0 * sum(fetch) / len(fetch), sum(write) / len(write)
    nd = max(len(ids) for pc, ids in disp[k].items()) / max(calls.values())
    res["kernels"][k] = {"fetch_bytes_per_call": int(fb), "write_bytes_per_call": int(wb),
                         "launches_per_call": nd, "hbm_bytes_per_image": (fb + wb) / batch}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
