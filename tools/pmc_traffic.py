#!/usr/bin/env python3
"""HBM traffic per kernel from a tools/gpu_pmc.sh run (FETCH_SIZE / WRITE_SIZE passes).

FETCH_SIZE and WRITE_SIZE are reported in KiB per dispatch.  On gfx950 FETCH_SIZE counts half
the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so reads are doubled;
WRITE_SIZE is taken as is.  Writes profiles/pmc_traffic.json for bench.py's roofline.traffic.

    python3 tools/pmc_traffic.py gpurun_out/pmc_<tag> <batch> [out.json]
"""
import collections
import csv
import glob
import json
import sys

root, batch = sys.argv[1], int(sys.argv[2])
out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/pass*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("rj::", "")
        if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]) * 1024.0)
res = {"source": root, "batch": batch,
       "method": "per dispatch: 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), mean over dispatches, / batch",
       "kernels": {}}
for k, c in sorted(vals.items()):
    if k.startswith("__amd") or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        continue
    fetch = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"]) * 2.0
    write = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
    res["kernels"][k] = {"fetch_bytes_per_launch": int(fetch), "write_bytes_per_launch": int(write),
                         "hbm_bytes_per_image": (fetch + write) / batch}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
