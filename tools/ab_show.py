"""Summarise gpurun_out/ab_*.log bench lines (tools/ab_bench.sh)."""
import glob
import json
import sys

for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st = d["stages_ms_per_step"]
            print(f"{f[14:-4]:14s} {d['value']:10.1f} img/s {d['ms_per_step']:7.3f} ms | " +
                  " ".join(f"{k[:-3]}={v:.3f}" for k, v in st.items()))
