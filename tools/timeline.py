"""Print the kernel timeline of the last decode call from a rocprofv3 --kernel-trace CSV
(development aid for the pipelined launch)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{r['Kernel_Name'][:60]:60s} q={r.get('Queue_Id', r.get('Stream_Id', '?')):>4s} "
          f"start={s / 1e6:7.3f} end={e / 1e6:7.3f} dur={(e - s) / 1e6:6.3f} ms grid={r.get('Grid_Size', '?')}")
