#!/usr/bin/env python3
"""Per-call GPU idle gaps from a rocprofv3 kernel trace of bench.py (development aid).

A call is K0 (k_destuff) -> K1 (k_huff / k_entropy) -> K2 (k_rows) in launch order; for each one
prints the idle time since the previous call's K2 ended, the K0 -> K1 and K1 -> K2 gaps and the
call's span.  Usage: trace_gaps.py <prof_kernel_trace.csv> [max_calls]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    prev_end, i, n = None, 0, 0
    print("call  idle_before_K0_us  K0->K1_us  K1->K2_us  span_us  other kernels since the last call")
    while i + 2 < len(ev) and n < limit:
        s, e, name = ev[i]
        k1, k2 = ev[i + 1], ev[i + 2]
        if "k_destuff" in name and ("k_huff" in k1[2] or "k_entropy" in k1[2]) and "k_rows" in k2[2]:
            other = [x[2].split("(")[0][:24] for x in ev[max(0, i - 4):i] if prev_end is not None and x[0] >= prev_end]
            idle = (s - prev_end) / 1e3 if prev_end is not None else float("nan")
            print(f"{n:4d}  {idle:17.1f}  {(k1[0] - e) / 1e3:9.1f}  {(k2[0] - k1[1]) / 1e3:9.1f}  "
                  f"{(k2[1] - s) / 1e3:7.1f}  {' '.join(other)}")
            prev_end, i, n = k2[1], i + 3, n + 1
            while i < len(ev) and "k_rows" in ev[i][2]:  # the call's other K2 launches (split-aware, fix-up)
                prev_end, i = ev[i][1], i + 1
            continue
        i += 1


if __name__ == "__main__":
    main()
