"""Print the headline numbers of a bench.py JSON line (file argument: a log holding the line)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    r = d["roofline"]
    print(f"value {d['value']:.0f} img/s  ms/step {d['ms_per_step']}  dominant {r['kernel']} {r['avg_launch_ms']} ms "
          f"frac {r['frac']}  kernels {r['per_kernel_launch_ms_sum']}")
    print("  host_input", d.get("host_input_images_per_s_per_gpu"), " stages", d.get("stages_ms_per_step"))
    if "live_rows" in d:
        print("  live", d["live_rows"], " placement", d.get("entry_placement"), " parity", d.get("parity_timed_output"))
    for k, v in d.get("extra_workloads", {}).items():
        print(f"  {k}: {v['value']:.0f} img/s  {v['ms_per_step']} ms  {v.get('per_kernel_launch_ms_sum')}  parity {v.get('parity_sample')}")
