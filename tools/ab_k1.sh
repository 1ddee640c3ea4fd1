#!/usr/bin/env bash
# Same-box A/B of the K1 variants: each spec "tag:ENV=VAL,..." runs bench.py (C2, no extras).
set -o pipefail
mkdir -p gpurun_out/ab
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  ( IFS=',' read -ra kvs <<< "$envs"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/ab/$tag.log 2>&1 ) || exit $?
done
python3 - "$@" <<'PY'
import json, sys
for spec in sys.argv[1:]:
    tag = spec.split(':')[0]
    d = json.loads(open(f'gpurun_out/ab/{tag}.log').read().strip().splitlines()[-1])
    k = d['roofline']['per_kernel_launch_ms_sum']
    print(f"{tag:14s} {d['value']:10.0f} img/s  {d['ms_per_step']:7.3f} ms  K1 {k.get('k_entropy',0)+k.get('k_huff',0):6.3f}  K2 {k.get('k_rows',0):6.3f}  parity {d['parity_timed_output']}")
PY
