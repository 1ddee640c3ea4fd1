#!/usr/bin/env bash
# K1 time per image vs batch (occupancy) for the exact and lean kernels, one K1 launch per call
# (RJ_PIPE_GROUPS=1).  Development aid: gpurun_out/occ/<variant>_<batch>.log
set -o pipefail
mkdir -p gpurun_out/occ
export RJ_PIPE_GROUPS=1
for v in old lean; do
  for b in ${BATCHES:-256 1024 2048}; do
    RJ_LEAN=$([ $v = lean ] && echo 1 || echo 0) timeout -k 10 200 python bench.py --steps 5 --warmup 1 --batch $b \
      --no-cpu-baseline --no-extras > gpurun_out/occ/${v}_$b.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/occ/*.log')):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d['roofline']['per_kernel_launch_ms_sum']; n = d['config']['batch_per_gpu']
    k1 = k.get('k_entropy', 0) + k.get('k_huff', 0)
    print(f"{f.split('/')[-1]:16s} {d['value']:9.0f} img/s  K1 {k1:7.3f} ms = {k1/n*1e3:6.2f} us/img  K2 {k.get('k_rows',0):6.3f}  parity {d['parity_timed_output']}")
PY
