#!/usr/bin/env bash
# Same-box A/B of library builds: each arg "tag:libsuffix[:ENV=VAL,...]" (libsuffix "-" = the
# default build) runs a C2 bench (no extras, no CPU baselines); prints one summary line per tag.
set -o pipefail
mkdir -p gpurun_out/abl
for spec in "$@"; do
  IFS=':' read -r tag lib envs <<< "$spec"
  ( if [ "$lib" != "-" ]; then export RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_$lib.so; fi
    IFS=',' read -ra kvs <<< "$envs"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras ${BENCH_EXTRA:-} > gpurun_out/abl/$tag.log 2>&1 ) || exit $?
done
python3 - "$@" <<'PY'
import json, sys
for spec in sys.argv[1:]:
    tag = spec.split(':')[0]
    d = json.loads(open(f'gpurun_out/abl/{tag}.log').read().strip().splitlines()[-1])
    k = d['roofline']['per_kernel_launch_ms_sum']; h = d['huffman_detail']
    print(f"{tag:10s} {d['value']:9.0f} img/s {d['ms_per_step']:7.3f} ms  K1 {k.get('k_entropy',0)+k.get('k_huff',0)+k.get('k_huff_chunk',0):6.3f} K2 {k.get('k_rows',0):6.3f}  chunks {h['chunks']} split {h['split_intervals']}/{h.get('lean_split',0)} five {h.get('lean_five',0)} fb {h['serial_fallbacks']} hc {h.get('chunk_k1',0)}  parity {d['parity_timed_output']}")
PY
