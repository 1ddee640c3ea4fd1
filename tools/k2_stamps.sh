#!/usr/bin/env bash
# K2 phase split (stamps build) + the default bench A/B line, one GPU call.
set -o pipefail
mkdir -p gpurun_out/st
RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_stamps.so RJ_DEBUG_STAMPS=1 RJ_PIPE_GROUPS=1 timeout -k 10 300 \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras ${BENCH_EXTRA:-} > gpurun_out/st/stamps.log 2>&1 || exit $?
grep "rj stamps" gpurun_out/st/stamps.log | tail -1
STEPS=10 bash tools/ab_k1.sh "$@"
