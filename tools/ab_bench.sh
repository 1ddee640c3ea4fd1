#!/usr/bin/env bash
# A/B bench runs on the GPU box: each argument is "tag:ENV=VAL,ENV2=VAL2" (empty env list ok).
# Every run has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
STEPS=${STEPS:-10}
for spec in "$@"; do
  tag=${spec%%:*}
  envs=${spec#*:}
  ( IFS=',' read -ra kvs <<< "$envs"
    for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline ${BENCH_EXTRA:-} > gpurun_out/ab_$tag.log 2>&1 ) || exit $?
done
