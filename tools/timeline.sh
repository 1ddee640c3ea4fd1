#!/usr/bin/env bash
# Pipelined-launch timeline (RJ_DEBUG_K1: per class K1 / K2 start and end, ms after K0) for the
# env variants given as args ("tag:ENV=V,..."); development aid.
set -o pipefail
mkdir -p gpurun_out/tl
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  ( IFS=',' read -ra kvs <<< "$envs"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && export "$kv"; done
    RJ_DEBUG_K1=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/tl/$tag.log 2>&1 ) || exit $?
  echo "== $tag"; grep "\[rj\] class" gpurun_out/tl/$tag.log | tail -${GROUPS_SHOWN:-2}
done
