#!/usr/bin/env bash
# Same-box A/B of handle settings: each arg "tag:ENV=VAL,ENV=VAL" (or "tag:-") runs a C2 bench
# (no extras, no CPU baseline) with those variables; the list runs twice (ABAB) and one summary
# line per run is printed.  BENCH_EXTRA adds bench arguments, STEPS the timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for pass in 1 2; do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    ( if [ "$envs" != "-" ]; then IFS=',' read -ra kvs <<< "$envs"; for kv in "${kvs[@]}"; do export "$kv"; done; fi
      timeout -k 10 240 python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras ${BENCH_EXTRA:-} \
        > gpurun_out/ab/${tag}_$pass.log 2>&1 ) || { tail -5 gpurun_out/ab/${tag}_$pass.log; exit 1; }
    echo "== $tag pass $pass"; python3 tools/bench_summary.py gpurun_out/ab/${tag}_$pass.log
  done
done
