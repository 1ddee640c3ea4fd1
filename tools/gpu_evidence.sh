#!/usr/bin/env bash
# Measurement evidence for profiles/: default bench (with CPU baselines), rocprofv3 kernel
# trace + stats of the same bench command, and the FETCH_SIZE/WRITE_SIZE PMC passes.
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || exit $?
STEPS=10 bash tools/gpu_prof.sh $TAG || exit $?
PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh $TAG || exit $?
echo done
