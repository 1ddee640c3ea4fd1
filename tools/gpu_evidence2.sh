#!/usr/bin/env bash
# Evidence run: default bench (CPU baselines, extras), rocprofv3 kernel trace + stats of the C2
# bench, FETCH/WRITE_SIZE traffic passes, and the SQ counter sets of tools/pmc_sets_k2c.txt.
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full_$TAG.log 2>&1 || exit $?
STEPS=10 bash tools/gpu_prof.sh $TAG || exit $?
PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh $TAG || exit $?
PMC_FILE=tools/pmc_sets_k2c.txt bash tools/pmc_run.sh sq_$TAG || exit $?
echo done
