#!/usr/bin/env bash
# Round-5 evidence, part B (one GPU call): the HBM traffic passes (FETCH_SIZE, WRITE_SIZE, each its
# own rocprofv3 run) for C2 and C5, and the SQ counter sets for C2.
set -o pipefail
TAG=${1:-r5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--steps 1 --warmup 1 --runs 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh traffic_$TAG || exit $?
PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--workload c5 --steps 1 --warmup 1 --runs 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh traffic_c5_$TAG || exit $?
BENCH_ARGS="--runs 1" PMC_FILE=tools/pmc_sets_k2c.txt bash tools/pmc_run.sh sq_$TAG || exit $?
echo evidence-b done
