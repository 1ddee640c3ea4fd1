#!/usr/bin/env bash
# Round-5 evidence run (one GPU call): smoke, the GPU suite, the default bench line (CPU
# baselines, extra configs, call shapes), rocprofv3 kernel trace + stats of the C2, c2nori and C5
# benches, the HBM traffic passes (FETCH_SIZE, WRITE_SIZE: each its own rocprofv3 run) for C2 and
# C5, and the SQ counter sets for C2.  Every GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
TAG=${1:-r5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --steps 20 > gpurun_out/bench_full_$TAG.log 2>&1 || exit $?
STEPS=10 bash tools/gpu_prof.sh $TAG || exit $?
STEPS=10 BENCH_EXTRA="--workload c2nori" bash tools/gpu_prof.sh ${TAG}_c2nori || exit $?
STEPS=3 BENCH_EXTRA="--workload c5 --runs 1" bash tools/gpu_prof.sh ${TAG}_c5 || exit $?
PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--steps 1 --warmup 1 --runs 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh traffic_$TAG || exit $?
PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--workload c5 --steps 1 --warmup 1 --runs 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh traffic_c5_$TAG || exit $?
BENCH_ARGS="--runs 1" PMC_FILE=tools/pmc_sets_k2c.txt bash tools/pmc_run.sh sq_$TAG || exit $?
echo done
