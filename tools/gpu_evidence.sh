#!/usr/bin/env bash
# The one evidence script for profiles/ (one GPU call per part; every step under its own time
# limit, the parts stop at the first failure):
#   tools/gpu_evidence.sh TAG suite   smoke(), the GPU test suite, the default bench line
#   tools/gpu_evidence.sh TAG prof    rocprofv3 kernel trace + stats of the C2, c2nori and C5 benches
#   tools/gpu_evidence.sh TAG pmc     HBM traffic passes (FETCH_SIZE, WRITE_SIZE: each its own
#                                     rocprofv3 run) for C2 and C5, and the SQ counter sets for C2
#   tools/gpu_evidence.sh TAG ab SPEC...   same-box A/B of handle settings (tools/gpu_ab_env.sh)
# Outputs under gpurun_out/; tools/bench_summary.py prints a bench line's headline numbers.
set -o pipefail
TAG=${1:?tag}
PART=${2:?part}
shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
case "$PART" in
  suite)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
    tail -1 gpurun_out/pytest_$TAG.log
    timeout -k 10 600 python3 bench.py --steps 20 > gpurun_out/bench_full_$TAG.log 2>&1 || { tail gpurun_out/bench_full_$TAG.log; exit 1; }
    python3 tools/bench_summary.py gpurun_out/bench_full_$TAG.log ;;
  prof)
    STEPS=10 bash tools/gpu_prof.sh $TAG || exit $?
    STEPS=10 BENCH_EXTRA="--workload c2nori" bash tools/gpu_prof.sh ${TAG}_c2nori || exit $?
    STEPS=3 BENCH_EXTRA="--workload c5 --runs 1" bash tools/gpu_prof.sh ${TAG}_c5 || exit $? ;;
  pmc)
    PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--steps 1 --warmup 1 --runs 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh traffic_$TAG || exit $?
    PMC_FILE=tools/pmc_sets_traffic.txt BENCH_ARGS="--workload c5 --steps 1 --warmup 1 --runs 1 --no-cpu-baseline --no-extras" bash tools/gpu_pmc.sh traffic_c5_$TAG || exit $?
    BENCH_ARGS="--runs 1" PMC_FILE=tools/pmc_sets_k2c.txt bash tools/pmc_run.sh sq_$TAG || exit $? ;;
  ab)
    bash tools/gpu_ab_env.sh "$@" || exit $? ;;
  *)
    echo "unknown part $PART"; exit 2 ;;
esac
echo "evidence $TAG $PART done"
