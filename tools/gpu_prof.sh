#!/usr/bin/env bash
# Profiling run on the GPU box: kernel trace + stats of a short bench (rocprofv3), output
# under gpurun_out/prof_$TAG.  Counters (--pmc) run separately (gpu_pmc.sh).
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o prof -- \
  python3 bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-extras ${BENCH_EXTRA:-} > gpurun_out/prof_$TAG/bench.log 2>&1
