#!/usr/bin/env bash
# Round-5 evidence, part A (one GPU call): smoke, the GPU suite, the default bench line, and the
# rocprofv3 kernel trace + stats of the C2, c2nori and C5 benches.  Part B: gpu_evidence5b.sh.
set -o pipefail
TAG=${1:-r5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python3 bench.py --steps 20 > gpurun_out/bench_full_$TAG.log 2>&1 || { tail gpurun_out/bench_full_$TAG.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_full_$TAG.log
STEPS=10 bash tools/gpu_prof.sh $TAG || exit $?
STEPS=10 BENCH_EXTRA="--workload c2nori" bash tools/gpu_prof.sh ${TAG}_c2nori || exit $?
STEPS=3 BENCH_EXTRA="--workload c5 --runs 1" bash tools/gpu_prof.sh ${TAG}_c5 || exit $?
echo evidence-a done
