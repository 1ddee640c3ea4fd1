#!/usr/bin/env bash
# GPU-box check run: smoke -> pytest -m gpu -> short bench.  Every GPU step has its own time
# limit and the chain stops at the first crash/timeout (exit >= 124 or signal).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --batch 256 --no-cpu-baseline} > gpurun_out/bench_$TAG.log 2>&1
