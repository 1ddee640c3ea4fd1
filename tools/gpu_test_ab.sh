#!/usr/bin/env bash
# GPU tests (one process, per-test timeouts) then a same-box A/B of library builds (tools/ab_lib.sh
# specs in $AB, default: the HEAD build vs the working tree).  Development aid.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pt_ab.log 2>&1
rc=$?; tail -5 gpurun_out/pt_ab.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab_lib.sh ${AB:-base:base new:-}
