#!/usr/bin/env bash
# One GPU call: same-box A/B of library builds (tools/ab_lib.sh specs), output to gpurun_out/ab_$TAG.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/ab_lib.sh "$@" > gpurun_out/ab_${TAG:-x}.txt 2>&1
rc=$?
cat gpurun_out/ab_${TAG:-x}.txt
exit $rc
