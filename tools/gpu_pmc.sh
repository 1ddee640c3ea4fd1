#!/usr/bin/env bash
# PMC counter passes (each pass its own rocprofv3 run, kernel-trace only -- no sys/runtime
# trace) over a short bench; results under gpurun_out/pmc_$TAG/passN.
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --batch 256 --no-cpu-baseline}
i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d $OUT/pass$i -o pmc -- \
    python3 bench.py $ARGS > $OUT/pass$i.log 2>&1 || exit $?
done < "${PMC_FILE:-tools/pmc_sets.txt}"
