#!/usr/bin/env bash
# Counter passes (one rocprofv3 run per line of $PMC_FILE) over a short C2 bench; summary per
# kernel into gpurun_out/pmc_$TAG.txt.  Development aid.
set -o pipefail
TAG=${1:-run}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT; i=0
while IFS= read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d $OUT/pass$i -o pmc -- \
    python3 bench.py --steps 1 --warmup 1 --no-extras --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/pass$i.log 2>&1 || exit $?
done < "${PMC_FILE:-tools/pmc_sets_k2c.txt}"
python3 tools/pmc_summary.py $OUT > gpurun_out/pmc_$TAG.txt
