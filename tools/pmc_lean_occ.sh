#!/usr/bin/env bash
# SQ counters of the lean K1 (RJ_LEAN=1, one K1 launch per call) at two batch sizes (occupancy).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export RJ_PIPE_GROUPS=1 RJ_LEAN=${RJ_LEAN:-1}
for b in ${BATCHES:-1024 2048}; do
  OUT=gpurun_out/pmc_occ/b$b; mkdir -p $OUT; i=0
  while IFS= read -r counters; do
    [ -z "$counters" ] && continue
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d $OUT/pass$i -o pmc -- \
      python3 bench.py --steps 1 --warmup 1 --batch $b --no-extras --no-cpu-baseline > $OUT/pass$i.log 2>&1 || exit $?
  done < tools/pmc_sets_sq.txt
  python3 tools/pmc_summary.py $OUT | grep -i "huff\|entropy" > gpurun_out/pmc_occ/b$b.txt
done
