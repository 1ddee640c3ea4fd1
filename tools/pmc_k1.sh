#!/usr/bin/env bash
# K1 counter passes (SQ sets of tools/pmc_sets_sq.txt) on a C2 bench with K1 and K2 as single
# sequential launches (RJ_PIPE_GROUPS=1), lean (RJ_LEAN=1) and old (default) kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_k1_${1:-run}
mkdir -p $OUT
export RJ_PIPE_GROUPS=1
for variant in lean old; do
  if [ $variant = old ]; then export RJ_LEAN=0; else export RJ_LEAN=1; fi
  i=0; mkdir -p $OUT/$variant
  while IFS= read -r counters; do
    [ -z "$counters" ] && continue
    case "$counters" in FETCH_SIZE*|WRITE_SIZE*) continue;; esac
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d $OUT/$variant/pass$i -o pmc -- \
      python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > $OUT/$variant/pass$i.log 2>&1 || exit $?
  done < tools/pmc_sets_sq.txt
  python3 tools/pmc_summary.py $OUT/$variant > $OUT/$variant.txt
done
