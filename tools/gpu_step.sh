set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6x
for k in 1 2 3 4; do
  for mode in on off; do
    if [ $mode = off ]; then export RJ_PLACE_TUNE=0; else unset RJ_PLACE_TUNE; fi
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r6x/${mode}_$k.log 2>&1 || { tail -5 gpurun_out/r6x/${mode}_$k.log; exit 1; }
    echo "== $mode $k"; python3 tools/bench_summary.py gpurun_out/r6x/${mode}_$k.log | head -1 | cut -c1-110; grep -o '"entry_placement": {[^}]*}' gpurun_out/r6x/${mode}_$k.log
  done
done
