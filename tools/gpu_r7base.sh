set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6base
for k in 1 2; do timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r6base/bench$k.log 2>&1 || exit $?; done
python3 tools/bench_summary.py gpurun_out/r6base/bench1.log; python3 tools/bench_summary.py gpurun_out/r6base/bench2.log
