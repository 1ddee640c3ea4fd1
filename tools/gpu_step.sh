set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6y
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6y/suite.log 2>&1 || { tail -30 gpurun_out/r6y/suite.log; exit 1; }
tail -1 gpurun_out/r6y/suite.log
RJ_DEBUG_HOST=1 timeout -k 10 240 python3 bench.py --steps 10 --warmup 2 --runs 1 --no-cpu-baseline --no-extras > gpurun_out/r6y/bench_host.log 2>&1 || { tail -20 gpurun_out/r6y/bench_host.log; exit 1; }
grep "rj host" gpurun_out/r6y/bench_host.log | sed -n 8,11p
STEPS=10 bash tools/gpu_ab_env.sh par:- 
