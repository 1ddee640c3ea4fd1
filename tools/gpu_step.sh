set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6s
timeout -k 10 400 python3 -u -m pytest tests/test_batch_gpu.py -m gpu -x -q -k "placement or host_streams" --timeout 200 --timeout-method thread > gpurun_out/r6s/tests.log 2>&1 || { tail -30 gpurun_out/r6s/tests.log; exit 1; }
tail -2 gpurun_out/r6s/tests.log
RJ_DEBUG_HOST=1 timeout -k 10 240 python3 bench.py --steps 10 --warmup 2 --runs 1 --no-cpu-baseline --no-extras > gpurun_out/r6s/bench_host.log 2>&1 || { tail -20 gpurun_out/r6s/bench_host.log; exit 1; }
grep "rj host\|rj call" gpurun_out/r6s/bench_host.log | sed -n 10,24p
bash tools/gpu_evidence.sh r6c pmc
