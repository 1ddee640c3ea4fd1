set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6u
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6u/suite.log 2>&1 || { tail -30 gpurun_out/r6u/suite.log; exit 1; }
tail -1 gpurun_out/r6u/suite.log
STEPS=10 BENCH_EXTRA="--runs 3" bash tools/gpu_ab_env.sh k0new:- k0old:RJ_LIB_PATH=/root/repo/rocjpeg_amd/librocjpeg_amd_prev.so
