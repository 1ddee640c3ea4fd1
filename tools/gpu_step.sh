set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6o
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6o/suite.log 2>&1 || { tail -30 gpurun_out/r6o/suite.log; exit 1; }
tail -3 gpurun_out/r6o/suite.log
bash tools/gpu_ab_env.sh k0old:RJ_K0_LDS=0 k0lds:-
