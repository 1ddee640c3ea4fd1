set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6v
RJ_K2_LPT=1 timeout -k 10 400 python3 -u -m pytest tests/test_batch_gpu.py tests/test_decode_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6v/tests.log 2>&1 || { tail -30 gpurun_out/r6v/tests.log; exit 1; }
tail -1 gpurun_out/r6v/tests.log
STEPS=10 bash tools/gpu_ab_env.sh lpt:RJ_K2_LPT=1 img:-
