set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6q
timeout -k 10 400 python3 -u -m pytest tests/test_batch_gpu.py tests/test_decode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6q/tests.log 2>&1 || { tail -30 gpurun_out/r6q/tests.log; exit 1; }
tail -2 gpurun_out/r6q/tests.log
STEPS=10 bash tools/gpu_ab_env.sh off:RJ_PLACE_TUNE=0 on:- off2:RJ_PLACE_TUNE=0 on2:-
