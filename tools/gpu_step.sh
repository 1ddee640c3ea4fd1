set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6l
timeout -k 10 300 python3 -u -m pytest tests/test_batch_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6l/pytest.log 2>&1 || { tail -30 gpurun_out/r6l/pytest.log; exit 1; }
tail -1 gpurun_out/r6l/pytest.log
STEPS=10 bash tools/gpu_ab_env.sh eff0:RJ_K1_LPT_EFF=0 eff1:-
