set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6t
timeout -k 10 400 python3 -u -m pytest tests/test_batch_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6t/tests.log 2>&1 || { tail -30 gpurun_out/r6t/tests.log; exit 1; }
tail -1 gpurun_out/r6t/tests.log
STEPS=10 bash tools/gpu_ab_env.sh k2side:- k2seq:RJ_K2_SPLIT_SIDE=0
for f in k2side_1 k2seq_1 k2side_2 k2seq_2; do grep -o '"entry_placement": {[^}]*}' gpurun_out/ab/$f.log; done
