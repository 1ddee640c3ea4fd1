# five-wave lean layout: plain (1) vs reversed hosting workgroups (2, default) vs two rounds (0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_batch_gpu.py -k "c2_1024" \
  > gpurun_out/pytest_r6i.log 2>&1 || { tail -30 gpurun_out/pytest_r6i.log; exit 1; }
tail -1 gpurun_out/pytest_r6i.log
bash tools/ab_lib.sh two:-:RJ_K1_FIVE=0 f1:-:RJ_K1_FIVE=1 f2:- two2:-:RJ_K1_FIVE=0 f1b:-:RJ_K1_FIVE=1 f2b:- two3:-:RJ_K1_FIVE=0 f1c:-:RJ_K1_FIVE=1 f2c:-
