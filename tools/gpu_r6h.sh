# lean K1 with five decoder waves per CU (C2's overflow intervals as fifth waves): the batch
# GPU tests, then same-box A/B against the two-round layout (RJ_K1_FIVE=0)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_batch_gpu.py \
  > gpurun_out/pytest_r6h.log 2>&1 || { tail -30 gpurun_out/pytest_r6h.log; exit 1; }
tail -2 gpurun_out/pytest_r6h.log
bash tools/ab_lib.sh two:-:RJ_K1_FIVE=0 five:- two2:-:RJ_K1_FIVE=0 five2:- two3:-:RJ_K1_FIVE=0 five3:-
