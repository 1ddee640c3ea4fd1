# K2 of a split call in two launches (plain rows, then the split intervals' rows): GPU suite, A/B vs c7f3bf9
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_batch_gpu.py tests/test_decode_gpu.py tests/test_fuzz_gpu.py \
  > gpurun_out/pytest_r6q.log 2>&1 || { tail -30 gpurun_out/pytest_r6q.log; exit 1; }
tail -2 gpurun_out/pytest_r6q.log
bash tools/ab_lib.sh prev:prev new:- prev2:prev new2:- prev3:prev new3:- nos:-:RJ_K1_SPLIT5_T=0
