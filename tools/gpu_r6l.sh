# split tails' pieces start at their recorded entry (no K2 skip walk): split-path GPU tests, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_batch_gpu.py tests/test_decode_gpu.py tests/test_fuzz_gpu.py \
  > gpurun_out/pytest_r6l.log 2>&1 || { tail -30 gpurun_out/pytest_r6l.log; exit 1; }
tail -2 gpurun_out/pytest_r6l.log
bash tools/ab_lib.sh nos:-:RJ_K1_SPLIT5_T=0 s80:- nos2:-:RJ_K1_SPLIT5_T=0 s80b:- nos3:-:RJ_K1_SPLIT5_T=0 s80c:-
