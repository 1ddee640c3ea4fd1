# two-workgroup split instance: skip-walk tails (records without entry counts), 20 records: split tests, C4 and C2 A/B vs previous build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_batch_gpu.py tests/test_fuzz_gpu.py tests/test_decode_gpu.py \
  > gpurun_out/pytest_r6n.log 2>&1 || { tail -30 gpurun_out/pytest_r6n.log; exit 1; }
tail -2 gpurun_out/pytest_r6n.log
BENCH_EXTRA="--workload c4" bash tools/ab_lib.sh c4prev:prev c4new:- c4prev2:prev c4new2:- && \
bash tools/ab_lib.sh prev:prev new:- prev2:prev new2:- prev3:prev new3:-
