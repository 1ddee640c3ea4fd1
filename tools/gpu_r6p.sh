# K1 zero-fills a split tail that stopped short (K2 without the terminator check: no spills in
# the split instance): GPU suite, then A/B vs the previous commit (C2, C4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/pytest_r6p.log 2>&1 || { tail -30 gpurun_out/pytest_r6p.log; exit 1; }
tail -2 gpurun_out/pytest_r6p.log
bash tools/ab_lib.sh prev:prev new:- prev2:prev new2:- prev3:prev new3:- && \
BENCH_EXTRA="--workload c4" bash tools/ab_lib.sh c4prev:prev c4new:- c4prev2:prev c4new2:-
