# split tails flagged when they may end early (K2's terminator check only for those): GPU suite,
# then A/B: C2 without / with the in-launch split, C4 (outlier split) previous build vs this one
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/pytest_r6m.log 2>&1 || { tail -30 gpurun_out/pytest_r6m.log; exit 1; }
tail -2 gpurun_out/pytest_r6m.log
bash tools/ab_lib.sh prev:prev nos:-:RJ_K1_SPLIT5_T=0 s80:- prev2:prev nos2:-:RJ_K1_SPLIT5_T=0 s80b:- && \
BENCH_EXTRA="--workload c4" bash tools/ab_lib.sh c4prev:prev c4new:- c4prev2:prev c4new2:-
