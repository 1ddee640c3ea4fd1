# in-launch split of the longest intervals (default RJ_K1_SPLIT5_T=0.8): the GPU suite, then A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/pytest_r6k.log 2>&1 || { tail -30 gpurun_out/pytest_r6k.log; exit 1; }
tail -2 gpurun_out/pytest_r6k.log
bash tools/ab_lib.sh nos:-:RJ_K1_SPLIT5_T=0 s80:- s70:-:RJ_K1_SPLIT5_T=0.7 nos2:-:RJ_K1_SPLIT5_T=0 s80b:- s82:-:RJ_K1_SPLIT5_T=0.82
