set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=6 BENCH_EXTRA="--workload c5 --runs 1" TAG=r5p12 bash tools/gpu_ab.sh pm1:- pm4:pm4 pm5:pm5 pm0:pm0 pm1b:- pm4b:pm4 pm5b:pm5 || exit $?
