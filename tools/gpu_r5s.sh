set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=6 BENCH_EXTRA="--workload c5 --runs 1" TAG=r5p10 bash tools/gpu_ab.sh base:- prio3:prio3 prio1:prio1 base2:- prio3b:prio3 || exit $?
