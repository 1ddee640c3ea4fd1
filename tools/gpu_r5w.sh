set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r5p15 bash tools/gpu_ab.sh g1:- g2:-:RJ_PIPE_GROUPS=2 g3:-:RJ_PIPE_GROUPS=3 g1b:- g2b:-:RJ_PIPE_GROUPS=2 || exit $?
STEPS=6 BENCH_EXTRA="--workload c5 --runs 1" TAG=r5p16 bash tools/gpu_ab.sh base:- dcprio:dcprio base2:- dcprio2:dcprio || exit $?
