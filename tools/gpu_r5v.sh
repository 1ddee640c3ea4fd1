set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r5p13 bash tools/gpu_ab.sh base:- dprio:dprio2 base2:- dprio2:dprio2 || exit $?
BENCH_EXTRA="--workload c2nori" TAG=r5p14 bash tools/gpu_ab.sh base:- dprio:dprio2 base2:- dprio2:dprio2 || exit $?
