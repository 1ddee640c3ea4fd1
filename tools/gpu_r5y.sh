set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r5p17 bash tools/gpu_ab.sh base:- ntwin:ntwin base2:- ntwin2:ntwin || exit $?
