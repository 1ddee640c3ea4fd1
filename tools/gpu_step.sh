set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6o
bash tools/gpu_ab_env.sh side0:RJ_UPLOAD_B_SIDE=0 side1:-
