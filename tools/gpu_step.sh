set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS=10 BENCH_EXTRA="--runs 1" bash tools/gpu_ab_env.sh p3noside:RJ_UPLOAD_B_SIDE=0 p3notune:RJ_PLACE_TUNE=0 p3:-
