set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS=10 bash tools/gpu_ab_env.sh on:- off:RJ_PLACE_TUNE=0
for f in on_1 off_1 on_2 off_2; do grep -o '"entry_placement": {[^}]*}' gpurun_out/ab/$f.log; done
