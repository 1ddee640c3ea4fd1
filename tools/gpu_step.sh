set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
STEPS=10 bash tools/gpu_ab_env.sh c3:- c4:RJ_PLACE_CANDS=4
for f in c3_1 c4_1 c3_2 c4_2; do grep -o '"entry_placement": {[^}]*}' gpurun_out/ab/$f.log; done
