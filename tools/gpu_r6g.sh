# C2 with the lean outlier split at higher thresholds (only the longest intervals split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh def:- t70:-:RJ_SPLIT_OUTLIER_T=0.7,RJ_SPLIT_OUTLIER_FRAC=1.0 t80:-:RJ_SPLIT_OUTLIER_T=0.8,RJ_SPLIT_OUTLIER_FRAC=1.0 \
  t88:-:RJ_SPLIT_OUTLIER_T=0.88,RJ_SPLIT_OUTLIER_FRAC=1.0 def2:- t80b:-:RJ_SPLIT_OUTLIER_T=0.8,RJ_SPLIT_OUTLIER_FRAC=1.0
