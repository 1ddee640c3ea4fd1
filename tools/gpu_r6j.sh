# five-wave lean layout with the longest intervals split in the same launch (RJ_K1_SPLIT5_T)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh f:- s90:-:RJ_K1_SPLIT5_T=0.9 s85:-:RJ_K1_SPLIT5_T=0.85 s80:-:RJ_K1_SPLIT5_T=0.8 \
  f2:- s90b:-:RJ_K1_SPLIT5_T=0.9 s85b:-:RJ_K1_SPLIT5_T=0.85 s80b:-:RJ_K1_SPLIT5_T=0.8
