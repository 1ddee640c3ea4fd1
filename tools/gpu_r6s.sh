# development: six decoder waves per CU in the lean split layout (RJ_K1_WAVES=6) vs five
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh w5:- w6t80:-:RJ_K1_WAVES=6 w6t70:-:RJ_K1_WAVES=6,RJ_K1_SPLIT5_T=0.7 w5b:- w6t80b:-:RJ_K1_WAVES=6 w6t70b:-:RJ_K1_WAVES=6,RJ_K1_SPLIT5_T=0.7
