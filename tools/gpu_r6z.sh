# timing probe: the entry streams' base shifted by 0 / 4 KB / 64 KB / 1 MB / 4 MB (RJ_EXP_ENT_SHIFT, entries)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh s0:- s4k:-:RJ_EXP_ENT_SHIFT=1024 s64k:-:RJ_EXP_ENT_SHIFT=16384 s1m:-:RJ_EXP_ENT_SHIFT=262144 s4m:-:RJ_EXP_ENT_SHIFT=1048576 s0b:-
