# plain K2 at 3 waves per SIMD (p3) vs 4 (default), C2 and c2nori
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh o4:- p3:p3 o4b:- p3b:p3 && \
BENCH_EXTRA="--workload c2nori" bash tools/ab_lib.sh no4:- np3:p3
