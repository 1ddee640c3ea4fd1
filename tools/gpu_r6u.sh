# split-aware K2 with a 3-waves-per-SIMD budget (s3: no spills) vs 4 (default: spills), C2 and C4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh o4:- s3:s3 o4b:- s3b:s3 && \
BENCH_EXTRA="--workload c4" bash tools/ab_lib.sh c4o4:- c4s3:s3 c4o4b:- c4s3b:s3
