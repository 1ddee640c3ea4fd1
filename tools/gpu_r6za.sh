# timing probe: interval entry regions reserved at 16 / 12 entries per byte vs 8 (default)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh e8:- e12:e12 e16:e16 e8b:- e12b:e12 e16b:e16 && \
BENCH_EXTRA="--workload c4" bash tools/ab_lib.sh c4e8:- c4e16:e16
