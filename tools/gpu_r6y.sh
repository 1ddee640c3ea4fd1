# timing probe: interval entry regions reserved at 4 / 2 entries per byte (e4 / e2, unsafe for arbitrary
# tables; C2's standard tables spend >= 2 bits per entry) vs 8 (default): does the density of the
# K1 -> K2 intermediate matter (pages / TLB reach)?  The parity check of each line says whether e2 overflowed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh e8:- e4:e4 e2:e2 e8b:- e4b:e4 e2b:e2
