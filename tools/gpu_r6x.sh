# K0 destuff blocks of 4 KB (ds4) vs 2 KB (default): C2 and c2nori, same box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib.sh b2:- b4:ds4 b2b:- b4b:ds4 && \
BENCH_EXTRA="--workload c2nori" bash tools/ab_lib.sh nb2:- nb4:ds4
for t in b2 b4 b2b b4b nb2 nb4; do python3 -c "
import json; d=json.loads(open('gpurun_out/abl/$t.log').read().strip().splitlines()[-1]); print('$t', d['value'], d['roofline']['per_kernel_launch_ms_sum'].get('k_destuff'))"; done
