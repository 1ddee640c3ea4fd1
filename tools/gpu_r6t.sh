# progressive K2 with its own register budget (3 waves per SIMD, no spills) vs the shared 4 (d4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_progressive_gpu.py \
  > gpurun_out/pytest_r6t.log 2>&1 || { tail -30 gpurun_out/pytest_r6t.log; exit 1; }
tail -2 gpurun_out/pytest_r6t.log
STEPS=4 BENCH_EXTRA="--workload c5 --runs 3" bash tools/ab_lib.sh d4:d4 d3:- d4b:d4 d3b:-
for t in d4 d3 d4b d3b; do python3 -c "
import json; d=json.loads(open('gpurun_out/abl/$t.log').read().strip().splitlines()[-1]); print('$t', d['value'], d['roofline']['per_kernel_launch_ms_sum'])"; done
