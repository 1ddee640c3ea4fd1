set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
STEPS=6 BENCH_EXTRA="--workload c5 --runs 1" TAG=r5p11 bash tools/gpu_ab.sh pm1:- pm0:pm0 pm2:pm2 pm3:pm3 pm1b:- pm3b:pm3 || exit $?
