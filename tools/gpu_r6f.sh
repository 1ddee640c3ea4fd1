# lean K1 with the lookup issued before the entry work (sched barrier) and the escape settled in
# its block: stamps, then same-box A/B against the previous build (C2, c2nori)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hl
for v in basest newst; do
  RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_$v.so RJ_DEBUG_STAMPS=1 timeout -k 10 200 python bench.py --steps 2 --warmup 0 --runs 1 --no-cpu-baseline --no-extras > gpurun_out/hl/$v.log 2>&1 || exit $?
  echo "== $v"; grep "rj k_huff" gpurun_out/hl/$v.log | tail -3
done
bash tools/ab_lib.sh base:base new:- base2:base new2:- && \
BENCH_EXTRA="--workload c2nori" bash tools/ab_lib.sh nbase:base nnew:- nbase2:base nnew2:-
