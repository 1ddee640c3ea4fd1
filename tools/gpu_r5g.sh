set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r5p6 bash tools/gpu_ab.sh base:- pf4:pf4 pf8:pf8 pf16:pf16 base2:- pf8b:pf8 pf16b:pf16 || exit $?
timeout -k 10 600 python3 bench.py --steps 20 > gpurun_out/bench_r5g.json 2> gpurun_out/bench_r5g.err || exit $?
python3 tools/bench_summary.py gpurun_out/bench_r5g.json || true
