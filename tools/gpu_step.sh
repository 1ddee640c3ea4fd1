set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6z
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z/smoke.log 2>&1 || { cat gpurun_out/r6z/smoke.log; exit 1; }
tail -1 gpurun_out/r6z/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6z/suite.log 2>&1 || { tail -30 gpurun_out/r6z/suite.log; exit 1; }
tail -1 gpurun_out/r6z/suite.log
timeout -k 10 300 python3 bench.py --steps 10 --no-cpu-baseline --no-extras > gpurun_out/r6z/bench.log 2>&1 || { tail -20 gpurun_out/r6z/bench.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/r6z/bench.log
