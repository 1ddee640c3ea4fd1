set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG:-r5b}.log 2>&1 || exit $?
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG:-r5b}.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/bench_full_${TAG:-r5b}.log 2>&1 || exit $?
echo done
