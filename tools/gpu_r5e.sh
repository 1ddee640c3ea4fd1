set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5e.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r5e.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 tools/scan_timing.py > gpurun_out/scan_r5e.txt 2>&1 || exit $?
cat gpurun_out/scan_r5e.txt
TAG=r5p4 bash tools/gpu_ab.sh base:- l2store:l2store nofast:nofast base2:- l2store2:l2store || exit $?
