set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5c.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r5c.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 tools/scan_timing.py > gpurun_out/scan_r5c.txt 2>&1 || exit $?
cat gpurun_out/scan_r5c.txt
TAG=r5p2 bash tools/gpu_ab.sh base:nofast fast:- nocont:nocont lds14:lds14 lds13:lds13 stag1:stag1 stag3:stag3 base2:nofast fast2:- || exit $?
