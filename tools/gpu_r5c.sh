set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5d.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r5d.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 tools/scan_timing.py > gpurun_out/scan_r5d.txt 2>&1 || exit $?
cat gpurun_out/scan_r5d.txt
TAG=r5p3 bash tools/gpu_ab.sh base:nofast fast:- nopair:-:RJ_K1_PAIR=0 synthwin:synthwin synthload:synthload base2:nofast fast2:- nopair2:-:RJ_K1_PAIR=0 || exit $?
