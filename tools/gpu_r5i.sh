set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5i.log 2>&1 || { tail -30 gpurun_out/pytest_r5i.log; exit 1; }
tail -2 gpurun_out/pytest_r5i.log
rm -f gpurun_out/threads_r5i.txt
for cfg in "RJ_COALESCE_WAIT_US=300" "RJ_COALESCE_WAIT_US=300 RJ_COALESCE_INFLIGHT=2" "RJ_COALESCE_WAIT_US=1000" "RJ_COALESCE=0"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5i.txt 2>&1 || { cat gpurun_out/threads_r5i.txt; exit 1; }
done
grep threads gpurun_out/threads_r5i.txt
timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/shapes_r5i.txt 2>&1 || exit $?
cat gpurun_out/shapes_r5i.txt
