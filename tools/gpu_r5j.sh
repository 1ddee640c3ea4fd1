set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_scan_gpu.py tests/test_threads_gpu.py tests/test_samples_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5j.log 2>&1 || { tail -30 gpurun_out/pytest_r5j.log; exit 1; }
tail -2 gpurun_out/pytest_r5j.log
rm -f gpurun_out/threads_r5j.txt gpurun_out/scan_r5j.txt
for cfg in "RJ_COALESCE_WAIT_US=300" "RJ_COALESCE_WAIT_US=300 RJ_COALESCE_INFLIGHT=2" "RJ_COALESCE_WAIT_US=1000" "RJ_COALESCE=0"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5j.txt 2>&1 || { cat gpurun_out/threads_r5j.txt; exit 1; }
done
grep threads gpurun_out/threads_r5j.txt
for us in 1 2 1 2; do
  echo "RJ_SCAN_UPLOAD_STREAMS=$us" >> gpurun_out/scan_r5j.txt
  RJ_SCAN_UPLOAD_STREAMS=$us timeout -k 10 300 python3 tools/scan_timing.py >> gpurun_out/scan_r5j.txt 2>&1 || exit $?
done
grep -E "UPLOAD|device parse|host parse" gpurun_out/scan_r5j.txt
timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/shapes_r5j.txt 2>&1 || exit $?
cat gpurun_out/shapes_r5j.txt
