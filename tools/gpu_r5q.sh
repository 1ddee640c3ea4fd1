set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5q.log 2>&1 || { tail -40 gpurun_out/pytest_r5q.log; exit 1; }
tail -2 gpurun_out/pytest_r5q.log
rm -f gpurun_out/shapes_r5q.txt
for cfg in "RJ_K1_HYP=6" "RJ_K1_HYP=1"; do
  echo "== $cfg" >> gpurun_out/shapes_r5q.txt
  env $cfg SHAPES=1,4,8,16,32,128 timeout -k 10 180 python3 tools/shape_profile.py 384 >> gpurun_out/shapes_r5q.txt 2>&1 || { tail gpurun_out/shapes_r5q.txt; exit 1; }
done
grep -E "==|batch" gpurun_out/shapes_r5q.txt
rm -f gpurun_out/threads_r5q.txt
for cfg in "RJ_K1_HYP=6" "RJ_K1_HYP=6 RJ_COALESCE_INFLIGHT=2"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5q.txt 2>&1 || { cat gpurun_out/threads_r5q.txt; exit 1; }
done
grep threads gpurun_out/threads_r5q.txt
