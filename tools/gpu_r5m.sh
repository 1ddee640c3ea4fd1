set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5m.log 2>&1 || { tail -40 gpurun_out/pytest_r5m.log; exit 1; }
tail -2 gpurun_out/pytest_r5m.log
for hy in 6 1; do
  RJ_K1_HYP=$hy RJ_DEBUG_K1=1 SHAPES=1,8,16,128 timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/shapes_r5m_h$hy.txt 2>&1 || { tail gpurun_out/shapes_r5m_h$hy.txt; exit 1; }
  echo "== RJ_K1_HYP=$hy"; grep -E "batch|\[K1\]" gpurun_out/shapes_r5m_h$hy.txt
done
rm -f gpurun_out/threads_r5m.txt
for cfg in "RJ_COALESCE_INFLIGHT=1" "RJ_COALESCE_INFLIGHT=2" "RJ_COALESCE_INFLIGHT=1 RJ_K1_HYP=1"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5m.txt 2>&1 || { cat gpurun_out/threads_r5m.txt; exit 1; }
done
grep threads gpurun_out/threads_r5m.txt
BENCH_EXTRA="--workload c2nori" TAG=r5p7 bash tools/gpu_ab.sh prev:prev hyp:- prev2:prev hyp2:- || exit $?
STEPS=6 BENCH_EXTRA="--workload c5" TAG=r5p8 bash tools/gpu_ab.sh prev:prev dcref:- prev2:prev dcref2:- || exit $?
