set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r5n.log 2>&1 || { tail -40 gpurun_out/pytest_r5n.log; exit 1; }
tail -2 gpurun_out/pytest_r5n.log
for cfg in "RJ_K1_HYP_WARM=0" "RJ_K1_HYP_WARM=1" "RJ_K1_HYP=1"; do
  env $cfg RJ_DEBUG_K1=1 SHAPES=1,8,16,32,64 timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/shapes_r5n.txt 2>&1 || { tail gpurun_out/shapes_r5n.txt; exit 1; }
  echo "== $cfg"; grep -E "batch|\[K1\]" gpurun_out/shapes_r5n.txt
done
rm -f gpurun_out/threads_r5n.txt
for cfg in "RJ_K1_HYP_WARM=0" "RJ_K1_HYP_WARM=1"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5n.txt 2>&1 || { cat gpurun_out/threads_r5n.txt; exit 1; }
done
grep threads gpurun_out/threads_r5n.txt
BENCH_EXTRA="--workload c2nori" TAG=r5p9 bash tools/gpu_ab.sh prev:prev cur:- prev2:prev cur2:- || exit $?
