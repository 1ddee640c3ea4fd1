set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/shapes_r5r.txt
for cfg in "RJ_K1_HYP_CB_MUL=1" "RJ_K1_HYP_CB_MUL=2" "RJ_K1_HYP_CB_MUL=4"; do
  echo "== $cfg" >> gpurun_out/shapes_r5r.txt
  env $cfg SHAPES=16,32,64,128,256 timeout -k 10 180 python3 tools/shape_profile.py 384 >> gpurun_out/shapes_r5r.txt 2>&1 || { tail gpurun_out/shapes_r5r.txt; exit 1; }
done
grep -E "==|batch" gpurun_out/shapes_r5r.txt
rm -f gpurun_out/threads_r5r.txt
for cfg in "RJ_COALESCE_INFLIGHT=1" "RJ_COALESCE_INFLIGHT=2" "RJ_COALESCE_INFLIGHT=1" "RJ_COALESCE_INFLIGHT=2"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5r.txt 2>&1 || { cat gpurun_out/threads_r5r.txt; exit 1; }
done
grep threads gpurun_out/threads_r5r.txt
