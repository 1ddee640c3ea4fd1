set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/st
timeout -k 10 120 python3 tools/h2d_probe.py > gpurun_out/h2d_r5h.txt 2>&1 || exit $?
cat gpurun_out/h2d_r5h.txt
RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_stamps.so RJ_DEBUG_STAMPS=1 timeout -k 10 300 \
  python3 bench.py --steps 3 --warmup 1 --runs 1 --no-cpu-baseline --no-extras > gpurun_out/st/stamps_r5h.log 2>&1 || exit $?
grep "rj stamps" gpurun_out/st/stamps_r5h.log | tail -3
for cfg in "RJ_COALESCE_WAIT_US=0" "RJ_COALESCE_WAIT_US=300" "RJ_COALESCE_WAIT_US=300 RJ_COALESCE_INFLIGHT=2" "RJ_COALESCE=0"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5h.txt 2>&1 || exit $?
done
cat gpurun_out/threads_r5h.txt
timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/shapes_r5h.txt 2>&1 || exit $?
cat gpurun_out/shapes_r5h.txt
