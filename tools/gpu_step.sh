set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/rocjpeg_amd
STEPS=5 bash tools/gpu_ab_env.sh off:RJ_LIB_PATH=$L/librocjpeg_amd_hlstamps.so,RJ_DEBUG_STAMPS=1,RJ_K2_LIVE=0 live:RJ_LIB_PATH=$L/librocjpeg_amd_hlstamps.so,RJ_DEBUG_STAMPS=1
for f in gpurun_out/ab/off_1.log gpurun_out/ab/live_1.log gpurun_out/ab/off_2.log gpurun_out/ab/live_2.log; do echo $f; grep "rj k_huff\]" $f | tail -3; done
