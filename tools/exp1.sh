set -o pipefail
mkdir -p gpurun_out/e1
BATCHES=1024 bash tools/hl_stamps.sh || exit $?
RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_stamps.so RJ_DEBUG_STAMPS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/e1/k2st.log 2>&1 || exit $?
grep "rj stamps" gpurun_out/e1/k2st.log | tail -1
bash tools/ab_lib.sh base:- nodep:-:RJ_DEBUG_NODEP=1
