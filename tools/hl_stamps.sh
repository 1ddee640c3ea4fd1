set -o pipefail
mkdir -p gpurun_out/hl
for b in ${BATCHES:-256 1024}; do
RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_hlst.so RJ_DEBUG_STAMPS=1 RJ_PIPE_GROUPS=1 timeout -k 10 200 python bench.py --steps 2 --warmup 0 --batch $b --no-cpu-baseline --no-extras > gpurun_out/hl/b$b.log 2>&1 || exit $?
grep "rj k_huff" gpurun_out/hl/b$b.log | tail -2
done
