set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_chunking_gpu.py tests/test_decode_gpu.py tests/test_fuzz_gpu.py tests/test_threads_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r6a.log 2>&1 || { tail -30 gpurun_out/pytest_r6a.log; exit 1; }
tail -1 gpurun_out/pytest_r6a.log
for b in 1 8; do
  RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_hcstamps2.so RJ_DEBUG_STAMPS=1 SHAPES=$b timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/hcst2_$b.txt 2>&1 || { tail gpurun_out/hcst2_$b.txt; exit 1; }
  grep "k_huff_chunk" gpurun_out/hcst2_$b.txt | tail -1
done
for lib in prevk1 cur prevk1 cur; do
  if [ $lib = cur ]; then unset RJ_LIB_PATH; else export RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_$lib.so; fi
  echo "== $lib"; SHAPES=1,8,16,32 timeout -k 10 180 python3 tools/shape_profile.py 384 2>&1 | grep batch
done
unset RJ_LIB_PATH
BENCH_EXTRA="--workload c2nori" TAG=r6a bash tools/gpu_ab.sh prev:prevk1 cur:- prev2:prevk1 cur2:- || exit $?
