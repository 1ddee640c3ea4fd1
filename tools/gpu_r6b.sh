set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in 1 8; do
  RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_hcstamps3.so RJ_DEBUG_STAMPS=1 SHAPES=$b timeout -k 10 180 python3 tools/shape_profile.py 384 > gpurun_out/hcst3_$b.txt 2>&1 || { tail gpurun_out/hcst3_$b.txt; exit 1; }
  grep "k_huff_chunk" gpurun_out/hcst3_$b.txt | tail -2
done
