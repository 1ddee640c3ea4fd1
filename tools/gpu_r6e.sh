# lean K1 stamps (RJ_HL_STAMPS builds): previous step arithmetic vs the bitfield/LDS-address step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hl
for v in basest newst basest newst; do
  RJ_LIB_PATH=$PWD/rocjpeg_amd/librocjpeg_amd_$v.so RJ_DEBUG_STAMPS=1 timeout -k 10 200 python bench.py --steps 2 --warmup 0 --runs 1 --no-cpu-baseline --no-extras > gpurun_out/hl/$v.log 2>&1 || exit $?
  echo "== $v"; grep "rj k_huff\]" gpurun_out/hl/$v.log | tail -1
done
