set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for ws in 0 2 3 4 0 2 3; do
  echo "== RJ_K1_HYP_WARM_SHIFT=$ws"; RJ_K1_HYP_WARM_SHIFT=$ws RJ_DEBUG_K1=1 SHAPES=1,8,16 timeout -k 10 180 python3 tools/shape_profile.py 384 2>&1 | grep -E "batch|\[K1\]"
done
