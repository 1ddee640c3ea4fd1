set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/shapes_r5p.txt
for m in 384 256 192 128; do
  echo "== RJ_CHUNK_MIN=$m" >> gpurun_out/shapes_r5p.txt
  SHAPES=1,8,16,32 timeout -k 10 180 python3 tools/shape_profile.py $m >> gpurun_out/shapes_r5p.txt 2>&1 || { tail gpurun_out/shapes_r5p.txt; exit 1; }
done
grep -E "==|batch" gpurun_out/shapes_r5p.txt
SHAPES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b1 -o b1 -- python3 tools/shape_profile.py 384 > gpurun_out/shapes_b1.txt 2>&1 || exit $?
find gpurun_out/prof_b1 -name '*kernel_stats.csv' -exec cat {} \;
for b in 960 1024 960 1024; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --runs 1 --no-cpu-baseline --no-extras --batch $b > gpurun_out/k1_b$b.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/k1_b$b.json') if l.startswith('{')][-1]); k=d['roofline']['per_kernel_launch_ms_sum']
print('batch $b', round(d['value']), d['ms_per_step'], 'K1', k.get('k_huff'), 'K2', k.get('k_rows'))"
done
