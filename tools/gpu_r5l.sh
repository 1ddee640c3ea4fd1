set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/threads_r5l.txt
for cfg in "RJ_COALESCE_INFLIGHT=1" "RJ_COALESCE_INFLIGHT=2" "RJ_COALESCE_INFLIGHT=3" "RJ_COALESCE_INFLIGHT=4" "RJ_COALESCE_INFLIGHT=2"; do
  env $cfg timeout -k 10 120 python3 tools/threads_probe.py >> gpurun_out/threads_r5l.txt 2>&1 || { cat gpurun_out/threads_r5l.txt; exit 1; }
done
grep threads gpurun_out/threads_r5l.txt
for b in 960 1024 960 1024; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --runs 1 --no-cpu-baseline --no-extras --batch $b > gpurun_out/k1_b$b.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/k1_b$b.json') if l.startswith('{')][-1]); k=d['roofline']['per_kernel_launch_ms_sum']
print('batch $b', round(d['value']), d['ms_per_step'], 'K1', k.get('k_huff'), 'K2', k.get('k_rows'))"
done
