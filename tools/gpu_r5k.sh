set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b8 -o b8 -- python3 tools/shape_profile.py 384 > gpurun_out/shapes_b8.txt 2>&1 || { tail gpurun_out/shapes_b8.txt; exit 1; }
grep "batch" gpurun_out/shapes_b8.txt
find gpurun_out/prof_b8 -name '*kernel_stats.csv' -exec cat {} \;
timeout -k 10 600 python3 bench.py --steps 20 > gpurun_out/bench_r5k.json 2> gpurun_out/bench_r5k.err || { tail gpurun_out/bench_r5k.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_r5k.json
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_r5k.json') if l.startswith('{')][-1])
c=d['call_shapes']; print({k:(v.get('images_per_s_summed') or v.get('images_per_s')) for k,v in c.items() if isinstance(v,dict)})
print(d['parse_images_per_s']); print(d['extra_workloads']['c5'].get('decode_batch1'))"
