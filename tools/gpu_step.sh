set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6r
timeout -k 10 300 python3 tools/host_parts_probe.py 3 > gpurun_out/r6r/parts.log 2>&1 || { tail -20 gpurun_out/r6r/parts.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r6r/prof3b -o prof -- python3 tools/host_parts_probe.py 3 > gpurun_out/r6r/prof3b.log 2>&1 || { tail -20 gpurun_out/r6r/prof3b.log; exit 1; }
grep parts gpurun_out/r6r/prof3b.log
