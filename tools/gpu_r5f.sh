set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r5p5 bash tools/gpu_ab.sh base:- synthwin:synthwin swnowait:swnowait swl2:swl2 swl2nw:swl2nw l2store:l2store base2:- swnowait2:swnowait || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_scan5f -o scan -- python3 tools/scan_timing.py > gpurun_out/scan_r5f.txt 2>&1 || exit $?
cat gpurun_out/scan_r5f.txt
find gpurun_out/prof_scan5f -name '*kernel_stats.csv' -exec cat {} \;
