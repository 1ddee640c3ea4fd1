set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PMC_FILE=tools/pmc_sets_place.txt BENCH_ARGS="--runs 3 --steps 4" bash tools/pmc_run.sh place_on && RJ_PLACE_TUNE=0 PMC_FILE=tools/pmc_sets_place.txt BENCH_ARGS="--runs 3 --steps 4" bash tools/pmc_run.sh place_off && ls gpurun_out/pmc_place_on gpurun_out/pmc_place_off
