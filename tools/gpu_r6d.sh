# K1 step arithmetic (bitfield extracts, LDS byte addresses): parity on the Huffman-heavy GPU
# tests, then same-box A/B against the previous build (C2 and c2nori, interleaved)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_batch_gpu.py tests/test_chunking_gpu.py tests/test_decode_gpu.py tests/test_fuzz_gpu.py \
  > gpurun_out/pytest_r6d.log 2>&1 || { tail -30 gpurun_out/pytest_r6d.log; exit 1; }
tail -3 gpurun_out/pytest_r6d.log
bash tools/ab_lib.sh base:base new:- base2:base new2:- && \
BENCH_EXTRA="--workload c2nori" bash tools/ab_lib.sh nbase:base nnew:- nbase2:base nnew2:-
