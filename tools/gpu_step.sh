set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6j
timeout -k 10 300 python3 -u -m pytest tests/test_batch_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6j/pytest.log 2>&1 || { tail -30 gpurun_out/r6j/pytest.log; exit 1; }
tail -1 gpurun_out/r6j/pytest.log
timeout -k 10 300 python3 tools/host_input_threads.py 6 1,2 > gpurun_out/r6j/host_threads.log 2>&1 || { tail -20 gpurun_out/r6j/host_threads.log; exit 1; }
grep "T=" gpurun_out/r6j/host_threads.log
RJ_SPLIT_HOST=0 timeout -k 10 300 python3 tools/host_input_threads.py 6 1 > gpurun_out/r6j/host_threads_nosplit.log 2>&1 || { tail -20 gpurun_out/r6j/host_threads_nosplit.log; exit 1; }
grep "T=" gpurun_out/r6j/host_threads_nosplit.log
