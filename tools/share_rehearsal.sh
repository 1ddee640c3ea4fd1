cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for N in 2 4; do
  RJ_BENCH_SHARE_GPU=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 1 --batch 128 > gpurun_out/share_n${N}.log 2>&1 || { echo "N=$N failed"; tail -20 gpurun_out/share_n${N}.log; exit 1; }
  grep '^{' gpurun_out/share_n${N}.log | tail -1 | cut -c1-600
done
