# bench.py's multi-rank path end-to-end on one GPU: 2 ranks, gloo bootstrap, fused in-kernel exchange.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo > gpurun_out/rehearse2.log 2>&1
echo rc=$?
