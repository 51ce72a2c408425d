R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && P=29540 && \
for v in "--warmup 64 --steps 512" "--warmup 64 --steps 512 --no-graph" "--warmup 0 --steps 512"; do P=$((P+1)); echo "== $v" >> gpurun_out/r2c.log; CSED_ALLREDUCE=fused timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --backend gloo --no-epoch $v 2>&1 | grep -o '"ms_per_step": [0-9.]*' >> gpurun_out/r2c.log || exit 1; done
echo rc=$?
