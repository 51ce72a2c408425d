# 2 ranks sharing the GPU (gloo bootstrap): fused-exchange step, one kernel vs two kernels.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/dp_step_bench.py --gloo > gpurun_out/dp1k_one.log 2>&1 && \
CSED_ONE_KERNEL_STEP=0 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29562 tools/dp_step_bench.py --gloo > gpurun_out/dp1k_two.log 2>&1
echo rc=$?
