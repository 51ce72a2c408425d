# Diagnose 2-rank shared-GPU step time: fused-only mode, steps-per-graph, and two independent N=1 benches at once.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
CSED_ALLREDUCE=fused timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --no-epoch > gpurun_out/r2_fused.log 2>&1 && \
CSED_ALLREDUCE=fused timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --backend gloo --no-epoch --steps 512 --steps-per-graph 128 > gpurun_out/r2_fused128.log 2>&1 && \
(timeout -k 10 200 python bench.py --no-epoch --global-batch 32 > gpurun_out/r2_indep_a.log 2>&1 & timeout -k 10 200 python bench.py --no-epoch --global-batch 32 > gpurun_out/r2_indep_b.log 2>&1; wait) && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 tools/dp_step_bench.py --gloo > gpurun_out/r2_dpstep.log 2>&1
echo rc=$?
