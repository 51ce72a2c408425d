R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_comm_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/two_tests.log 2>&1 && \
timeout -k 10 200 python tools/step_timeline.py 64 > gpurun_out/tl.log 2>&1 && \
CSED_ONE_KERNEL_STEP=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch > gpurun_out/s_bench2k.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-epoch > gpurun_out/s_bench.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 tools/dp_step_bench.py --gloo > gpurun_out/dp_two.log 2>&1
echo rc=$?
