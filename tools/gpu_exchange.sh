# Exchange checks on one GPU: the loopback and shared-GPU 2-rank tests, the loopback cost
# table at virtual N = 1/2/4/8 (profiles/dp_exchange_r3.md), the capture-order rehearsal of
# two ranks on one GPU (dp_step_bench --no-time-steps), the driver's bench command.
#   gpurun --timeout 900 -- bash tools/gpu_exchange.sh [tag]
T=${1:-r3x}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_exchange_loopback_gpu.py tests/test_comm_gpu.py tests/test_dropout_pin_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/exchange_loopback.py 8 16 32 64 > gpurun_out/${T}_loopback.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 tools/dp_step_bench.py --gloo --no-time-steps > gpurun_out/${T}_dp_order.log 2>&1 && \
timeout -k 10 200 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/dp_step_bench.py --gloo > gpurun_out/${T}_dp.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8 --loopback-world 8 --steps 500 --warmup 50 > gpurun_out/${T}_bench_lb8.log 2>&1
echo rc=$?
