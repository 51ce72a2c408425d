# bf16 train kernel with LDS-only barriers: GPU tests of the fused paths, stage stamps, benches.
T=${1:-r3p}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_engine_gpu.py tests/test_exchange_loopback_gpu.py tests/test_dropout_pin_gpu.py tests/test_comm_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/stage_profile.py 64 8 > gpurun_out/${T}_stages.log 2>&1 ; \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.log 2>&1 && \
timeout -k 10 200 python bench.py --no-epoch > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_b8.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 32 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_b32.log 2>&1
echo rc=$?
