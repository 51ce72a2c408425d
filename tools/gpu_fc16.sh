# FC16 check: fused / tile / dropout / loopback GPU tests, then the large-batch, 1024, default and B=8 benches.
T=${1:-f16a}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_tile_gpu.py tests/test_dropout_pin_gpu.py tests/test_exchange_loopback_gpu.py tests/test_fused_f32_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > gpurun_out/${T}_bench_lb.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/${T}_bench_1024.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-epoch > gpurun_out/${T}_bench_64.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8 --steps 1000 --warmup 100 --no-epoch > gpurun_out/${T}_bench_8.log 2>&1 && \
NFC=88 timeout -k 10 200 python -u tools/update_stamps.py 8192 > gpurun_out/${T}_upd.log 2>&1 && \
NFC=88 timeout -k 10 200 python -u tools/update_stamps.py 1024 >> gpurun_out/${T}_upd.log 2>&1
echo rc=$?
