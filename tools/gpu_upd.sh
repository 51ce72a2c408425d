# Update-kernel iteration: fused / tile tests, update phase stamps, benches at B = 64 / 1024 / 8192.
T=${1:-r3m}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_tile_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/update_stamps.py 64 8 1024 8192 > gpurun_out/${T}_upd.log 2>&1 && \
timeout -k 10 200 python bench.py --no-epoch > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/${T}_bench_1024.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > gpurun_out/${T}_bench_lb.log 2>&1
echo rc=$?
