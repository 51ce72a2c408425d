# Weight DMA off the preamble (fp32 kernel: LDS-DMA of fc1.w / conv2.w at stage 0; tile kernel:
# untracked DMA waited for before conv2) + fp32 tile-8 sharing: tests, stage stamps, benches.
T=${1:-r3f}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_f32_gpu.py tests/test_dropout_pin_gpu.py tests/test_tile_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/stage_profile_f32.py 64 8 > gpurun_out/${T}_f32stages.log 2>&1 && \
timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 8192 > gpurun_out/${T}_tilestages.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --no-epoch > gpurun_out/${T}_bench_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --global-batch 8 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_fp32_b8.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > gpurun_out/${T}_bench_lb.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/${T}_bench_1024.log 2>&1
echo rc=$?
cd $R && timeout -k 10 200 python -u tools/update_stamps.py 8192 1024 > gpurun_out/${T}_upd.log 2>&1
echo rc=$?
