# Tile kernel iteration: its tests, its stage profile, the large-batch benches.
T=${1:-r3u}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_tile_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tile_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 8192 > gpurun_out/${T}_tilestages.log 2>&1 && \
timeout -k 10 200 python -u tools/stage_profile_f32.py 64 > gpurun_out/${T}_f32stages.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 > gpurun_out/${T}_bench_lb.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/${T}_bench_1024.log 2>&1
echo rc=$?
