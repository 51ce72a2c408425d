# Stage stamps at small and large per-WG sample counts + large-batch bench.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lb_tests.log 2>&1 && \
timeout -k 10 200 python tools/stage_profile.py 64 > gpurun_out/lb_stage64.log 2>&1 && \
timeout -k 10 200 python tools/stage_profile.py 1024 256 > gpurun_out/lb_stage1024.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > gpurun_out/lb_bench8192.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/lb_bench1024.log 2>&1
echo rc=$?
