R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_comm_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/u3_tests.log 2>&1 && \
timeout -k 10 200 python tools/update_profile.py 64 > gpurun_out/u3_prof.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 --no-epoch > gpurun_out/u3_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/u3_bench1k.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > gpurun_out/u3_bench8k.log 2>&1
echo rc=$?
