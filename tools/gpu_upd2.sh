R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/u_tests.log 2>&1 && \
timeout -k 10 200 python tools/update_profile.py 64 > gpurun_out/u_prof.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 --no-epoch > gpurun_out/u_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 3000 --warmup 300 --no-epoch > gpurun_out/u_bench_b.log 2>&1
echo rc=$?
