R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1 && \
timeout -k 10 200 python tools/step_timeline.py 64 > gpurun_out/tl.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/s_bench.log 2>&1
echo rc=$?
