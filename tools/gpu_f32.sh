# fp32 fused path: its GPU tests and an fp32 bench line.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_fused_f32_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 ; \
timeout -k 10 200 python bench.py --dtype fp32 --steps 200 --warmup 20 > gpurun_out/f32_bench.log 2>&1
echo rc=$?
