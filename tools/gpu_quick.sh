# Fused-kernel check: fused + kernel GPU tests, stage stamps, N=1 bench.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/q_tests.log 2>&1 && \
timeout -k 10 200 python tools/stage_profile.py > gpurun_out/q_stage.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/q_bench.log 2>&1
echo rc=$?
