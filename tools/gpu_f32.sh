# fp32 kernel check: fp32 + dropout-pin tests, stage stamps at B = 64 / 8, the two fp32 benches.
T=${1:-r3g}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_fused_f32_gpu.py tests/test_dropout_pin_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/stage_profile_f32.py 64 8 > gpurun_out/${T}_f32stages.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --no-epoch > gpurun_out/${T}_bench_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --global-batch 8 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_fp32_b8.log 2>&1
echo rc=$?
