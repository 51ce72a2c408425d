# fp32 split step with tile 8 shared over the parts: fp32 tests, stage stamps, benches; then a
# graph vs native-executor A/B of the driver's 20-step window (3 alternations).
T=${1:-r3c}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_fused_f32_gpu.py tests/test_dropout_pin_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 200 python -u tools/stage_profile_f32.py 64 8 > gpurun_out/${T}_f32stages.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --no-epoch > gpurun_out/${T}_bench_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --global-batch 8 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_fp32_b8.log 2>&1 && \
for i in 1 2 3; do
  timeout -k 10 100 python bench.py --gpus 1 --steps 20 --warmup 5 --no-epoch > gpurun_out/${T}_win_graph$i.log 2>&1 && \
  CSED_NATIVE_STEPS=64 timeout -k 10 100 python bench.py --gpus 1 --steps 20 --warmup 5 --no-epoch > gpurun_out/${T}_win_native$i.log 2>&1 || exit 1
done
echo rc=$?
