# conv1 stage change: tests on the working tree's build, stage stamps A / B, then same-box
# A/B at global batch 64 and 8 and the driver command.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_engine_gpu.py tests/test_tile_gpu.py tests/test_exchange_loopback_gpu.py tests/test_dropout_pin_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/abc1_tests.log 2>&1 ; [ $? -le 1 ] && \
CSED_NATIVE_SO=$R/ab/A_C.so timeout -k 10 120 python tools/stage_profile.py 64 > gpurun_out/stab_A.log 2>&1 && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 120 python tools/stage_profile.py 64 > gpurun_out/stab_B.log 2>&1 && \
bash tools/gpu_ab_b64_b8.sh
echo rc=$?
