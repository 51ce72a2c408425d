# fp32 kernel change: fp32 + dropout-pin tests on the working tree's build, fp32 stage stamps
# A / B, then same-box fp32 A/B at global batch 64 and 8.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/ab2.log && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 600 python -u -m pytest tests/test_fused_f32_gpu.py tests/test_kernels_f32_gpu.py tests/test_dropout_pin_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/abf32_tests.log 2>&1 ; [ $? -le 1 ] && \
CSED_NATIVE_SO=$R/ab/A_C.so timeout -k 10 120 python tools/stage_profile_f32.py 64 > gpurun_out/stf_A.log 2>&1 && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 120 python tools/stage_profile_f32.py 64 > gpurun_out/stf_B.log 2>&1 && \
for gb in 64 8; do for i in 1 2 3; do for v in A B; do echo "f32 gb=$gb $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch $gb --dtype fp32 --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab2.log || exit 1; done; done; done
echo rc=$?
