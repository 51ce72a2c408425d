# Loss-stage rewrite: tests on the working tree's build, then same-box A/B (bf16 B=64/8 +
# driver command, fp32 B=64/8, tile kernel B=1024).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_engine_gpu.py tests/test_tile_gpu.py tests/test_fused_f32_gpu.py tests/test_kernels_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/abloss_tests.log 2>&1 ; [ $? -le 1 ] && \
bash tools/gpu_ab_b64_b8.sh && \
for gb in 64 8; do for i in 1 2; do for v in A B; do echo "f32 gb=$gb $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch $gb --dtype fp32 --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab2.log || exit 1; done; done; done && \
for i in 1 2; do for v in A B; do echo "gb=1024 $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch 1024 --dtype fp16 --steps 400 --warmup 20 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab2.log || exit 1; done; done
echo rc=$?
