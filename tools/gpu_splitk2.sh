# Split-K FC update: GPU tests, lenet_update in isolation at B=8192 (A vs B), bench A/B.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/sk_*.log gpurun_out/up_*.log && \
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sk_tests.log 2>&1 && \
for v in A B; do CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 120 python tools/update_profile.py 8192 > gpurun_out/up_${v}.log 2>&1 || exit 1; done && \
for i in 1 2; do for v in A B; do echo "$v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch 8192 --dtype fp16 --steps 300 --warmup 30 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/sk_ab_large.log || exit 1; done; done && \
for i in 1 2 3; do for v in A B; do echo "$v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/sk_ab_64.log || exit 1; done; done
echo rc=$?
