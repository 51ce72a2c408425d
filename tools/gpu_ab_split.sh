# Split-step + tile tests on the working tree's build, split stage stamps (A vs B), then the
# same-box A/B benches at global batch 64 and 8 (tools/gpu_ab_b64_b8.sh).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_tile_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/absplit_tests.log 2>&1 ; [ $? -le 1 ] && \
for v in A B; do CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 200 python -u tools/split_diag.py 64 > gpurun_out/absplit_diag_$v.log 2>&1 || exit 1; done && \
bash tools/gpu_ab_b64_b8.sh
