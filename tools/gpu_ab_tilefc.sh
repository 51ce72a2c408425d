# Tile-kernel change: tile tests on the working tree's build, tile stage stamps A / B, then
# same-box A/B at global batch 1024 and 8192 (fp16).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/ab2.log && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 600 python -u -m pytest tests/test_tile_gpu.py tests/test_fused_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/abtile_tests.log 2>&1 ; [ $? -le 1 ] && \
CSED_NATIVE_SO=$R/ab/A_C.so timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 > gpurun_out/tstg_A.log 2>&1 && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 > gpurun_out/tstg_B.log 2>&1 && \
for gb in 1024 8192; do for i in 1 2 3; do for v in A B; do echo "gb=$gb $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch $gb --dtype fp16 --steps 200 --warmup 20 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab2.log || exit 1; done; done; done
echo rc=$?
