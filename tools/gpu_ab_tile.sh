# Tile tests on the working tree's build, then a same-box A/B (ab/A_C.so vs ab/B_C.so) of the
# large-batch steps: global batch 1024 and 8192 fp16, 3 alternating rounds each.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/ab_tile.log && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 300 python -u -m pytest tests/test_tile_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/ab_tile_tests.log 2>&1 ; [ $? -le 1 ] && \
for gb in 1024 8192; do st=$([ $gb = 1024 ] && echo 400 || echo 60); for i in 1 2 3; do for v in A B; do echo "gb=$gb $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch $gb --dtype fp16 --steps $st --warmup 20 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab_tile.log || exit 1; done; done; done
echo rc=$?
