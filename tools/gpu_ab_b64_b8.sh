# Same-box A/B of ab/A_C.so vs ab/B_C.so (tools/ab_build.sh) at global batch 64 and 8 (the
# strong-scaling floor), 3 alternating rounds each, plus the driver's 20-step command.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/ab2.log && \
for gb in 64 8; do for i in 1 2 3; do for v in A B; do echo "gb=$gb $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch $gb --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab2.log || exit 1; done; done; done && \
for i in 1 2; do for v in A B; do echo "driver $v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --gpus 1 --steps 20 --warmup 5 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab2.log || exit 1; done; done
echo rc=$?
