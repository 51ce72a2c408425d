R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/bsweep.log && \
for b in 8 16 32 64; do for m in 1 0; do echo "B=$b one_kernel=$m $(CSED_ONE_KERNEL_STEP=$m timeout -k 10 100 python bench.py --global-batch $b --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/bsweep.log || exit 1; done; done
echo rc=$?
