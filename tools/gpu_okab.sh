# one-kernel vs two-kernel step, same build, alternating (B = $OKB, default 64)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/okab.log && \
for b in ${OKB:-64 8}; do for i in 1 2 3; do for m in 1 0; do echo "B=$b one=$m $(CSED_ONE_KERNEL_STEP=$m timeout -k 10 100 python bench.py --global-batch $b --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/okab.log || exit 1; done; done; done
echo rc=$?
