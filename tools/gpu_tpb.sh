R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/tpb.log && \
for t in 8 4 2 1 2 4 1 8; do echo "tpb=$t $(CSED_FC_TPB=$t timeout -k 10 100 python bench.py --steps 3000 --warmup 300 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/tpb.log || exit 1; done
echo rc=$?
