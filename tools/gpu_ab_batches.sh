# Same-box A/B of ab/A_C.so vs ab/B_C.so (tools/ab_build.sh) at per-rank batches 8/16/32/64
# (global batch 64 over 8/4/2/1 ranks): alternating bench runs, one log per batch.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
for b in ${AB_BATCHES:-8 16 32 64}; do
  rm -f gpurun_out/ab_b$b.log
  for i in 1 2; do for v in A B; do
    echo "$v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --global-batch $b --steps 2000 --warmup 200 --no-epoch 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab_b$b.log || exit 1
  done; done
done
echo rc=$?
