# Same-box A/B of one build under two environments: ENV_A vs ENV_B (e.g. "CSED_MASK_STAGE=0"),
# alternating bench runs; BENCH_ARGS replaces the default flags (--steps 3000 --warmup 300 --no-epoch),
# AB_ARGS are extra bench.py flags; N_AB alternations (default 3).  Output: gpurun_out/ab_env.log
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/ab_env.log && \
for i in $(seq ${N_AB:-3}); do for v in A B; do
  if [ $v = A ]; then E="$ENV_A"; else E="$ENV_B"; fi
  echo "$v $(env $E timeout -k 10 100 python bench.py ${BENCH_ARGS:---steps 3000 --warmup 300 --no-epoch} $AB_ARGS 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab_env.log || exit 1
done; done
