# Same-box A/B of ab/A_C.so vs ab/B_C.so (tools/ab_build.sh): alternating bench runs.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/ab.log && \
for i in 1 2 3; do for v in A B; do echo "$v $(CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 100 python bench.py --steps 3000 --warmup 300 --no-epoch $AB_ARGS 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> gpurun_out/ab.log || exit 1; done; done
echo rc=$?
