# lenet_update in isolation + stamps at large batch, A (HEAD) vs B (tree)
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/up_*.log && \
for v in A B; do CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 120 python tools/update_profile.py 8192 > gpurun_out/up_${v}.log 2>&1 || exit 1; done
echo rc=$?
