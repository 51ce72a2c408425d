# Tile-kernel stage stamps for ab/A_C.so and ab/B_C.so (B = 1024 and 8192), twice each.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
for i in 1 2; do for v in A B; do CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 8192 > gpurun_out/tstg_${v}$i.log 2>&1 || exit 1; done; done
echo rc=$?
