# Stage stamps of lenet_train (split step, B = 64) for ab/A_C.so and ab/B_C.so on one box.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
CSED_NATIVE_SO=$R/ab/A_C.so timeout -k 10 120 python tools/stage_profile.py 64 > gpurun_out/stab_A.log 2>&1 && \
CSED_NATIVE_SO=$R/ab/B_C.so timeout -k 10 120 python tools/stage_profile.py 64 > gpurun_out/stab_B.log 2>&1
echo rc=$?
