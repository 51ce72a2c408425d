R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 200 python tools/stage_profile.py 64 > gpurun_out/st64.log 2>&1 && \
timeout -k 10 200 python tools/stage_profile.py 8 > gpurun_out/st8.log 2>&1
echo rc=$?
