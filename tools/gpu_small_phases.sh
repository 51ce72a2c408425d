# Small-batch phase stamps: lenet_update (B = 8, 64) and lenet_train stages (B = 64, 8).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 120 python tools/update_stamps.py 8 64 > gpurun_out/sp_update.log 2>&1 && \
timeout -k 10 120 python tools/stage_profile.py 64 > gpurun_out/sp_stage64.log 2>&1 && \
timeout -k 10 120 python tools/stage_profile.py 8 > gpurun_out/sp_stage8.log 2>&1
echo rc=$?
