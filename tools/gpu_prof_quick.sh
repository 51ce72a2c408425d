# Quick stage profiles: the sample-tile kernel at B = 1024 / 8192 and the fp32 kernel at 64 / 8.
T=${1:-r3p}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 8192 > gpurun_out/${T}_tilestages.log 2>&1 && \
timeout -k 10 200 python -u tools/stage_profile_f32.py 64 8 > gpurun_out/${T}_f32stages.log 2>&1
echo rc=$?
