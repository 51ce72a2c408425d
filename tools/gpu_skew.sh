# Stage profiles with workgroup start / end skew (realtime stamps): tile and fp32 kernels.
T=${1:-r3c}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 200 python -u tools/stage_profile_tile.py 1024 8192 > gpurun_out/${T}_tilestages.log 2>&1 && \
timeout -k 10 200 python -u tools/stage_profile_f32.py 64 8 > gpurun_out/${T}_f32stages.log 2>&1
echo rc=$?
