# Stage stamps of lenet_train (B = 64 and 8) and per-rank-batch step times (the strong-scaling
# per-GPU floor: global batch 64 split over N = 1/2/4/8 ranks).
#   gpurun -- bash tools/gpu_stages.sh [tag]
T=${1:-st}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 120 python tools/stage_profile.py 64 > gpurun_out/${T}_stage64.log 2>&1 && \
timeout -k 10 120 python tools/stage_profile.py 8 > gpurun_out/${T}_stage8.log 2>&1 && \
for b in 8 16 32 64; do timeout -k 10 120 python bench.py --global-batch $b --steps 1000 --warmup 100 --no-epoch > gpurun_out/${T}_b$b.log 2>&1 || exit 1; done
echo rc=$?
