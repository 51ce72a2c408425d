# Graph size A/B (same box, alternating): every graph replay starts ~8 us after the previous
# one's last kernel (rocprofv3 trace, profiles/bench_r2.md), so fewer, larger graphs shorten a
# run of many steps.  bench.py default (500 timed steps + a warm epoch) at --steps-per-graph
# 32 vs 1024, then the driver's command.
#   gpurun --timeout 900 -- bash tools/gpu_ab_spg.sh [tag]
T=${1:-spg}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps-per-graph 32 >> gpurun_out/${T}_32.log 2>&1 && \
  timeout -k 10 200 python bench.py --steps-per-graph 1024 >> gpurun_out/${T}_1024.log 2>&1 && \
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/${T}_driver.log 2>&1 || exit 1
done
echo rc=$?
