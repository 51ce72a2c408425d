# Native step executor vs graph replay for the driver's short timed window (same box,
# alternating runs): the GPU tests, the window probe (also with device-resident kernel
# arguments for eager launches, HIP_FORCE_DEV_KERNARG=1), then bench.py with graphs (default)
# vs the executor (CSED_NATIVE_STEPS=64) with device kernargs.
#   gpurun --timeout 900 -- bash tools/gpu_ab_native.sh [tag] [bench flags]
T=${1:-nat}
shift
ARGS=${*:-"--gpus 1 --steps 20 --warmup 5"}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
timeout -k 10 120 python tools/timed_window_probe.py 64 > gpurun_out/${T}_window64.log 2>&1 && \
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python tools/timed_window_probe.py 64 > gpurun_out/${T}_window64_devka.log 2>&1 && \
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $ARGS >> gpurun_out/${T}_graph.log 2>&1 && \
  HIP_FORCE_DEV_KERNARG=1 CSED_NATIVE_STEPS=64 timeout -k 10 200 python bench.py $ARGS >> gpurun_out/${T}_native_devka.log 2>&1 && \
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 200 python bench.py $ARGS >> gpurun_out/${T}_graph_devka.log 2>&1 || exit 1
done
echo rc=$?
