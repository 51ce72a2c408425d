# Round-4 exchange diagnosis + fault-injection tests on one GPU:
#   gpurun --timeout 900 -- bash tools/gpu_r4a.sh [tag]
T=${1:-r4a}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u tools/exchange_trace.py --batch 8 32 --worlds 1 2 8 > gpurun_out/${T}_trace.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_fault_injection_gpu.py tests/test_exchange_loopback_gpu.py tests/test_comm_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_kt1 -o run -- python3 $R/tools/exchange_trace.py --batch 8 --worlds 1 > $R/gpurun_out/${T}_kt1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_kt8 -o run -- python3 $R/tools/exchange_trace.py --batch 8 --worlds 8 > $R/gpurun_out/${T}_kt8.log 2>&1
echo rc=$?
