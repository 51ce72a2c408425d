# Round-4 exchange / large-batch work on one GPU: exchange / fault / comm / fused / tile tests,
# then the per-step breakdowns (tools/exchange_trace.py: loopback exchange at B x N, and the
# tile-kernel step at B = 1024 / 8192 with the split-K fc update and without it) and the
# loopback table (tools/exchange_loopback.py).
#   gpurun --timeout 1100 -- bash tools/gpu_r4a.sh [tag]
T=${1:-r4a}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_exchange_loopback_gpu.py tests/test_fault_injection_gpu.py tests/test_comm_gpu.py tests/test_fused_gpu.py tests/test_tile_gpu.py -v --timeout 240 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; [ $? -le 1 ] && \
timeout -k 10 300 python -u tools/exchange_trace.py --batch 8 16 32 64 --worlds 1 2 4 8 > gpurun_out/${T}_trace.log 2>&1 && \
timeout -k 10 200 python -u tools/exchange_trace.py --batch 1024 2048 8192 --worlds 1 --steps 12 > gpurun_out/${T}_tiletrace.log 2>&1 && \
CSED_FC_SLICES=1 timeout -k 10 200 python -u tools/exchange_trace.py --batch 2048 8192 --worlds 1 --steps 12 > gpurun_out/${T}_tiletrace_s1.log 2>&1 && \
CSED_FC_SLICES=2 timeout -k 10 200 python -u tools/exchange_trace.py --batch 1024 --worlds 1 --steps 12 > gpurun_out/${T}_tiletrace_s2.log 2>&1 && \
timeout -k 10 300 python -u tools/exchange_loopback.py 8 16 32 64 > gpurun_out/${T}_loopback.log 2>&1
echo rc=$?
