# Same-box A/B of the exchange receive buffer's allocation (csrc/comm/ipc_allreduce.hip:
# hipDeviceMallocUncached, the default, vs CSED_IPC_MEM=finegrained): the looped-back exchange
# tests under the fine-grained buffer, then tools/exchange_trace.py with each.
#   gpurun --timeout 900 -- bash tools/gpu_ipcmem.sh [tag]
T=${1:-ipcmem}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
CSED_IPC_MEM=finegrained timeout -k 10 300 python -u -m pytest tests/test_exchange_loopback_gpu.py tests/test_comm_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/${T}_tests_fine.log 2>&1 && \
timeout -k 10 200 python -u tools/exchange_trace.py --batch 8 32 --worlds 1 2 8 > gpurun_out/${T}_trace_uncached.log 2>&1 && \
CSED_IPC_MEM=finegrained timeout -k 10 200 python -u tools/exchange_trace.py --batch 8 32 --worlds 1 2 8 > gpurun_out/${T}_trace_fine.log 2>&1 && \
timeout -k 10 200 python -u tools/exchange_trace.py --batch 8 32 --worlds 1 2 8 > gpurun_out/${T}_trace_uncached2.log 2>&1
echo rc=$?
