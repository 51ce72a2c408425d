# 2 ranks sharing the GPU: standalone IPC all-reduce + fused in-kernel exchange, then the fused suite.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/comm.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fused.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench1.log 2>&1
echo rc=$?
