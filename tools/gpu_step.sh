# One-kernel step check: fused/engine/kernel/comm GPU tests, N=1 bench, kernel trace.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/s_bench.log 2>&1 && \
CSED_ONE_KERNEL_STEP=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/s_bench2k.log 2>&1 && \
[ -n "$PROF" ] && cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s_prof -o run -- python3 $R/bench.py --steps 300 --warmup 30 > $R/gpurun_out/s_prof.log 2>&1
echo rc=$?
