# Comm test (diagnostics on mismatch), then kernel traces of the large-batch steps
# (B = 1024 / 8192, fp16) and of the bf16 per-rank batch-8 / 64 steps.
T=${1:-r3b}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/${T}_comm.log 2>&1 ; \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt1024 -o run -- python3 $R/bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > $R/gpurun_out/${T}_kt1024.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt8192 -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > $R/gpurun_out/${T}_kt8192.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt8 -o run -- python3 $R/bench.py --global-batch 8 --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_kt8.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt64 -o run -- python3 $R/bench.py --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_kt64.log 2>&1
echo rc=$?
