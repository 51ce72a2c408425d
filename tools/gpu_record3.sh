# Round-3 record: the whole GPU suite, smoke(), the driver's bench command, the default bench,
# fp32 / per-rank batch 8 / large-batch benches, a 2-rank gloo rehearsal of the multi-rank
# bench flow (two ranks sharing the GPU), and kernel traces of the default and batch-8 steps.
T=${1:-r3rec}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/${T}_bench_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8 --steps 500 --warmup 50 > gpurun_out/${T}_bench_b8.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --global-batch 8 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_fp32_b8.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 > gpurun_out/${T}_bench_1024.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 > gpurun_out/${T}_bench_lb.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 > gpurun_out/${T}_bench_gloo2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt64 -o run -- python3 $R/bench.py --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_kt64.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt8 -o run -- python3 $R/bench.py --global-batch 8 --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_kt8.log 2>&1
echo rc=$?
