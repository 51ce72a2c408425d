# Final check of the committed tree: the whole GPU suite, smoke(), the driver's bench command and
# the default / fp32 / per-rank-8 benches.
T=${1:-r3fin3}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/${T}_bench_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8 --steps 500 --warmup 50 > gpurun_out/${T}_bench_b8.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 --global-batch 8 --steps 500 --warmup 50 --no-epoch > gpurun_out/${T}_bench_fp32_b8.log 2>&1
echo rc=$?
