# GPU check of the tree: GPU tests, smoke(), the driver's bench command, the default bench,
# the fp32 and large-batch fp16 configs, and kernel-trace profiles of the default bench and
# of the per-rank batch-8 step (global 64 over 8 ranks: the strong-scaling floor).
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh [tag]
T=${1:-r2}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 200 python bench.py --dtype fp32 > gpurun_out/${T}_bench_fp32.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 > gpurun_out/${T}_bench_lb.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 300 --warmup 30 > $R/gpurun_out/${T}_prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof8 -o run -- python3 $R/bench.py --global-batch 8 --steps 300 --warmup 30 --no-epoch > $R/gpurun_out/${T}_prof8.log 2>&1
echo rc=$?
