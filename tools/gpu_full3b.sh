# Round-3 rehearsal: the whole GPU suite, smoke(), the driver's bench command, the default bench,
# then the timed-window probe (graph vs native-then-graph plans for the 20-step window).
T=${1:-r3full}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 ; \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 && \
timeout -k 10 300 python -u tools/timed_window_probe.py 64 > gpurun_out/${T}_window.log 2>&1
echo rc=$?
