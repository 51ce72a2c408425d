# Round-end rehearsal: the whole GPU suite, smoke(), bench (N=1), kernel-trace profile.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/full_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/full_prof -o run -- python3 $R/bench.py --steps 300 --warmup 30 > $R/gpurun_out/full_prof.log 2>&1
echo rc=$?
