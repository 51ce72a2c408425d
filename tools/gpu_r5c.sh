# round-5 one-off: kernel / modular / exchange tests, the modular engine's step times and kernel
# trace, and the default bench line (bring-up breakdown)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; T=${1:-r5k}
cd $R && timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_f32_gpu.py tests/test_modular_graph_gpu.py tests/test_engine_gpu.py tests/test_fused_gpu.py -v --timeout 240 --timeout-method thread > $O/${T}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/ddp_overlap.py --graph graph > $O/${T}_ddp.log 2>&1 && \
timeout -k 10 200 python bench.py > $O/${T}_bench_default.json 2> $O/${T}_bench_default.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_mod64 -o run -- python3 $R/tools/modular_step.py 64 200 > $O/${T}_mod64.log 2>&1
