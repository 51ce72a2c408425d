# round-5 one-off: same-box A/B of two exchange builds (ab/A_C.so vs ab/B_C.so, and B with the
# loopback check switched off) at the looped-back world-8 / world-4 steps; then the kernel,
# exchange and modular tests and the modular engine's step times / kernel trace on the B build
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; T=${1:-r5g}
cd $R && rm -f $O/${T}_ab3.log && \
for i in 1 2 3; do for c in "--global-batch 8 --loopback-world 8" "--global-batch 16 --loopback-world 4"; do
  for v in A B C; do
    so=$v; env=""; if [ $v = C ]; then so=B; env="CSED_LOOPBACK_CHECK=0"; fi
    echo "$v [$c] $(env $env CSED_NATIVE_SO=$R/ab/${so}_C.so timeout -k 10 100 python bench.py $c --steps 3000 --warmup 300 --no-epoch --no-fp32-record 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')" >> $O/${T}_ab3.log || exit 1
  done; done; done && \
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_f32_gpu.py tests/test_modular_graph_gpu.py tests/test_exchange_loopback_gpu.py tests/test_engine_gpu.py tests/test_fused_gpu.py -v --timeout 240 --timeout-method thread > $O/${T}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/ddp_overlap.py --graph graph > $O/${T}_ddp.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_mod64 -o run -- python3 $R/tools/modular_step.py 64 200 > $O/${T}_mod64.log 2>&1
