# Kernel traces (rocprofv3 --kernel-trace --stats) of the large-batch steps (B = 1024 / 8192, fp16)
# and the fp32 step (B = 64 / 8), then PMC passes over the tile kernel (tools/pmc_tile.sh).
T=${1:-r3k}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && mkdir -p $R/gpurun_out && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt1024 -o run -- python3 $R/bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > $R/gpurun_out/${T}_kt1024.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt8192 -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 --no-epoch > $R/gpurun_out/${T}_kt8192.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_ktf32 -o run -- python3 $R/bench.py --dtype fp32 --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_ktf32.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_ktf32b8 -o run -- python3 $R/bench.py --dtype fp32 --global-batch 8 --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_ktf32b8.log 2>&1 && \
cd $R && bash tools/pmc_tile.sh ${T}pmc
echo rc=$?
