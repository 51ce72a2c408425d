# B = 1024 (fp16) step check: bench with native / torch data, then a kernel trace.
T=${1:-r3b}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/${T}_b1.log 2>&1 && \
CSED_TORCH_DATA=1 timeout -k 10 200 python bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > gpurun_out/${T}_b2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt -o run -- python3 $R/bench.py --global-batch 1024 --dtype fp16 --steps 200 --warmup 20 --no-epoch > $R/gpurun_out/${T}_kt.log 2>&1
echo rc=$?
