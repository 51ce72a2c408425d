R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lbprof -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 20 --warmup 3 --no-epoch > $R/gpurun_out/lbprof.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lbprof1k -o run -- python3 $R/bench.py --global-batch 1024 --dtype fp16 --steps 50 --warmup 5 --no-epoch > $R/gpurun_out/lbprof1k.log 2>&1
echo rc=$?
