# Record run: GPU test suite, bench (headline + large batch), kernel trace of the headline bench, stage stamps.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/rec && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rec/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/rec/bench64.log 2>&1 && \
timeout -k 10 200 python bench.py --global-batch 8192 --dtype fp16 --steps 40 --warmup 5 > gpurun_out/rec/bench8192.log 2>&1 && \
timeout -k 10 200 python tools/stage_profile.py 64 > gpurun_out/rec/stage64.log 2>&1 && \
timeout -k 10 200 python tools/update_profile.py 64 > gpurun_out/rec/update64.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rec/trace64 -o run -- python3 $R/bench.py --steps 300 --warmup 30 --no-epoch > $R/gpurun_out/rec/trace64.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rec/trace8k -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 20 --warmup 3 --no-epoch > $R/gpurun_out/rec/trace8k.log 2>&1
echo rc=$?
