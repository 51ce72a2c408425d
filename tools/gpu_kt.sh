R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && mkdir -p $R/gpurun_out && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt1 -o one -- python3 $R/tools/step_loop.py 64 300 > $R/gpurun_out/kt1.log 2>&1 && \
CSED_ONE_KERNEL_STEP=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt2 -o two -- python3 $R/tools/step_loop.py 64 300 > $R/gpurun_out/kt2.log 2>&1
echo rc=$?
