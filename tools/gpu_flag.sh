# Flagship (bf16, B = 64 and per-rank 8) stage stamps + kernel traces.
T=${1:-r3i}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
timeout -k 10 200 python -u tools/stage_profile.py 64 > gpurun_out/${T}_stages64.log 2>&1 && \
timeout -k 10 200 python -u tools/stage_profile.py 8 > gpurun_out/${T}_stages8.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt64 -o run -- python3 $R/bench.py --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_kt64.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt8 -o run -- python3 $R/bench.py --global-batch 8 --steps 500 --warmup 50 --no-epoch > $R/gpurun_out/${T}_kt8.log 2>&1
echo rc=$?
