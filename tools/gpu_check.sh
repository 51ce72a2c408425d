R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 300 python -m pytest tests/test_fused_gpu.py -x -q > gpurun_out/t.log 2>&1 && \
timeout -k 10 200 python tools/stage_profile.py > gpurun_out/stage.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/pmc8 -o run -- python3 $R/tools/kernel_counters.py 64 200 > $R/gpurun_out/pmc8.log 2>&1
