# Per-step time of the fused engine at the per-rank batches of N = 1/2/4/8 (64/N) on one GPU,
# the 2-rank IPC all-reduce latency (ranks sharing the GPU), and a kernel trace at B=8.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
for gb in 8 16 32 64; do timeout -k 10 120 python bench.py --global-batch $gb --steps 2000 --warmup 200 --no-epoch >> gpurun_out/sb_bench.log 2>&1 || exit 1; done && \
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/allreduce_bench.py --gloo > gpurun_out/sb_ar.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sb_prof -o run -- python3 $R/bench.py --global-batch 8 --steps 300 --warmup 30 --no-epoch > $R/gpurun_out/sb_prof.log 2>&1
echo rc=$?
