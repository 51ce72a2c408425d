# round-5 one-off: (1) split-K hand-off A/B at B = 8192 fp16 (ab/A_C.so = release/acquire fences,
# ab/B_C.so = write-through sc1 form) by rocprofv3 kernel stats, alternating; (2) the loopback
# world-8 soak; (3) the import A/B (with / without the HIP-context thread)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; T=${1:-r5j}
cd /tmp && export TMPDIR=/tmp && \
for i in 1 2; do for v in A B; do
  CSED_NATIVE_SO=$R/ab/${v}_C.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_splitk_${v}$i -o run -- python3 $R/bench.py --global-batch 8192 --dtype fp16 --steps 60 --warmup 6 --no-epoch --no-fp32-record > $O/${T}_splitk_${v}$i.log 2>&1 || exit 1
done; done && \
cd $R && timeout -k 10 400 python -u tools/loopback_soak.py --rounds 20 > $O/${T}_soak.log 2>&1; rc=$?; [ $rc -le 1 ] && \
timeout -k 10 400 python -u tools/import_probe.py --n 5 > $O/${T}_import.log 2>&1
