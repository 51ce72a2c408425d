# The shared-GPU comm test, four times in one call (diagnostics of the intermittent one-shot vs
# fused parameter mismatch: max / count of differences, error words).
T=${1:-r3h}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
for i in 1 2 3; do
  timeout -k 10 200 python -u -m pytest tests/test_comm_gpu.py -k two_ranks_one_gpu -v --timeout 150 --timeout-method thread > gpurun_out/${T}_comm$i.log 2>&1
  rc=$?; echo "run $i rc=$rc"; [ $rc -le 1 ] || exit $rc
done
echo done
