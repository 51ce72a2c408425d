# Comm test twice (one-shot checks conditional on the shared device co-scheduling the ranks),
# then the fp32 kernel with bank-conflict-free DY2 / conv2-weight pitches: tests, stamps, benches.
T=${1:-r3i}
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out && \
for i in 1 2; do
  timeout -k 10 200 python -u -m pytest tests/test_comm_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/${T}_comm$i.log 2>&1
  rc=$?; echo "comm run $i rc=$rc"; [ $rc -le 1 ] || exit $rc
done
bash tools/gpu_f32.sh ${T}
