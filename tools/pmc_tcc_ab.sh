# L2 (TCC) hit / miss counters of the fused step under ab/A_C.so vs ab/B_C.so (tools/ab_build.sh),
# one rocprofv3 --pmc pass each over tools/kernel_counters.py (200 eager steps at B = 64).
#   gpurun -- bash tools/pmc_tcc_ab.sh ; then python tools/kernel_counters.py --summarize gpurun_out/tcc{A,B}/run_counter_collection.csv
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && \
export CSED_NATIVE_SO=$R/ab/A_C.so && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/tccA -o run -- python3 $R/tools/kernel_counters.py 64 200 > $R/gpurun_out/tccA.log 2>&1 && \
export CSED_NATIVE_SO=$R/ab/B_C.so && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/tccB -o run -- python3 $R/tools/kernel_counters.py 64 200 > $R/gpurun_out/tccB.log 2>&1
echo rc=$?
