# rocprofv3 PMC passes over the sample-tile kernel (B = 1024 per step, 100 steps), one pass each.
T=${1:-pmct}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/${T}1 -o run -- python3 $R/tools/kernel_counters.py 1024 100 > $R/gpurun_out/${T}1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/${T}2 -o run -- python3 $R/tools/kernel_counters.py 1024 100 > $R/gpurun_out/${T}2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM --output-format csv -d $R/gpurun_out/${T}3 -o run -- python3 $R/tools/kernel_counters.py 1024 100 > $R/gpurun_out/${T}3.log 2>&1 && \
cd $R && python3 tools/kernel_counters.py --summarize gpurun_out/${T}1/run_counter_collection.csv gpurun_out/${T}2/run_counter_collection.csv gpurun_out/${T}3/run_counter_collection.csv > gpurun_out/${T}_summary.log 2>&1
echo rc=$?
